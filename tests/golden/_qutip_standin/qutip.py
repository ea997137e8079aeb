"""Minimal stand-in for the slice of the QuTiP API that dipolar_ensemble_with_rare.py uses.

GOLDEN-VECTOR TOOLING ONLY (used by tests/golden/make_golden.py in the build
container, never shipped, never imported by the package or by the tests).

QuTiP is not installed and cannot be installed offline.  The reference module
calls only: sigmax/sigmay/sigmaz/qeye/jmat/basis/tensor, Qobj arithmetic
(+, -, scalar *, operator @ via *), unit/norm/eigenstates/full, and sesolve.
This file implements exactly those on scipy.sparse matrices with QuTiP's
conventions (tensor = Kronecker product, first factor most significant;
basis(2, 0) = spin up; jmat ordered m = +j ... -j).  ``sesolve`` restates QuTiP 5's
default integrator (scipy ZVODE, Adams, normalize_output=True); it is the
"reference-behaviour" integrator for the traces, clearly labelled as such.
"""
from __future__ import annotations

import numbers

import numpy as np
import scipy.linalg as _la
import scipy.sparse as _sp
from scipy.integrate import ode as _ode


class Qobj:
    # make numpy scalars (np.float64 * Qobj) defer to our __rmul__
    __array_ufunc__ = None
    __array_priority__ = 100

    def __init__(self, data=None, dims=None):
        if isinstance(data, Qobj):
            dims = data.dims if dims is None else dims
            data = data.data
        if isinstance(data, numbers.Number):
            raise TypeError("Qobj from a bare number is not supported by this stand-in")
        m = _sp.csr_matrix(data, dtype=complex)
        self.data = m
        if dims is None:
            dims = [[m.shape[0]], [m.shape[1]]]
        self.dims = dims

    @property
    def shape(self):
        return self.data.shape

    def _check(self, other):
        if self.dims != other.dims:
            raise TypeError(f"Incompatible Qobj dimensions: {self.dims} vs {other.dims}")

    def __add__(self, other):
        if isinstance(other, numbers.Number) and other == 0:
            return Qobj(self.data, self.dims)
        self._check(other)
        return Qobj(self.data + other.data, self.dims)

    __radd__ = __add__

    def __sub__(self, other):
        self._check(other)
        return Qobj(self.data - other.data, self.dims)

    def __neg__(self):
        return Qobj(-self.data, self.dims)

    def __mul__(self, other):
        if isinstance(other, numbers.Number):
            return Qobj(self.data * other, self.dims)
        if self.dims[1] != other.dims[0]:
            raise TypeError(f"Incompatible Qobj dimensions for product: {self.dims} x {other.dims}")
        return Qobj(self.data @ other.data, [self.dims[0], other.dims[1]])

    def __rmul__(self, other):
        if isinstance(other, numbers.Number):
            return Qobj(other * self.data, self.dims)
        return NotImplemented

    __matmul__ = __mul__

    def full(self):
        return self.data.toarray()

    def norm(self):
        return float(np.sqrt(np.real(np.vdot(self.full().ravel(), self.full().ravel()))))

    def unit(self):
        return Qobj(self.data / self.norm(), self.dims)

    def eigenstates(self):
        w, v = _la.eigh(self.full())
        kets = [Qobj(v[:, [k]], [self.dims[0], [1] * len(self.dims[0])]) for k in range(len(w))]
        return w, kets


def sigmax():
    return Qobj(np.array([[0, 1], [1, 0]]))


def sigmay():
    return Qobj(np.array([[0, -1j], [1j, 0]]))


def sigmaz():
    return Qobj(np.array([[1, 0], [0, -1]]))


def qeye(d):
    return Qobj(_sp.identity(d, dtype=complex, format="csr"))


def jmat(j, which):
    m = np.arange(j, -j - 1, -1)
    d = len(m)
    jp = np.zeros((d, d), dtype=complex)
    for k in range(1, d):
        jp[k - 1, k] = np.sqrt(j * (j + 1) - m[k] * (m[k] + 1))
    if which == "x":
        return Qobj(0.5 * (jp + jp.conj().T))
    if which == "y":
        return Qobj(-0.5j * (jp - jp.conj().T))
    if which == "z":
        return Qobj(np.diag(m))
    raise ValueError(which)


def basis(d, i):
    v = np.zeros((d, 1), dtype=complex)
    v[i, 0] = 1.0
    return Qobj(v, [[d], [1]])


def tensor(ops):
    ops = list(ops)
    out = ops[0].data
    dims0, dims1 = list(ops[0].dims[0]), list(ops[0].dims[1])
    for q in ops[1:]:
        out = _sp.kron(out, q.data, format="csr")
        dims0 += q.dims[0]
        dims1 += q.dims[1]
    return Qobj(out, [dims0, dims1])


class _Result:
    pass


# Filled by sesolve so the generator can record the RHS count.
LAST_SOLVE_INFO = {}


def sesolve(H, psi0, tlist, e_ops=None, options=None):
    opts = {"atol": 1e-8, "rtol": 1e-6, "nsteps": 2500, "max_step": 0.0, "order": 12,
            "normalize_output": True, "store_states": None}
    if options:
        opts.update(options)
    mHi = (-1j) * H.data
    count = [0]

    def rhs(_t, y):
        count[0] += 1
        return mHi @ y

    r = _ode(rhs)
    r.set_integrator("zvode", method="adams", atol=opts["atol"], rtol=opts["rtol"],
                     nsteps=opts["nsteps"], max_step=opts["max_step"], order=opts["order"])
    y0 = psi0.full().ravel()
    r.set_initial_value(y0, tlist[0])
    states = [y0]
    for tk in tlist[1:]:
        r.integrate(tk)
        if not r.successful():
            raise RuntimeError("ZVODE failed")
        states.append(r.y.copy())
    states = np.array(states)
    if opts["normalize_output"]:
        states = states / np.linalg.norm(states, axis=1)[:, None]
    res = _Result()
    res.expect = []
    for op in (e_ops or []):
        res.expect.append(np.einsum("td,td->t", states.conj(), (op.data @ states.T).T))
    store = opts["store_states"]
    if store is None:
        store = not e_ops
    res.states = [Qobj(s.reshape(-1, 1), [H.dims[0], [1] * len(H.dims[0])]) for s in states] if store else []
    LAST_SOLVE_INFO.clear()
    LAST_SOLVE_INFO.update({"rhs": count[0]})
    return res
