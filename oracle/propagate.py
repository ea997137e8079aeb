"""Exact and ODE propagators for the oracle / CPU baseline (TEST INFRASTRUCTURE).

* ``eigh_trace``      exact: dense Hermitian eigendecomposition, psi(t) = V e^{-i L t} V^H psi0.
                      The primary parity oracle for N <= 12 (dimension <= 4096).
* ``expm_trace``      exact to double precision: scipy ``expm_multiply`` (truncated Taylor
                      with its own error control) on a uniform grid; used above N = 12.
* ``zvode_trace``     the reference's integrator: QuTiP 5 ``sesolve`` drives scipy's ZVODE
                      in Adams mode with a CSR right-hand side -1j H psi, then (default
                      ``normalize_output=True``) normalises each output state before the
                      expectation values.  QuTiP itself is not installed here (not vendored
                      by the reference, version unpinned: README.md:71; >= 5 by the dict
                      options at dipolar_ensemble_with_rare.py:639-651), so this restates that
                      published algorithm; it is the ``cpu_baseline`` "port" that bench.py times.

Expectation values are Re<psi|O|psi> as in dipolar_ensemble_with_rare.py:671-679.
"""
from __future__ import annotations

import time
from typing import Dict, Sequence, Tuple

import numpy as np
import scipy.linalg as la
import scipy.sparse as sp
from scipy.integrate import ode
from scipy.sparse.linalg import expm_multiply

from .reference_model import OBS_ORDER


def _expect(states: np.ndarray, obs: Dict[str, sp.spmatrix], normalize: bool) -> Dict[str, np.ndarray]:
    """states: (n_t, dim).  Returns the six expectations and ||psi||."""
    norms = np.linalg.norm(states, axis=1)
    use = states / norms[:, None] if normalize else states
    out = {}
    for name in OBS_ORDER:
        ops = obs[name]
        out[name] = np.real(np.einsum("td,td->t", np.conj(use), (ops @ use.T).T))
    out["state_norm"] = norms
    return out


def eigh_trace(H, psi0: np.ndarray, t: np.ndarray, obs: Dict[str, sp.spmatrix]) -> Dict[str, np.ndarray]:
    Hd = H.toarray() if sp.issparse(H) else np.asarray(H)
    w, V = la.eigh(Hd)
    c0 = V.conj().T @ psi0
    states = (V @ (np.exp(-1j * np.outer(w, t)) * c0[:, None])).T
    return _expect(states, obs, normalize=False)


def expm_trace(H, psi0: np.ndarray, t: np.ndarray, obs: Dict[str, sp.spmatrix]) -> Dict[str, np.ndarray]:
    t = np.asarray(t, dtype=float)
    A = (-1j) * sp.csr_matrix(H)
    states = expm_multiply(A, psi0, start=t[0], stop=t[-1], num=len(t), endpoint=True)
    return _expect(np.asarray(states), obs, normalize=False)


def zvode_trace(H, psi0: np.ndarray, t: np.ndarray, obs: Dict[str, sp.spmatrix],
                atol: float = 1e-8, rtol: float = 1e-6, nsteps: int = 2500,
                max_step: float = 0.0, order: int = 12, normalize: bool = True,
                time_budget_s: float | None = None) -> Tuple[Dict[str, np.ndarray], Dict[str, float]]:
    """QuTiP-5-sesolve-equivalent trace.  Defaults are QuTiP 5's; the sweep overrides them
    (sweep_sea_detuning.py:1247-1250 -> dipolar_ensemble_with_rare.py:644-651).

    Returns (trace, info) where info has the RHS count and wall time.  With
    ``time_budget_s`` the integration stops at the first output time after the
    budget is spent (info["t_reached"]), which is how bench.py bounds its sample.
    """
    Hc = sp.csr_matrix(H, dtype=complex)
    mHi = (-1j) * Hc
    n_rhs = [0]

    def rhs(_t, y):
        n_rhs[0] += 1
        return mHi @ y

    r = ode(rhs)
    r.set_integrator("zvode", method="adams", atol=atol, rtol=rtol, nsteps=nsteps,
                     max_step=max_step, order=order)
    r.set_initial_value(np.asarray(psi0, dtype=complex), t[0])
    states = [np.asarray(psi0, dtype=complex)]
    t0 = time.perf_counter()
    reached = 1
    for tk in t[1:]:
        r.integrate(tk)
        if not r.successful():
            raise RuntimeError(f"ZVODE failed at t={tk}")
        states.append(r.y.copy())
        reached += 1
        if time_budget_s is not None and time.perf_counter() - t0 > time_budget_s:
            break
    wall = time.perf_counter() - t0
    tr = _expect(np.array(states), obs, normalize=normalize)
    return tr, {"rhs": float(n_rhs[0]), "wall_s": wall, "t_reached": float(t[reached - 1]),
                "outputs": reached}


def trace_max_abs_diff(a: Dict[str, np.ndarray], b: Dict[str, np.ndarray],
                       names: Sequence[str] = OBS_ORDER) -> float:
    return max(float(np.max(np.abs(np.asarray(a[k]) - np.asarray(b[k])))) for k in names)
