"""Generate the N = 14 golden fixtures (BASELINE config 3 workload) from the reference's own code.

Run ONLY in the build container (it reads /root/reference, which the GPU box does not have):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_n14.py            (200 us grid)
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_n14.py --bench    (bench grid, ~15 min)

Same route as make_golden.py: the reference's ``dipolar_ensemble_with_rare.py`` is imported by
path with the QuTiP stand-in (``_qutip_standin``, scipy.sparse-backed) first on sys.path, so H,
psi0 and the six observables are the reference's own ``build_hamiltonian_rare`` /
``initial_state_rare`` output at n_sea = 13 (14 qubits; shell_off: 14 sea sites).  Sweep-point
parameters follow sweep_sea_detuning.py:414-668 with the __main__ constants of :1201-1251
(make_golden.sweep_params).

Fixture written: hpsi_traces_n14.npz, for variant in (center_off, center_on, shell_off) and
delta in (0, 75, 150 kHz):
  <v>_<d>_Hv          H @ v for v = the seeded random state rand_state(2^14, 1400) (reference
                      basis order, site 0 = most significant bit)
  <v>_<d>_expect_<O>  <v|O|v> for the six observables
  <v>_<d>_psi0_index  argmax |psi0>
  <v>_<d>_<O>         <O>(t) of the exact evolution of the reference H from psi0 on
                      t = linspace(0, 2e-4, 21) (20 output intervals of 10 us), and state_norm
  t                   that grid
The traces come from a Chebyshev propagation of the reference's CSR matrix in numpy (spectrum
enclosed by Gershgorin discs, scipy Bessel J_k, series run ~20 (alpha dt)^(1/3) terms past the
argument).  The generator repeats it with a different enclosure (the extreme eigenvalues from
scipy eigsh, +-1e-6 relative margin: a different alpha changes every coefficient and vector of
the series) and stores the largest difference as <v>_<d>_cross_check (2e-13 to 1.2e-12; asserted
< 5e-12); it also stores the distance to scipy's expm_multiply stepped per output interval as
<v>_<d>_expm_diff.  expm_multiply over the whole grid in one call is NOT used: at alpha t ~ 1e3 it
drifts to 1e-11 here, with a norm error of 1e-12, while both Chebyshev runs keep the norm to
1e-14.

With --bench: hpsi_traces_n14_bench.npz, the same traces (no H @ v) on bench.py's whole config-3
grid, t = linspace(0, 1e-3, 101) (1 ms, 101 outputs), for the same 9 (variant, delta) cases; the
cases run in parallel worker processes.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import expm_multiply
from scipy.special import jv

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (loads the reference through the stand-in)

ref = mg.ref
VARIANTS = mg.VARIANTS
OBS = mg.OBS
DELTAS = (0.0, 75000.0, 150000.0)
T = np.linspace(0.0, 2e-4, 21)
T_BENCH = np.linspace(0.0, 1e-3, 101)   # bench.py's config-3 grid (1 ms, 101 outputs)


def gershgorin(Hc: sp.csr_matrix):
    d = Hc.diagonal().real
    r = np.asarray(abs(Hc).sum(axis=1)).ravel() - np.abs(d)
    return float(np.min(d - r)), float(np.max(d + r))


def eig_bounds(Hc: sp.csr_matrix):
    from scipy.sparse.linalg import eigsh
    hi = float(eigsh(Hc, k=1, which="LA", return_eigenvectors=False)[0].real)
    lo = float(eigsh(Hc, k=1, which="SA", return_eigenvectors=False)[0].real)
    m = 1e-6 * (hi - lo)
    return lo - m, hi + m


def chebyshev_trace(Hc: sp.csr_matrix, psi0: np.ndarray, t: np.ndarray, bounds) -> np.ndarray:
    """exp(-iH dt) = e^{-i beta dt} sum_k (2 - d_k0) (-i)^k J_k(alpha dt) T_k((H - beta)/alpha)
    with the spectrum inside bounds = (lo, hi)."""
    lo, hi = bounds
    alpha, beta = 0.5 * (hi - lo), 0.5 * (hi + lo)
    Hs = (Hc - beta * sp.identity(Hc.shape[0], format="csr")) / alpha
    states = [psi0.astype(complex)]
    psi = psi0.astype(complex)
    for m in range(1, len(t)):
        z = alpha * (t[m] - t[m - 1])
        K = int(z + 20 * np.cbrt(z + 1) + 40)
        J = jv(np.arange(K + 1), z)
        w0, w1 = psi, Hs @ psi
        acc = J[0] * w0 + 2 * (-1j) * J[1] * w1
        for k in range(2, K + 1):
            w0, w1 = w1, 2 * (Hs @ w1) - w0
            acc = acc + 2 * (-1j) ** k * J[k] * w1
        psi = np.exp(-1j * beta * (t[m] - t[m - 1])) * acc
        states.append(psi)
    return np.array(states)


def expect(states: np.ndarray, op) -> np.ndarray:
    return np.real(np.einsum("td,td->t", states.conj(), (op @ states.T).T))


def one_case(v: str, dlt: float, t: np.ndarray, with_hv: bool):
    p = mg.sweep_params(13, dlt, v, float(t[-1]), len(t))
    H, eops = ref.build_hamiltonian_rare(p)
    Hc = H.data.tocsr()
    psi0 = ref.initial_state_rare(p).full().ravel()
    key = f"{v}_{int(dlt)}"
    out = {}
    if with_hv:
        vec = mg.rand_state(Hc.shape[0], 1400)
        out[f"{key}_Hv"] = Hc @ vec
        for k in OBS:
            out[f"{key}_expect_{k}"] = float(np.real(np.vdot(vec, eops[k].data @ vec)))
    out[f"{key}_psi0_index"] = int(np.argmax(np.abs(psi0)))
    st = chebyshev_trace(Hc, psi0, t, gershgorin(Hc))
    ch = chebyshev_trace(Hc, psi0, t, eig_bounds(Hc))
    ex = [psi0.astype(complex)]
    for m in range(1, len(t)):
        ex.append(expm_multiply(-1j * (t[m] - t[m - 1]) * Hc, ex[-1]))
    ex = np.array(ex)
    cross = dexp = 0.0
    for k in OBS:
        a = expect(st, eops[k].data)
        cross = max(cross, float(np.max(np.abs(a - expect(ch, eops[k].data)))))
        dexp = max(dexp, float(np.max(np.abs(a - expect(ex, eops[k].data)))))
        out[f"{key}_{k}"] = a
    out[f"{key}_state_norm"] = np.linalg.norm(st, axis=1)
    out[f"{key}_cross_check"] = cross
    out[f"{key}_expm_diff"] = dexp
    print(f"{key}: dim {Hc.shape[0]}, nnz {Hc.nnz}, Chebyshev(Gershgorin) vs "
          f"Chebyshev(eigsh) {cross:.2e}, vs expm_multiply per interval {dexp:.2e}", flush=True)
    assert cross < 5e-12, cross
    return out


def _case(args):
    return one_case(*args)


def main():
    t0 = time.time()
    bench = "--bench" in sys.argv
    t = T_BENCH if bench else T
    out = {"t": t}
    cases = [(v, dlt, t, not bench) for v in VARIANTS for dlt in DELTAS]
    if bench:
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(max_workers=min(len(cases), os.cpu_count() or 1)) as ex:
            for o in ex.map(_case, cases):
                out.update(o)
    else:
        for c in cases:
            out.update(one_case(*c))
    name = "hpsi_traces_n14_bench.npz" if bench else "hpsi_traces_n14.npz"
    np.savez(os.path.join(HERE, name), **out)
    print(f"done in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
