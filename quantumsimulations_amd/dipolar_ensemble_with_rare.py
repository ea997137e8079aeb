"""Drop-in replacement for the reference's ``dipolar_ensemble_with_rare`` module.

Same public names and call contracts as TimHarrelson/QuantumSimulations'
``dipolar_ensemble_with_rare.py``; ``sweep_sea_detuning.py`` imports exactly
``DipolarRareParams, get_derived_frequencies, simulate_rare,
shell_positions_with_rare_center, dipolar_couplings_from_positions``
(sweep_sea_detuning.py:103-109), all provided here, with no QuTiP import.

``simulate_rare`` (reference :611-680) keeps its signature and return contract:
``(t, {"Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R", "state_norm"})``,
float64 arrays of length ``steps``, keys in that order.  The evolution runs on
an MI355X through libdse (exact Chebyshev propagation of the time-independent
rotating-frame H); the reference's ZVODE knobs (``solver_*``) do not apply to
an exact propagator and are accepted and ignored.  The truncation tolerance of
the Chebyshev series is ``DSE_TOL`` (default 1e-14).

Functions that return QuTiP objects in the reference return numpy / scipy.sparse
equivalents here (``build_hamiltonian_rare``, ``initial_state_rare``), in the
reference's basis order (site 0 = most significant bit).
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np
import scipy.sparse as sp

from .model import (  # noqa: F401  (re-exported API)
    DipolarRareParams,
    _platonic_vertices,
    dipolar_couplings_from_positions,
    get_derived_frequencies,
    shell_positions_with_rare_center,
)
from .problem import OBS_NAMES, Problem, build_problem, time_grid

__all__ = [
    "DipolarRareParams", "get_derived_frequencies", "shell_positions_with_rare_center",
    "dipolar_couplings_from_positions", "simulate_rare", "simulate_rare_batch",
    "build_hamiltonian_rare", "initial_state_rare", "dims_with_rare",
]

_ENGINES: Dict[int, object] = {}


def _default_device() -> int:
    for key in ("DSE_DEVICE", "LOCAL_RANK"):
        v = os.environ.get(key)
        if v is not None and v.strip() != "":
            return int(v)
    return 0


def _engine(device: int):
    from .engine import Engine  # loads libdse.so; raises if it is missing
    eng = _ENGINES.get(device)
    if eng is None:
        eng = Engine(device)
        _ENGINES[device] = eng
    return eng


def _tol() -> float:
    return float(os.environ.get("DSE_TOL", "1e-14"))


def dims_with_rare(n_sea: int, is_spin_three_half: bool = False) -> List[int]:
    """Local dimensions, dipolar_ensemble_with_rare.py:28-34."""
    return [2] * n_sea + ([4] if is_spin_three_half else [2])


def simulate_rare_batch(params_list: Sequence[DipolarRareParams], device: int | None = None
                        ) -> List[Tuple[np.ndarray, Dict[str, np.ndarray]]]:
    """Many evolutions at once on one device (same results as calling simulate_rare on each)."""
    device = _default_device() if device is None else device
    grids = [time_grid(p) for p in params_list]       # raises ValueError like :620-621
    probs = [build_problem(p, order="engine", reduce=True) for p in params_list]
    eng = _engine(device)
    results: List = [None] * len(params_list)
    # one engine call per distinct time grid and engine class (engine.evolve_groups)
    from .engine import batches_for_memory, evolve_groups
    by_grid = evolve_groups([(float(p.t_final), int(p.steps)) for p in params_list], probs)
    for key, idxs in by_grid.items():
        eng.clear()  # free the previous group's buffers before sizing this group's batches
        for batch in batches_for_memory([probs[i] for i in idxs], device):
            members = [idxs[b] for b in batch]
            eng.clear()
            for i in members:
                eng.add(probs[i])
            t = grids[members[0]]
            obs, _ = eng.evolve(t, tol=_tol())
            for slot, i in enumerate(members):
                results[i] = (t.copy(), {name: obs[slot, j].copy() for j, name in enumerate(OBS_NAMES)})
    eng.clear()
    return results


def simulate_rare(params: DipolarRareParams) -> Tuple[np.ndarray, Dict[str, np.ndarray]]:
    """Time grid and the six expectation traces + state norm (reference :611-680).

    ``state_norm`` always has length ``steps`` here (||psi(t)|| of the exactly propagated state).
    The reference computes it from ``res.states`` (:669); when no ``solver_*`` override is set it
    passes ``options=None`` and QuTiP 5, by its ``store_states`` default with ``e_ops`` given,
    likely stores no states, so its ``state_norm`` would be empty.  That default cannot be
    checked offline (QuTiP is absent: parity unpinned); the sweep always sets the overrides
    (sweep_sea_detuning.py:1247-1250), where both return one norm per output time."""
    return simulate_rare_batch([params])[0]


def problem_to_csr(prob: Problem) -> sp.csr_matrix:
    """Dense-free CSR of the H described by ``prob`` (host helper; small registers only)."""
    n = prob.n_qubits
    if n > 20:
        raise ValueError("CSR construction is limited to 20 qubits")
    dim = 1 << n
    x = np.arange(dim, dtype=np.int64)
    s = [0.5 - ((x >> b) & 1) for b in range(n)]
    diag = np.full(dim, prob.shift)
    for b in range(n):
        diag = diag + prob.field[b] * s[b]
    for i in range(n):
        for j in range(i + 1, n):
            if prob.zz[i, j] != 0.0:
                diag = diag + prob.zz[i, j] * (s[i] * s[j])
    rows, cols, vals = [x], [x], [diag.astype(complex)]
    for b in range(n):
        f = prob.flip[b]
        if np.any(f != 0.0):
            bit = (x >> b) & 1
            rows.append(x)
            cols.append(x ^ (1 << b))
            vals.append(np.where(bit == 0, f[0] + 1j * f[1], f[2] + 1j * f[3]))
    for i in range(n):
        for j in range(i + 1, n):
            g = prob.pair[i, j]
            if g != 0.0:
                eq = ((x >> i) & 1) == ((x >> j) & 1)
                rows.append(x[eq])
                cols.append(x[eq] ^ ((1 << i) | (1 << j)))
                vals.append(np.full(int(eq.sum()), g, dtype=complex))
    m = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(dim, dim))
    m.sum_duplicates()
    return m


def build_hamiltonian_rare(params: DipolarRareParams) -> Tuple[sp.csr_matrix, Dict[str, sp.csr_matrix]]:
    """H and the six observables as scipy.sparse matrices in the reference's basis order
    (site 0 = most significant bit), as the QuTiP objects of :453-588 would be."""
    prob = build_problem(params, order="reference", reduce=False)
    H = problem_to_csr(prob)
    n = prob.n_qubits
    dim = 1 << n
    x = np.arange(dim, dtype=np.int64)

    def z_of(bits):
        d = np.zeros(dim)
        for b in bits:
            d += 0.5 - ((x >> b) & 1)
        return sp.diags(d.astype(complex), format="csr")

    def xy_of(bits, comp):
        m = sp.csr_matrix((dim, dim), dtype=complex)
        for b in bits:
            bit = (x >> b) & 1
            if comp == "x":
                v = np.full(dim, 0.5, dtype=complex)
            else:  # <x^e_b| Iy |x>: +i/2 when the output bit is 1 (input bit 0), -i/2 otherwise
                v = np.where(bit == 0, 0.5j, -0.5j)
            m = m + sp.csr_matrix((v, (x ^ (1 << b), x)), shape=(dim, dim))
        return m

    sea_bits = [b for b in range(n) if (prob.sea_mask >> b) & 1]
    rare = [prob.rare_bit]
    obs = {"Ix_sea": xy_of(sea_bits, "x"), "Iy_sea": xy_of(sea_bits, "y"), "Iz_sea": z_of(sea_bits),
           "Iz_R": z_of(rare), "Ix_R": xy_of(rare, "x"), "Iy_R": xy_of(rare, "y")}
    return H, obs


def initial_state_rare(params: DipolarRareParams) -> np.ndarray:
    """Product initial state as a dense ket in the reference's basis order (:591-606)."""
    prob = build_problem(params, order="reference", reduce=False)
    v = np.zeros(1 << prob.n_qubits, dtype=complex)
    v[prob.psi0_index] = 1.0
    return v
