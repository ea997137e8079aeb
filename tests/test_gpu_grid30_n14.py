"""BASELINE's "(full sweep)" grid at config 3's size, pinned by an independent CPU oracle:
t_final 30 s / 20 000 outputs (sweep_sea_detuning.py:1223-1224), N = 14 (n_sea = 13), the 3 variants
at 150 kHz (the sweep's stiffest point), against tests/golden/grid30_n14.npz
(make_golden_grid30_n14.py: the reference-built H through the QuTiP stand-in, LAPACK dsyevd of its
real rotated form, eigenvalues re-evaluated as double-double Rayleigh quotients with the exact
diagonal, phases reduced modulo 2 pi in 40-digit arithmetic; its pipeline is checked there against
the numpy Chebyshev propagation of the reference CSR at 1e-12, and the same code reproduces the
40-digit N = 7 fixture to 6.5e-13 over the 30 s grid).  Two fixture Hamiltonians per case, as at N = 7:
  "tables"  entries exact in the engine's fp64 coefficient tables (unreduced, reference order);
  "ref"     the reference's own fp64 matrix elements (its rounded diagonal sums).

* The dense engine (the engine the cost model and the bench's full_sweep use for this grid) on the
  unreduced registers, whole grid, against "tables": north_star's 1e-8 at every pinned output
  (1 ... 19999, t = 30 s included).  The bench's own registers (center_off reduced to the 2^13 sea
  block, one more rounding of the folded fields) against "ref": the same 1e-8, which also bounds the
  two fixtures' own difference.
* The Chebyshev kernels over the grid's first 100 intervals (0.15 s), unreduced, against "tables":
  held to 1e-10 + 1.5 eps ||H|| t (their fp64 drift), the rate recorded -- this says which of the two
  engines carries the dense-vs-Chebyshev difference test_gpu_dense.py measures.
"""
import json
import os

import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params

pytestmark = pytest.mark.gpu
OBS = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")
T = np.linspace(0.0, 30.0, 20000)
DELTA = 150000
TOL_NORTH_STAR = 1e-8


def _err_t(g, obs, idx, src):
    """max over variants and observables of |d<O>| at each pinned output"""
    e = np.zeros(len(idx))
    for i, v in enumerate(VARIANTS):
        key = f"{v}_{DELTA}" if src == "ref" else f"tables_{v}_{DELTA}"
        for j, k in enumerate(OBS):
            e = np.maximum(e, np.abs(obs[i, j, idx] - g[f"{key}_{k}"]))
    return e


def _probs(reduce):
    return [pb.build_problem(sweep_point_params(13, float(DELTA), v, 30.0, 20000), reduce=reduce)
            for v in VARIANTS]


def _evolve(engine, probs, t, **opts):
    engine.clear()
    for k, val in opts.items():
        engine.set_option(k, val)
    try:
        for p in probs:
            engine.add(p)
        return engine.evolve(t)
    finally:
        engine.set_option("dense", 1)
        engine.clear()


def _record(name, rec):
    rec_dir = os.environ.get("DSE_TEST_RECORD")
    if rec_dir:   # bench full_sweep.tolerance_at_t_final reads profiles/<round>/grid30_n14_oracle*.json
        with open(os.path.join(rec_dir, name), "w") as f:
            json.dump(rec, f, indent=1)


def test_dense_30s_n14_matches_oracle(engine, golden):
    g = golden("grid30_n14.npz")
    idx = g["t_index"]
    t = g["t"]
    assert np.array_equal(t, T[idx])
    obs, st = _evolve(engine, _probs(False), T, dense=2)
    assert st["dense_problems"] == 3 and st["mode"] == 4
    np.testing.assert_allclose(obs[:, 6, idx], 1.0, rtol=0, atol=1e-12)
    et = _err_t(g, obs, idx, "tables")
    obs_b, st_b = _evolve(engine, _probs(True), T, dense=2)     # the bench's registers
    assert st_b["dense_problems"] == 3
    eb_r = _err_t(g, obs_b, idx, "ref")
    eb_t = _err_t(g, obs_b, idx, "tables")
    fx = float(g["ref_vs_tables"])
    print(f"N=14 30 s grid, dense engine vs oracle: unreduced vs tables-H max {et.max():.2e} (t = 30 s: "
          f"{et[-1]:.2e}); bench registers vs reference-H {eb_r.max():.2e}, vs tables-H {eb_t.max():.2e}; "
          f"the two fixtures differ by {fx:.2e}")
    _record("grid30_n14_oracle_dense.json", {
        "t": t.tolist(), "t_index": idx.tolist(),
        "err_unreduced_vs_tables": et.tolist(), "err_bench_registers_vs_ref": eb_r.tolist(),
        "err_bench_registers_vs_tables": eb_t.tolist(),
        "max_unreduced_vs_tables": float(et.max()), "at_30s_unreduced_vs_tables": float(et[-1]),
        "max_bench_registers_vs_ref": float(eb_r.max()), "max_bench_registers_vs_tables": float(eb_t.max()),
        "fixtures_ref_vs_tables": fx, "eig_fallbacks": st.get("eig_fallbacks")})
    # north_star's 1e-8 and, below it, the early-time floor 1e-10 + 1.5 eps ||H|| t (refined
    # eigenvalues: nothing may grow with t; measured 2.5e-11 over the whole grid)
    hnorm = max(max(abs(a) for a in pb.spectral_bounds(p)) for p in _probs(False))
    bound = np.minimum(TOL_NORTH_STAR, 1e-10 + 1.5 * np.finfo(float).eps * hnorm * t)
    assert np.all(et <= bound), (et, bound)
    assert np.all(eb_r <= TOL_NORTH_STAR), eb_r   # the fixtures' own 4.5e-9 difference included


def test_chebyshev_30s_n14_prefix_against_oracle(engine, golden):
    g = golden("grid30_n14.npz")
    idx = g["t_index"]
    sel = np.nonzero(idx <= 100)[0]
    probs = _probs(False)
    ch, st = _evolve(engine, probs, T[:101], dense=0)
    assert st["dense_problems"] == 0 and st["mode"] == 1
    e = np.zeros(len(sel))
    for i, v in enumerate(VARIANTS):
        for j, k in enumerate(OBS):
            e = np.maximum(e, np.abs(ch[i, j, idx[sel]] - g[f"tables_{v}_{DELTA}_{k}"][sel]))
    tk = T[idx[sel]]
    hnorm = max(max(abs(a) for a in pb.spectral_bounds(p)) for p in probs)
    # drift rate for the extrapolation to 30 s: least squares through the origin, and the envelope
    # past the first 10 ms (earlier outputs carry the per-interval truncation floor, not the drift)
    rate_ls = float(np.sum(e * tk) / np.sum(tk * tk))
    rate = float(np.max((e / tk)[tk >= 0.01]))
    print(f"N=14 Chebyshev vs oracle over the first 100 intervals: {', '.join(f'{x:.1e}' for x in e)} at "
          f"t = {', '.join(f'{x:.3f}' for x in tk)} s; rate LS {rate_ls:.2e}/s, envelope past 10 ms {rate:.2e}/s (eps ||H|| = "
          f"{np.finfo(float).eps * hnorm:.2e}/s)")
    _record("grid30_n14_oracle_chebyshev.json", {
        "t": tk.tolist(), "t_index": idx[sel].tolist(), "err_vs_tables": e.tolist(),
        "rate_envelope_per_s": rate, "rate_ls_per_s": rate_ls, "hnorm_bound": hnorm, "eps_hnorm_per_s": float(np.finfo(float).eps * hnorm)})
    assert np.all(e <= 1e-10 + 1.5 * np.finfo(float).eps * hnorm * tk), e
