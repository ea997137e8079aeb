"""The dense engine's output times by a type-1 non-uniform FFT (csrc/dse_nufft.hip, option
dense_nufft): psi'(tau_j) = V (c o e^{-i lambda tau_j}) on a uniform grid from W = 15-point
spreading of the eigenvalue phases, rocFFT and deconvolution, plus the first-order correction of
np.linspace's ulp-sized departures delta_j from j s -- instead of the 4 dim^2 T-flop GEMM.

* N = 7 on the reference's 30 s / 20 000-output grid (dense_nufft = 2 forces the transform below
  2^10 amplitudes) against the 40-digit fixture (tests/golden/grid30_n7.npz, both Hamiltonians) at
  the early-time floor and north_star's 1e-8, and against the GEMM path;
* N = 12 and 13 registers (the transform's default range) on a 1 s / 4001-output grid against the
  GEMM path: every output and the final state (dse_get_state);
* a grid that is not uniform keeps the GEMM (stats dense_nufft_problems = 0), and so does
  dense_nufft = 0.
The N = 14 30 s oracle test (test_gpu_grid30_n14.py) runs the default, i.e. the transform."""
import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params

pytestmark = pytest.mark.gpu
OBS = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")


def _run(engine, probs, t, **opts):
    engine.clear()
    for k, v in opts.items():
        engine.set_option(k, v)
    try:
        for p in probs:
            engine.add(p)
        obs, st = engine.evolve(t)
        states = [engine.state(i) for i in range(len(probs))]
        return obs, st, states
    finally:
        engine.set_option("dense", 1)
        engine.set_option("dense_nufft", 1)
        engine.clear()


def test_nufft_outputs_n7_30s_grid_match_40_digit_fixture_and_gemm(engine, golden):
    g = golden("grid30_n7.npz")
    idx, t = g["t_index"], g["t"]
    T = np.linspace(0.0, 30.0, 20000)
    deltas = (0, 25000, 150000)
    probs = [pb.build_problem(sweep_point_params(6, float(d), v, 30.0, 20000), reduce=False)
             for v in VARIANTS for d in deltas]
    nu, st, s_nu = _run(engine, probs, T, dense=2, dense_nufft=2)
    gm, st0, s_gm = _run(engine, probs, T, dense=2, dense_nufft=0)
    assert st["dense_nufft_problems"] == 9 and st0["dense_nufft_problems"] == 0
    hnorm = max(float(np.max(np.abs(g[f"{v}_{d}_lambda"]))) for v in VARIANTS for d in deltas)
    bound = np.minimum(1e-8, 1e-10 + 1.5 * np.finfo(float).eps * hnorm * t)
    e = np.zeros(len(idx))
    for i, (v, d) in enumerate([(v, d) for v in VARIANTS for d in deltas]):
        for j, k in enumerate(OBS):
            e = np.maximum(e, np.abs(nu[i, j, idx] - g[f"tables_{v}_{d}_{k}"]))
    dg = float(np.max(np.abs(nu - gm)))
    print(f"N=7 30 s grid, non-uniform FFT outputs: vs 40-digit tables fixture {e.max():.2e} (30 s: {e[-1]:.2e}); "
          f"vs GEMM outputs {dg:.2e}; output stage {st['dense_output_ms']:.1f} vs {st0['dense_output_ms']:.1f} ms")
    np.testing.assert_allclose(nu[:, 6], 1.0, rtol=0, atol=1e-12)
    assert np.all(e <= bound), (e, bound)
    assert dg < 1e-11
    for a, b in zip(s_nu, s_gm):
        assert np.max(np.abs(a - b)) < 1e-11


@pytest.mark.parametrize("n_sea", [11, 12])
def test_nufft_outputs_match_gemm_n12_n13(engine, n_sea):
    t = np.linspace(0.0, 1.0, 4001)
    probs = [pb.build_problem(sweep_point_params(n_sea, d, v, 1.0, 4001)) for v in ("center_on", "shell_off")
             for d in (40e3, 150e3)]
    nu, st, s_nu = _run(engine, probs, t, dense=2)
    gm, st0, s_gm = _run(engine, probs, t, dense=2, dense_nufft=0)
    assert st["dense_nufft_problems"] == len(probs) and st0["dense_nufft_problems"] == 0
    d = float(np.max(np.abs(nu - gm)))
    ds = max(float(np.max(np.abs(a - b))) for a, b in zip(s_nu, s_gm))
    print(f"n_sea={n_sea}: non-uniform FFT vs GEMM outputs {d:.2e}, final states {ds:.2e}; output stage "
          f"{st['dense_output_ms']:.1f} vs {st0['dense_output_ms']:.1f} ms")
    np.testing.assert_allclose(nu[:, 6], 1.0, rtol=0, atol=1e-12)
    assert d < 1e-11 and ds < 1e-11


def test_non_uniform_grid_keeps_the_gemm(engine):
    t = np.linspace(0.0, 1.0, 4001)
    t[1000:] += 1e-7          # one jump: not j s + an ulp
    probs = [pb.build_problem(sweep_point_params(11, 75e3, "center_on", 1.0, 4001))]
    a, st, _ = _run(engine, probs, t, dense=2)
    b, st0, _ = _run(engine, probs, t, dense=2, dense_nufft=0)
    assert st["dense_nufft_problems"] == 0
    assert np.array_equal(a, b)
    with pytest.raises(ValueError):
        engine.set_option("dense_nufft", 3)
