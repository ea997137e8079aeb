"""BASELINE config 3 on bench.py's WHOLE grid (t_final 1 ms, 101 outputs -- the head-to-head grid
of the headline figure), against traces of the reference's own Hamiltonian
(tests/golden/make_golden_n14.py --bench -> hpsi_traces_n14_bench.npz: 3 variants x delta in
{0, 75, 150 kHz}, a numpy Chebyshev propagation of the reference-built CSR matrix per output
interval, cross-checked by a second spectral enclosure to <= 1.5e-12 and by expm_multiply).

Every N = 14 kernel path that the bench or a strong shard can take is held to 1e-10 (north_star
1e-8) at all 101 outputs:
  * k_interval<13> (the 192-register bench step), one and two output times per launch;
  * k_span with 2^11- and 2^10-amplitude tiles (a lone register, a strong shard) and with s = 3;
  * k_real (option real = 1) and the mixed real = 2;
  * the engine's own default choice for these 9 registers.
"""
import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params

pytestmark = pytest.mark.gpu
OBS = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")
DELTAS = (0, 75000, 150000)
TOL = 1e-10

PATHS = {
    "k_interval_m2": {"span_tile": 0, "real": 0, "outputs_per_launch": 2},
    "k_interval_m1": {"span_tile": 0, "real": 0, "outputs_per_launch": 1},
    "k_span_t11": {"span_tile": 11},
    "k_span_t10": {"span_tile": 10},
    "k_span_s3": {"span_tile": 0, "span": 3},
    "k_real": {"span_tile": 0, "real": 1},
    "k_real_mixed": {"span_tile": 0, "real": 2},
    "default": {},
}
DEFAULTS = {"span_tile": -1, "real": 0, "outputs_per_launch": 2, "span": 0}


@pytest.mark.parametrize("path", list(PATHS))
def test_bench_grid_matches_reference_n14(engine, golden, path):
    g = golden("hpsi_traces_n14_bench.npz")
    t = g["t"]
    assert len(t) == 101 and t[-1] == 1e-3
    keys, probs = [], []
    for v in VARIANTS:
        for d in DELTAS:
            keys.append(f"{v}_{d}")
            probs.append(pb.build_problem(sweep_point_params(13, float(d), v, 1e-3, 101)))
    engine.clear()
    for k, val in PATHS[path].items():
        engine.set_option(k, val)
    try:
        for p in probs:
            engine.add(p)
        obs, st = engine.evolve(t)
    finally:
        for k, val in DEFAULTS.items():
            engine.set_option(k, val)
        engine.clear()
    assert st["dense_problems"] == 0 and st["handoff_fallbacks"] == 0
    if path.startswith("k_span"):
        assert st["span_problems"] == 9
    if path == "k_real":
        assert st["real_problems"] == 9
    if path.startswith("k_interval"):
        assert st["mode"] == 1 and st["span_problems"] == 0 and st["real_problems"] == 0
    worst = 0.0
    for i, key in enumerate(keys):
        for j, k in enumerate(OBS):
            err = float(np.max(np.abs(obs[i, j] - g[f"{key}_{k}"])))
            worst = max(worst, err)
            assert err < TOL, (path, key, k, err)
        np.testing.assert_allclose(obs[i, 6], g[f"{key}_state_norm"], rtol=0, atol=1e-12)
    print(f"config 3, 1 ms / 101 outputs, {path}: max |GPU - reference-H oracle| = {worst:.2e} "
          f"(mode {st['mode']}, span {st['span_problems']}, real {st['real_problems']})")
