"""BASELINE config 3 (N = 14 sweep points) on the production path, against fixtures generated from
the reference's own Hamiltonian (tests/golden/make_golden_n14.py, hpsi_traces_n14.npz).

* H|v>: the reference-built CSR product at N = 14 for center_off / center_on / shell_off and
  delta in {0, 75, 150 kHz} (rel 1e-13 of max|Hv|), and <v|O|v> (abs 1e-13).
* <O>(t): the engine's DEFAULT configuration for a sweep -- every (variant, delta) in one context,
  engine bit order, the exact center_off reduction -- runs the persistent interval kernel
  k_interval<13, IMAG=true> (mode 1): center_off as 1-tile registers (13 qubits), center_on as
  2-tile registers whose crossing term is only the rare drive (raw w hand-off), shell_off as
  2-tile registers with 13 crossing pairs (generated hand-off).  Traces over 20 outputs (200 us)
  are held to the reference-H oracle at 1e-10 (north-star target 1e-8), for one and for two
  output times per launch.
"""
import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params

pytestmark = pytest.mark.gpu
OBS = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")
DELTAS = (0, 75000, 150000)


def _ref_state(dim, seed):
    """make_golden.rand_state: the fixture's random vector, regenerated from its seed."""
    rng = np.random.default_rng(seed)
    v = rng.standard_normal(dim) + 1j * rng.standard_normal(dim)
    return v / np.linalg.norm(v)


def _params(variant, delta, t):
    return sweep_point_params(13, float(delta), variant, float(t[-1]), len(t))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("delta", DELTAS)
def test_apply_h_and_observables_match_reference_n14(engine, golden, variant, delta):
    g = golden("hpsi_traces_n14.npz")
    key = f"{variant}_{delta}"
    prob = pb.build_problem(_params(variant, delta, g["t"]), order="reference", reduce=False)
    assert prob.n_qubits == 14 and prob.psi0_index == int(g[f"{key}_psi0_index"])
    v = _ref_state(1 << 14, 1400)
    engine.clear()
    pid = engine.add(prob)
    out = engine.apply_h(pid, v)
    ref = g[f"{key}_Hv"]
    assert np.max(np.abs(out - ref)) <= 1e-13 * np.max(np.abs(ref))
    o = engine.observables(pid, v)
    for j, k in enumerate(OBS):
        assert abs(o[j] - float(g[f"{key}_expect_{k}"])) < 1e-13, k
    engine.clear()


@pytest.mark.parametrize("real", [1, 0])
@pytest.mark.parametrize("m", [2, 1])
def test_production_interval_kernel_matches_reference_n14(engine, golden, m, real):
    g = golden("hpsi_traces_n14.npz")
    t = g["t"]
    keys, probs = [], []
    for variant in VARIANTS:
        for delta in DELTAS:
            keys.append(f"{variant}_{delta}")
            probs.append(pb.build_problem(_params(variant, delta, t)))   # production defaults
    # the register shapes this test is meant to cover
    assert [p.n_qubits for p in probs] == [13] * 3 + [14] * 6
    assert all(p.rare_bit == 13 for p in probs[3:6]) and all(p.rare_bit == 13 for p in probs[6:])
    assert all(np.all(p.pair[:13, 13] == 0.0) for p in probs[3:6])     # center_on: only the drive crosses
    assert all(np.count_nonzero(p.pair[:13, 13]) == 13 for p in probs[6:])  # shell_off: 13 pairs cross
    engine.clear()
    engine.set_option("outputs_per_launch", m)
    engine.set_option("real", real)   # 1: k_real, two real recurrences; 0 (default): k_interval
    engine.set_option("span_tile", 0)  # whole registers (no automatic span)
    try:
        for p in probs:
            engine.add(p)
        obs, st = engine.evolve(t)
    finally:
        engine.set_option("outputs_per_launch", 2)
        engine.set_option("real", 0)
        engine.set_option("span_tile", -1)
        engine.clear()
    assert st["mode"] == 1 and st["tile_bits"] == 13 and st["outputs_per_launch"] == m
    assert st["real_problems"] == (9 if real else 0)
    worst = 0.0
    for i, key in enumerate(keys):
        for j, k in enumerate(OBS):
            err = float(np.max(np.abs(obs[i, j] - g[f"{key}_{k}"])))
            worst = max(worst, err)
            assert err < 1e-10, (key, k, err)
        np.testing.assert_allclose(obs[i, 6], g[f"{key}_state_norm"], rtol=0, atol=1e-12)
    print(f"N=14 production path (M={m}): max |GPU - reference-H oracle| = {worst:.2e}")


@pytest.mark.parametrize("m", [2, 1])
def test_production_path_is_repeatable_in_one_context(engine, m):
    """The same evolve of the config-3 points, three times in one context (same allocations, same
    hand-off slots and flags): bitwise identical.  A build whose interval kernel read its
    coefficient rows through scalar loads varied here at the 1e-10 level (tools/diag_repeat.py)."""
    t = np.linspace(0.0, 2e-4, 21)
    engine.clear()
    engine.set_option("outputs_per_launch", m)
    try:
        for variant in VARIANTS:
            for delta in DELTAS:
                engine.add(pb.build_problem(_params(variant, delta, t)))
        runs = [engine.evolve(t)[0] for _ in range(3)]
    finally:
        engine.set_option("outputs_per_launch", 2)
        engine.clear()
    for r in runs[1:]:
        assert np.array_equal(r, runs[0])


def test_reference_grid_intervals_match_fine_stepping_n14(engine):
    """The full-sweep regime of config 3: the reference's own grid (t_final 30 s, 20000 outputs,
    sweep_sea_detuning.py:1223-1224) puts ~1e4 Chebyshev terms into one interval (alpha dt ~ 1e4,
    one output per launch).  Its first two intervals, on the production interval kernel for all
    three variants at delta 0 and 150 kHz, against the same evolutions stepped through 150
    sub-intervals each (10 us, two outputs per launch, ~100 terms per launch): the propagator is
    exact at both degrees, so the observables agree to 1e-10 and the norm stays 1 to 1e-12."""
    t_ref = np.linspace(0.0, 30.0, 20000)[:3]
    t_fine = np.concatenate([np.linspace(t_ref[0], t_ref[1], 151), np.linspace(t_ref[1], t_ref[2], 151)[1:]])
    assert t_fine[150] == t_ref[1] and t_fine[300] == t_ref[2]
    probs = [pb.build_problem(sweep_point_params(13, float(d), v, 30.0, 20000))
             for v in VARIANTS for d in (0.0, 150e3)]
    engine.clear()
    try:
        for p in probs:
            engine.add(p)
        coarse, st_c = engine.evolve(t_ref)
        fine, st_f = engine.evolve(t_fine)
    finally:
        engine.clear()
    assert st_c["mode"] == 1 and st_c["outputs_per_launch"] == 1 and st_c["max_degree"] > 5000
    assert st_f["mode"] == 1 and st_f["max_degree"] < 1000
    worst = float(np.max(np.abs(coarse[:, :6, :] - fine[:, :6, ::150])))
    assert worst < 1e-10, worst
    np.testing.assert_allclose(coarse[:, 6, :], 1.0, rtol=0, atol=1e-12)
    print(f"N=14 reference grid: degree {st_c['max_degree']} vs stepped, max |d<O>| = {worst:.2e}")


def test_mixed_launch_is_bitwise_identical(engine):
    """Option mixed_launch (default 1): the 1- and 2-tile problems of the config-3 points in one
    interval launch (stiffest pairs, then the 1-tile problems, then the remaining pairs) instead of
    one stream each (0).  Only the dispatch order changes, so every problem's results are bitwise
    those of the two-stream schedule, and the run stays on the persistent kernel."""
    t = np.linspace(0.0, 2e-4, 21)
    res = {}
    for mixed in (0, 1, 1):
        engine.clear()
        engine.set_option("mixed_launch", mixed)
        engine.set_option("real", 0)  # k_interval's launch schedule
        engine.set_option("span_tile", 0)  # whole registers (no automatic span)
        try:
            for variant in VARIANTS:
                for delta in DELTAS:
                    engine.add(pb.build_problem(_params(variant, delta, t)))
            obs, st = engine.evolve(t)
        finally:
            engine.set_option("mixed_launch", 1)
            engine.set_option("real", 0)
            engine.set_option("span_tile", -1)
            engine.clear()
        assert st["mode"] == 1
        if mixed in res:
            assert np.array_equal(obs, res[mixed])
        res[mixed] = obs
    assert np.array_equal(res[1], res[0])


@pytest.mark.parametrize("m", [2, 1])
def test_overlapped_observables_are_bitwise_identical(engine, m):
    """Option obs_overlap (default off): the observables of each interval launch run on a second
    stream per lane while the next launch runs, and the multi-output launches alternate between two
    sets of intermediate accumulators.  The arithmetic is unchanged, so the results are bitwise
    those of the in-line schedule, also when repeated in one context and over several flushes."""
    t = np.linspace(0.0, 2e-4, 41)
    res = {}
    for ovl in (1, 0, 1):
        engine.clear()
        engine.set_option("obs_overlap", ovl)
        engine.set_option("outputs_per_launch", m)
        engine.set_option("real", 0)  # k_interval's schedule (obs_overlap has no real-mode form)
        engine.set_option("span_tile", 0)  # whole registers (no automatic span)
        try:
            for variant in VARIANTS:
                for delta in DELTAS:
                    engine.add(pb.build_problem(_params(variant, delta, t)))
            obs, st = engine.evolve(t)
        finally:
            engine.set_option("obs_overlap", 0)
            engine.set_option("outputs_per_launch", 2)
            engine.set_option("real", 0)
            engine.set_option("span_tile", -1)
            engine.clear()
        assert st["mode"] == 1 and st["outputs_per_launch"] == m
        if ovl in res:
            assert np.array_equal(obs, res[ovl])
        res[ovl] = obs
    assert np.array_equal(res[1], res[0])
