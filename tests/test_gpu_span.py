"""Spanning registers (dse_span.hip, option "span"): one register over 2^s workgroups, one per
CU, with per-term cross-tile hand-offs (u operands of the crossing pairs, raw vectors under the
crossing drives and the pairs between two tile-index bits).

* The config-3 points (N = 14: center_off 13 qubits, center_on and shell_off 14) on k_span with
  2^11- and 2^10-amplitude tiles (4 to 16 workgroups per register) against the reference-H oracle traces (tests/golden/hpsi_traces_n14.npz, built
  from the reference's own Hamiltonian) at 1e-10, as the production kernel is held
  (test_gpu_config3.py).  shell_off over >= 4 tiles exercises every operand kind: u of crossing pairs,
  and the raw partner of the pairs between two tile-index bits; center_on the raw partner under
  the rare spin's drive.
* Bitwise repeatability of the spanned evolve in one context.
* A lone register (the reference's call pattern: simulate_rare one evolution at a time,
  sweep_sea_detuning.py:671-673) on k_span against the interval kernel (span_tile = 0).
* The automatic policy (span_tile = -1, the default): a set whose 2^11-amplitude tiles fit the
  chip at once spans; the bench's 192 evolutions do not.
"""
import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params

pytestmark = pytest.mark.gpu
OBS = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")
DELTAS = (0, 75000, 150000)


def _params(variant, delta, t):
    return sweep_point_params(13, float(delta), variant, float(t[-1]), len(t))


def _evolve(engine, probs, t, **opts):
    engine.clear()
    for k, v in opts.items():
        engine.set_option(k, v)
    try:
        for p in probs:
            engine.add(p)
        return engine.evolve(t)
    finally:
        engine.set_option("span", 0)
        engine.set_option("span_tile", -1)
        engine.set_option("outputs_per_launch", 2)
        engine.set_option("span_outputs", 4)
        engine.set_option("matrix", 1)
        engine.clear()


SPANS = [{"span_tile": 11}, {"span_tile": 10}, {"span": 3}]


@pytest.mark.parametrize("opt", SPANS, ids=lambda o: "-".join(f"{k}{v}" for k, v in o.items()))
def test_spanned_registers_match_reference_n14(engine, golden, opt):
    g = golden("hpsi_traces_n14.npz")
    t = g["t"]
    keys, probs = [], []
    for variant in VARIANTS:
        for delta in DELTAS:
            keys.append(f"{variant}_{delta}")
            probs.append(pb.build_problem(_params(variant, delta, t)))
    obs, st = _evolve(engine, probs, t, **opt)
    # every register spans: 14 qubits over 8 / 16, 13 over 4 / 8 workgroups
    assert st["mode"] == 1 and st["span_problems"] == 9, st
    worst = 0.0
    for i, key in enumerate(keys):
        for j, k in enumerate(OBS):
            err = float(np.max(np.abs(obs[i, j] - g[f"{key}_{k}"])))
            worst = max(worst, err)
            assert err < 1e-10, (opt, key, k, err)
        np.testing.assert_allclose(obs[i, 6], g[f"{key}_state_norm"], rtol=0, atol=1e-12)
    print(f"N=14 spanned ({opt}): max |GPU - reference-H oracle| = {worst:.2e}")


@pytest.mark.parametrize("m", [4, 3, 2, 1])
def test_spanned_evolve_is_repeatable(engine, m):
    """Option span_outputs = M outputs per launch (k_span staggers output j's sum to phase j % 3)."""
    t = np.linspace(0.0, 2e-4, 21)
    probs = [pb.build_problem(_params(v, d, t)) for v in VARIANTS for d in DELTAS]
    runs = []
    for _ in range(3):
        obs, st = _evolve(engine, probs, t, span_tile=11, span_outputs=m)
        assert st["span_problems"] == 9 and st["outputs_per_launch"] == m
        runs.append(obs)
    for r in runs[1:]:
        assert np.array_equal(r, runs[0])


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("tile", [11, 10])
def test_lone_spanned_register_matches_default_kernel(engine, variant, tile):
    """One register per evolve, 1 ms / 101 outputs (config 3's grid), 150 kHz (the stiffest
    point): k_span against the persistent interval kernel, both exact propagators (1e-11).  The
    13-qubit center_off register would take the propagator-matrix mode alone (matrix = 0 here)."""
    t = np.linspace(0.0, 1e-3, 101)
    p = pb.build_problem(_params(variant, 150e3, t))
    ref, st0 = _evolve(engine, [p], t, matrix=0, span_tile=0)
    obs, st = _evolve(engine, [p], t, span_tile=tile, matrix=0)
    assert st0["span_problems"] == 0 and st["span_problems"] == 1
    err = float(np.max(np.abs(obs - ref)))
    assert err < 1e-11, err


def test_automatic_span_policy(engine):
    """span_tile = -1 (default): the nine config-3 registers (4 + 8 + 8 tiles each) span over 2^11
    tiles; with span_tile = 0 they run on the whole-register kernels."""
    t = np.linspace(0.0, 1e-4, 11)
    probs = [pb.build_problem(_params(v, d, t)) for v in VARIANTS for d in DELTAS]
    auto, st_a = _evolve(engine, probs, t)
    off, st_o = _evolve(engine, probs, t, span_tile=0)
    assert st_a["span_problems"] == 9 and st_o["span_problems"] == 0
    assert float(np.max(np.abs(auto - off))) < 1e-11


def test_output_count_options_are_range_checked(engine):
    """span_outputs takes 1..4 (k_span staggers the sums); outputs_per_launch stays 1..2 (k_interval
    and k_real hold the sums of one term in registers); a bad value is refused, the old one kept."""
    for key, bad in (("span_outputs", 5), ("span_outputs", 0), ("outputs_per_launch", 3),
                     ("span_chunks", 3), ("span_partial_tile", 12), ("span_partial_tile", 9)):
        with pytest.raises(ValueError):
            engine.set_option(key, bad)
    t = np.linspace(0.0, 1e-4, 11)
    probs = [pb.build_problem(_params("center_on", 75000, t))]
    _, st = _evolve(engine, probs, t, span_tile=11)
    assert st["span_problems"] == 1 and st["outputs_per_launch"] == 4
    _, st = _evolve(engine, probs, t, span_tile=0)
    assert st["span_problems"] == 0 and st["outputs_per_launch"] == 2


def test_automatic_span_policy_strong_split_shares(engine):
    """span_tile = -1 on one GPU's share of a strong split of the 64-point sweep.  The 8-GPU share
    (24 registers) spans whole in one resident launch; the 4-GPU share (48 registers) and the 2-GPU
    share (96) take the partial form: the stiffest registers span over 2^11-amplitude tiles on a
    lane of their own beside k_interval (4-GPU: 151 against 167 ms for all spanned in two launches;
    2-GPU: 212 against 233 ms on k_interval alone, profiles/r06/span_partial_shards.jsonl).  All
    agree with span_tile = 0."""
    t = np.linspace(0.0, 1e-4, 11)
    dets = np.linspace(0.0, 150e3, 64)
    for world, rank in ((8, 7), (4, 3), (2, 1)):
        probs = [pb.build_problem(_params(v, float(d), t)) for d in dets[rank::world] for v in VARIANTS]
        auto, st_a = _evolve(engine, probs, t)
        off, st_o = _evolve(engine, probs, t, span_tile=0)
        if world == 8:
            assert st_a["span_problems"] == len(probs), (world, st_a["span_problems"])
        else:
            assert 0 < st_a["span_problems"] < len(probs), (world, st_a["span_problems"])
        assert st_o["span_problems"] == 0
        assert float(np.max(np.abs(auto - off))) < 1e-11, world


def test_automatic_span_policy_skips_contexts_with_larger_registers(engine):
    """The partial form's chain model covers 1- and 2-tile registers only: a context holding
    several larger registers (here two N = 16 registers, four tiles each, on the Walsh-Hadamard
    engine) leaves the policy before it prices them (round 6: an out-of-range table read there
    crashed the N = 30 loopback-shard test) and spans nothing."""
    t = np.linspace(0.0, 2e-5, 3)
    probs = [pb.build_problem(sweep_point_params(15, 75e3, v, float(t[-1]), len(t))) for v in ("center_on", "shell_off")]
    assert all(p.n_qubits == 16 for p in probs)
    obs, st = _evolve(engine, probs, t)
    assert st["span_problems"] == 0
    np.testing.assert_allclose(obs[:, 6], 1.0, atol=1e-12)
