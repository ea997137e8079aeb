"""Robustness of the persistent kernel's cross-workgroup hand-off (2-tile registers, N = 14).

The two tiles of a 2-tile problem are two workgroups that exchange an operand every Chebyshev
term through flags in global memory (dse_interval.hip); that needs both to be resident at once.
Launch chunks are sized by the occupancy query (dse_runtime.hip), and when a partner still does
not show up within the spin limit (the GPU shared with long-running work) the evolve is re-run on
the streaming kernels, which have no inter-workgroup dependency.
"""
import threading
import time

import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import sweep_point_params

pytestmark = pytest.mark.gpu
T = np.linspace(0.0, 2e-5, 5)


@pytest.fixture(autouse=True)
def _interval_kernel(engine):
    """These tests exercise k_interval's 2-tile hand-off: the real-component mode (dse_real.hip, no
    hand-off at all) and the automatic span are switched off for them."""
    engine.set_option("real", 0)
    engine.set_option("span_tile", 0)  # whole registers (no automatic span)
    yield
    engine.set_option("real", 0)
    engine.set_option("span_tile", -1)


def _two_tile_problems():
    return [pb.build_problem(sweep_point_params(13, d, v, float(T[-1]), len(T)))
            for d in (0.0, 150e3) for v in ("center_on", "shell_off")]


def test_handoff_failure_falls_back_to_streaming(engine):
    probs = _two_tile_problems()
    engine.clear()
    for p in probs:
        engine.add(p)
    ref, st = engine.evolve(T)
    assert st["mode"] == 1 and st["handoff_fallbacks"] == 0
    engine.set_option("spin_limit", -1)       # diagnostics: every hand-off wait fails
    try:
        got, st2 = engine.evolve(T)
    finally:
        engine.set_option("spin_limit", 1 << 22)
    assert st2["mode"] in (0, 2) and st2["handoff_fallbacks"] >= 1   # streaming (step or WHT)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)
    again, st3 = engine.evolve(T)              # the context keeps its persistent mode
    assert st3["mode"] == 1 and np.array_equal(again, ref)
    engine.clear()


def test_two_tile_launch_beside_a_busy_device(engine):
    """A second context on another host thread keeps the device busy with long 1-tile interval
    launches (as lane 1 of a sweep, or another job, would) while this context evolves 2-tile
    problems: the results are those of the idle device."""
    from quantumsimulations_amd.engine import Engine
    probs = _two_tile_problems()
    engine.clear()
    for p in probs:
        engine.add(p)
    alone, _ = engine.evolve(T)
    hog = Engine(0)
    t_hog = np.linspace(0.0, 3e-4, 3)
    for d in np.linspace(0.0, 150e3, 96):     # 96 one-tile registers (13 qubits), ~1e3 terms per launch
        hog.add(pb.build_problem(sweep_point_params(13, float(d), "center_off", float(t_hog[-1]), 3)))
    stop = threading.Event()
    errors = []

    def busy():
        try:
            while not stop.is_set():
                hog.evolve(t_hog)
        except BaseException as exc:  # re-raised below
            errors.append(exc)

    th = threading.Thread(target=busy)
    th.start()
    try:
        time.sleep(0.5)
        runs = [engine.evolve(T) for _ in range(4)]
    finally:
        stop.set()
        th.join()
        hog.close()
        engine.clear()
    assert not errors, errors
    for obs, st in runs:
        assert st["mode"] in (0, 1)
        np.testing.assert_allclose(obs, alone, rtol=0, atol=1e-12)


def test_handoff_with_release_acquire_fences(engine):
    """Option handoff_fences = 1 (agent-scope release before each flag store, acquire after each
    poll): the same results as the default sc1 hand-off, bitwise repeatable."""
    t = np.linspace(0.0, 1e-4, 11)
    probs = [pb.build_problem(sweep_point_params(13, 60e3, v, 1e-4, 11)) for v in ("center_on", "shell_off")]
    res = {}
    for f in (0, 1, 1):
        engine.clear()
        engine.set_option("handoff_fences", f)
        try:
            for p in probs:
                engine.add(p)
            obs, st = engine.evolve(t)
        finally:
            engine.set_option("handoff_fences", 0)
        assert st["mode"] == 1
        if f in res:
            assert np.array_equal(obs, res[f])
        res[f] = obs
    np.testing.assert_allclose(res[1], res[0], rtol=0, atol=1e-13)
    engine.clear()


def _run_states(engine, probs, t):
    engine.clear()
    for p in probs:
        engine.add(p)
    obs, st = engine.evolve(t)
    states = [engine.state(i) for i in range(len(probs))]
    return obs, st, states


def test_handoff_fallback_keeps_dense_registers_state(engine):
    """A context holding a dense-engine register beside a 2-tile register: after a hand-off timeout
    the evolve re-runs the Chebyshev registers on the streaming kernels and keeps the dense
    register's first-pass results -- its observables AND its final state (dse_get_state)."""
    import dataclasses
    dense_p = pb.build_problem(sweep_point_params(6, 75e3, "center_on", float(T[-1]), len(T)))
    # a drive phase off pi/2 makes the 14-qubit register's drives complex: not dense-eligible
    cheb_p = pb.build_problem(dataclasses.replace(sweep_point_params(13, 75e3, "shell_off", float(T[-1]), len(T)),
                                                  phi_sea=0.3))
    engine.set_option("dense", 2)
    try:
        ref, st, s_ref = _run_states(engine, [dense_p, cheb_p], T)
        assert st["dense_problems"] == 1 and st["handoff_fallbacks"] == 0
        engine.set_option("spin_limit", -1)
        try:
            got, st2, s_got = _run_states(engine, [dense_p, cheb_p], T)
        finally:
            engine.set_option("spin_limit", 1 << 22)
    finally:
        engine.set_option("dense", 1)
        engine.clear()
    assert st2["dense_problems"] == 1 and st2["handoff_fallbacks"] >= 1
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)
    assert np.array_equal(s_got[0], s_ref[0])            # the dense register's final state
    np.testing.assert_allclose(s_got[1], s_ref[1], rtol=0, atol=1e-12)


def test_span_handoff_failure_falls_back(engine):
    """k_span with an explicit tile (span_tile = 11: 8 workgroups per 14-qubit register): every
    partner wait failing (spin_limit = -1) re-runs the evolve on the streaming kernels with the
    same results."""
    probs = _two_tile_problems()
    engine.set_option("span_tile", 11)
    try:
        ref, st, _ = _run_states(engine, probs, T)
        assert st["span_problems"] == len(probs) and st["handoff_fallbacks"] == 0
        engine.set_option("spin_limit", -1)
        try:
            got, st2, _ = _run_states(engine, probs, T)
        finally:
            engine.set_option("spin_limit", 1 << 22)
    finally:
        engine.set_option("span_tile", 0)
        engine.clear()
    assert st2["handoff_fallbacks"] >= 1
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12)


def test_explicit_span_beyond_the_chip_runs_in_resident_chunks(engine):
    """span_tile = 11 on 48 fourteen-qubit registers: 384 spanning workgroups, more than the chip
    holds at once.  The runtime cuts the group into launches of whole 8-register blocks that fit
    (every register's tiles resident together), so no hand-off waits on a queued partner: no
    fallback, and the results are k_interval's."""
    t = np.linspace(0.0, 1e-4, 11)
    probs = [pb.build_problem(sweep_point_params(13, float(d), v, 1e-4, 11))
             for d in np.linspace(0.0, 150e3, 24) for v in ("center_on", "shell_off")]
    ref, st0, _ = _run_states(engine, probs, t)
    assert st0["span_problems"] == 0
    engine.set_option("span_tile", 11)
    try:
        got, st, _ = _run_states(engine, probs, t)
    finally:
        engine.set_option("span_tile", 0)
        engine.clear()
    assert st["span_problems"] == len(probs) and st["handoff_fallbacks"] == 0
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-11)


def test_handoff_options_are_per_context(engine):
    """spin_limit (and handoff_fences) are context options passed with every launch, not
    process-wide settings: a second context that fails every hand-off (spin_limit = -1) leaves
    this context's evolve on the persistent kernel with no fallback."""
    from quantumsimulations_amd.engine import Engine
    probs = _two_tile_problems()
    other = Engine(0)
    try:
        other.set_option("real", 0)
        other.set_option("span_tile", 0)
        other.set_option("spin_limit", -1)
        for p in probs:
            other.add(p)
        engine.clear()
        for p in probs:
            engine.add(p)
        ref, st = engine.evolve(T)
        _, st_o = other.evolve(T)
        again, st2 = engine.evolve(T)
    finally:
        other.close()
        engine.clear()
    assert st["handoff_fallbacks"] == 0 and st2["handoff_fallbacks"] == 0 and st2["mode"] == 1
    assert st_o["handoff_fallbacks"] >= 1
    assert np.array_equal(again, ref)
