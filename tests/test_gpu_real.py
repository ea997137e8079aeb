"""The real-component mode (dse_real.hip, option "real" = 1, or 2 for the 14-qubit registers only;
default 0 = the complex kernels): with imaginary drives the rotated
Hamiltonian H' = D H D^dagger is real symmetric, and the rotated state's real and imaginary parts
run as two independent real Chebyshev recurrences, one workgroup each holding the whole register
in LDS.  Checked against the persistent complex kernel k_interval (option real = 0) -- both exact
propagators, so the traces agree to rounding -- and against the reference-H oracle in
test_gpu_config3.py (parametrised over the mode).

* the bench's registers (N = 14: 13-qubit center_off, 14-qubit center_on / shell_off) at 8 of its
  64 detunings, 1 ms / 101 outputs, one and two outputs per launch: <O>(t) within 1e-11;
* the final state in the computational frame (the combine's i^{|x0| - |x|} phases, the shift
  folded into H') equals k_interval's (dse_get_state), and its energy;
* bitwise repeatable;
* option real = 2: only the 14-qubit (2-tile) registers on k_real, the 13-qubit ones on the 1-tile
  k_interval on a second stream at the same time, against real = 0 (1e-11).
"""
import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import sweep_params

pytestmark = pytest.mark.gpu
T = np.linspace(0.0, 1e-3, 101)


def _probs():
    return [pb.build_problem(p) for p in sweep_params(13, np.linspace(0.0, 150e3, 64)[::8], T[-1], len(T))]


def _run(engine, probs, real, m=2):
    engine.clear()
    engine.set_option("real", real)
    engine.set_option("span_tile", 0)  # whole registers: 24 would span automatically
    engine.set_option("outputs_per_launch", m)
    try:
        for p in probs:
            engine.add(p)
        obs, st = engine.evolve(T)
        states = [engine.state(i) for i in range(len(probs))]
        energies = [engine.energy(i) for i in range(len(probs))]
    finally:
        engine.set_option("real", 0)
        engine.set_option("span_tile", -1)
        engine.set_option("outputs_per_launch", 2)
        engine.clear()
    return obs, st, states, energies


@pytest.mark.parametrize("m", [2, 1])
def test_real_mode_matches_interval_kernel(engine, m):
    probs = _probs()
    ob_r, st_r, s_r, e_r = _run(engine, probs, 1, m)
    ob_c, st_c, s_c, e_c = _run(engine, probs, 0, m)
    assert st_r["real_problems"] == len(probs) and st_c["real_problems"] == 0
    assert st_r["mode"] == 1 and st_r["outputs_per_launch"] == m
    err = float(np.max(np.abs(ob_r - ob_c)))
    print(f"real mode vs k_interval (M={m}): max |d<O>| = {err:.2e}")
    assert err < 1e-11, err
    for a, b in zip(s_r, s_c):
        assert np.max(np.abs(a - b)) < 1e-11
    for (ea, na), (eb, nb) in zip(e_r, e_c):
        assert abs(ea - eb) <= 1e-11 * abs(eb) and abs(na - 1.0) < 5e-12  # truncation tol 1e-14 x 100 intervals


def test_real_mode_is_repeatable(engine):
    probs = _probs()[:6]
    runs = [_run(engine, probs, 1)[0] for _ in range(3)]
    for r in runs[1:]:
        assert np.array_equal(r, runs[0])


def test_mixed_real_and_interval_registers(engine):
    probs = _probs()
    ob_m, st_m, s_m, _ = _run(engine, probs, 2)
    ob_c, st_c, s_c, _ = _run(engine, probs, 0)
    n14 = sum(1 for p in probs if p.n_qubits == 14)
    assert 0 < n14 < len(probs) and st_m["real_problems"] == n14 and st_c["real_problems"] == 0
    err = float(np.max(np.abs(ob_m - ob_c)))
    print(f"real = 2 vs k_interval: max |d<O>| = {err:.2e}")
    assert err < 1e-11, err
    for a, b in zip(s_m, s_c):
        assert np.max(np.abs(a - b)) < 1e-11
