"""BASELINE config 5 at its own size on one GPU: N = 30 (n_sea = 29 + the driven rare spin,
center_on, 50 kHz; 2^30 amplitudes = 16 GiB per state vector), the register the 8-GPU run
partitions.  tests/test_gpu_config5.py holds the same checks at N = 26 and pins H element by
element at N = 28; here they run where the partitioned path's data movement is at full scale.

* Walsh-Hadamard engine (default for registers of more than two tiles) against the per-term step
  kernels (option wht = 0) over t = 0, 0.2, 0.4 us: all seven observables (abs 1e-11).
* The register as 8 loopback shards (top 3 qubits global; the index-swap exchange between shards
  around the MID pass, as device copies -- the 8-GPU run's data movement) against the unsharded
  engine over the bench's 5 us / 6-output window (abs 1e-12), and the exact invariants of the
  unitary evolution, size-independent: <H> of the final state equals <psi0|H|psi0> = D(x0)
  (rel 1e-11) and ||psi(t)|| = 1 at every output (1e-12).

(tools/check_config5_n30.py is the same check as a script; profiles/r02/config5_n30_check.json.)
Device memory: ~80 GiB unsharded, the same again as shards; the context is cleared between runs.
"""
import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import sweep_point_params
from test_gpu_config5 import diag_energy

pytestmark = pytest.mark.gpu
N_SEA = 29


@pytest.fixture(scope="module")
def prob30():
    p = pb.build_problem(sweep_point_params(N_SEA, 50e3, "center_on", 5e-6, 6))
    assert p.n_qubits == 30
    return p


def _evolve(engine, prob, t, wht=1, shards=0):
    engine.clear()
    engine.set_option("wht", wht)
    try:
        pid = engine.add_sharded(prob, shards) if shards else engine.add(prob)
        obs, st = engine.evolve(t)
        e, n2 = engine.energy(pid)
        return obs[pid], st, e, n2
    finally:
        engine.set_option("wht", 1)
        engine.clear()


def test_n30_wht_engine_matches_step_kernels(engine, prob30):
    t = np.linspace(0.0, 4e-7, 3)
    a, st_a, _, _ = _evolve(engine, prob30, t, wht=1)
    b, st_b, _, _ = _evolve(engine, prob30, t, wht=0)
    assert st_a["mode"] == 2 and st_b["mode"] == 0, (st_a["mode"], st_b["mode"])
    err = float(np.max(np.abs(a - b)))
    print(f"N=30 WHT vs step kernels: {err:.2e}")
    assert err < 1e-11, err


def test_n30_sharded_loopback_matches_unsharded(engine, prob30):
    t = np.linspace(0.0, 5e-6, 6)
    e0 = diag_energy(prob30)
    ref, st_u, e_u, n2_u = _evolve(engine, prob30, t)
    obs, st_s, e_s, n2_s = _evolve(engine, prob30, t, shards=3)
    assert st_u["mode"] == 2 and st_s["mode"] == 2
    err = float(np.max(np.abs(obs - ref)))
    print(f"N=30 8 loopback shards vs unsharded: {err:.2e}; energy rel {abs(e_u - e0) / abs(e0):.1e} / "
          f"{abs(e_s - e0) / abs(e0):.1e}")
    assert err < 1e-12, err
    for e, n2, o in ((e_u, n2_u, ref), (e_s, n2_s, obs)):
        assert abs(e - e0) / abs(e0) < 1e-11, (e, e0)
        assert abs(n2 - 1.0) < 1e-12, n2
        assert float(np.max(np.abs(o[6] - 1.0))) < 1e-12
