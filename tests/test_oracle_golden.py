"""Pin the CPU oracle to the golden vectors produced by the reference's own code.

Fixtures: tests/golden/make_golden.py (reference dipolar_ensemble_with_rare.py run
through a QuTiP-API stand-in in the build container).  Everything here is CPU-only.
"""
import dataclasses

import numpy as np
import pytest

from conftest import csr_from
from oracle import propagate, reference_model as rm
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params

OBS = rm.OBS_ORDER


def _pdict(n_sea, delta, variant, t_final=2e-3, steps=201):
    return dataclasses.asdict(sweep_point_params(n_sea, delta, variant, t_final, steps))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("delta", [0, 25000, 150000])
def test_oracle_hamiltonian_n7(golden, variant, delta):
    g = golden("hamiltonian_n7.npz")
    key = f"{variant}_{delta}"
    Href = csr_from(g, key)
    H, obs, psi0, aux = rm.build(_pdict(6, float(delta), variant))
    diff = abs(H - Href).max()
    assert diff <= 1e-15 * abs(Href).max()
    assert aux["psi0_index"] == int(g[f"{key}_psi0_index"])
    v = g[f"{key}_v"]
    for k in OBS:
        np.testing.assert_allclose(obs[k] @ v, g[f"{key}_O_{k}"], rtol=0, atol=1e-15)


@pytest.mark.parametrize("variant", VARIANTS)
def test_oracle_hpsi_n12(golden, variant):
    g = golden("hpsi_n12.npz")
    H, obs, psi0, aux = rm.build(_pdict(11, 50000.0, variant))
    v = g[f"{variant}_v"]
    hv = H @ v
    ref = g[f"{variant}_Hv"]
    assert np.max(np.abs(hv - ref)) <= 1e-14 * np.max(np.abs(ref))
    assert aux["psi0_index"] == int(g[f"{variant}_psi0_index"])
    for k in OBS:
        assert abs(np.real(np.vdot(v, obs[k] @ v)) - float(g[f"{variant}_expect_{k}"])) < 1e-13


@pytest.mark.parametrize("variant", VARIANTS)
def test_oracle_and_host_tables_hpsi_n14(golden, variant):
    """N = 14 (config 3): the oracle's Kronecker H and the host's bitwise tables (the engine's
    input) both reproduce the reference-built H @ v at the stiffest detuning."""
    from quantumsimulations_amd import problem as pb
    g = golden("hpsi_traces_n14.npz")
    key = f"{variant}_150000"
    rng = np.random.default_rng(1400)                     # make_golden.rand_state(2^14, 1400)
    v = rng.standard_normal(1 << 14) + 1j * rng.standard_normal(1 << 14)
    v /= np.linalg.norm(v)
    ref = g[f"{key}_Hv"]
    H, obs, psi0, aux = rm.build(_pdict(13, 150000.0, variant, 2e-4, 21))
    assert np.max(np.abs(H @ v - ref)) <= 1e-14 * np.max(np.abs(ref))
    assert aux["psi0_index"] == int(g[f"{key}_psi0_index"])
    prob = pb.build_problem(sweep_point_params(13, 150000.0, variant, 2e-4, 21), order="reference",
                            reduce=False)
    tab = {"n": prob.n_qubits, "field": prob.field, "zz": prob.zz, "pair": prob.pair,
           "flip": prob.flip, "shift": prob.shift}
    assert np.max(np.abs(rm.bitwise_apply(tab, v) - ref)) <= 1e-14 * np.max(np.abs(ref))
    for k in OBS:
        assert abs(np.real(np.vdot(v, obs[k] @ v)) - float(g[f"{key}_expect_{k}"])) < 1e-13
    # the fixture's traces: two independent Chebyshev enclosures agree to ~1e-12
    assert float(g[f"{key}_cross_check"]) < 5e-12


def test_oracle_geometry(golden):
    g = golden("geometry.npz")
    for n in (1, 2, 3, 4, 5, 6, 7, 8, 11, 12, 13, 20, 29):
        pos = rm.positions(n, 0.282393e-9)
        np.testing.assert_array_equal(pos, g[f"pos_{n}"])
        b = rm.couplings(pos, 1.0e-7 * 1.054571817e-34, 8.1812e7, 6.976e7)
        np.testing.assert_allclose(b, g[f"b_center_{n}"], rtol=1e-15, atol=0)


@pytest.mark.parametrize("variant", VARIANTS)
def test_oracle_exact_trace_n7(golden, variant):
    """Oracle exact propagation reproduces the exact trace of the reference-built H."""
    tr = golden("traces_n7.npz")
    H, obs, psi0, _ = rm.build(_pdict(6, 50000.0, variant))
    t = tr["t"]
    ex = propagate.eigh_trace(H, psi0, t, obs)
    for k in OBS:
        np.testing.assert_allclose(ex[k], tr[f"{variant}_exact_{k}"], rtol=0, atol=1e-11)
    # the QuTiP-5-equivalent integrator at the sweep's tolerances is ~1e-5 off exact (SURVEY finding 6)
    d_ref = max(np.max(np.abs(tr[f"{variant}_ref_{k}"] - tr[f"{variant}_exact_{k}"])) for k in OBS)
    assert 1e-7 < d_ref < 1e-3


def test_oracle_expm_matches_eigh_n7(golden):
    tr = golden("traces_n7.npz")
    H, obs, psi0, _ = rm.build(_pdict(6, 50000.0, "center_on"))
    t = tr["t"][:41]
    a = propagate.expm_trace(H, psi0, t, obs)
    for k in OBS:
        np.testing.assert_allclose(a[k], tr[f"center_on_exact_{k}"][:41], rtol=0, atol=1e-10)


def test_oracle_zvode_reproduces_reference_integrator(golden):
    """bench.py's CPU baseline integrator == the reference-behaviour trace (same algorithm)."""
    tr = golden("traces_n7.npz")
    H, obs, psi0, _ = rm.build(_pdict(6, 50000.0, "center_off"))
    t = tr["t"]
    z, info = propagate.zvode_trace(H, psi0, t, obs, atol=1e-10, rtol=1e-9, nsteps=10_000_000,
                                    max_step=1e-5)
    for k in OBS:
        np.testing.assert_allclose(z[k], tr[f"center_off_ref_{k}"], rtol=0, atol=1e-9)
    assert info["rhs"] == pytest.approx(float(tr["center_off_rhs_ref"]), rel=0.02)


def test_oracle_exact_trace_n12_fixture_consistency(golden):
    tr = golden("traces_n12.npz")
    # sanity of the fixture itself: norm 1, Iz_sea starts at -n_sea/2 (all sea spins down)
    np.testing.assert_allclose(tr["exact_state_norm"], 1.0, atol=1e-12)
    assert tr["exact_Iz_sea"][0] == pytest.approx(-5.5)
    assert tr["exact_Iz_R"][0] == pytest.approx(0.5)
