"""Partitioned registers (single large state): the top shard_bits qubits are
global, every shard holds 2^(n - shard_bits) amplitudes and terms that cross shards read the
partner shard.  Here all shards of a register live on one GPU (dse_add_problem_sharded with
shard_rank = -1): the kernels, tile indexing, partner addressing, psi0 placement and observable
sums are exactly those of the multi-process RCCL path, whose only difference is that partner
shards arrive through ncclSend/ncclRecv into receive buffers instead of being read in place.

Checks: H|psi> of a sharded register equals the unsharded engine's and the reference CSR (N = 12
golden); evolutions and final states equal the unsharded ones to 1e-12 and the oracle (expm)."""
import numpy as np
import pytest

from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.sweep import sweep_point_params
from test_gpu_parity import _random_problem

CASES = [(10, 1, 6), (12, 1, 10), (12, 2, 8), (12, 3, 6), (13, 3, 10), (14, 2, 12)]


@pytest.mark.gpu
@pytest.mark.parametrize("n,bits,tile", CASES)
def test_sharded_apply_h_matches_unsharded(engine, n, bits, tile):
    prob = _random_problem(n, 900 + 10 * n + bits, rare_bit=n - 1)
    rng = np.random.default_rng(n * 7 + bits)
    v = rng.standard_normal(1 << n) + 1j * rng.standard_normal(1 << n)
    engine.set_option("tile_bits", tile)
    try:
        engine.clear()
        p0 = engine.add(prob)
        ref = engine.apply_h(p0, v)
        obs_ref = engine.observables(p0, v)
        engine.clear()
        ps = engine.add_sharded(prob, bits)
        out = engine.apply_h(ps, v)
        obs = engine.observables(ps, v)
    finally:
        engine.clear()
        engine.set_option("tile_bits", 13)
    assert np.max(np.abs(out - ref)) <= 1e-12 * np.max(np.abs(ref))
    np.testing.assert_allclose(obs, obs_ref, rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["center_on", "shell_off"])
def test_sharded_apply_h_matches_reference_n12(engine, golden, variant):
    g = golden("hpsi_n12.npz")
    prob = pb.build_problem(sweep_point_params(11, 50000.0, variant, 2e-3, 201),
                            order="reference", reduce=False)
    engine.set_option("tile_bits", 9)
    try:
        engine.clear()
        ps = engine.add_sharded(prob, 3)
        out = engine.apply_h(ps, g[f"{variant}_v"])
    finally:
        engine.clear()
        engine.set_option("tile_bits", 13)
    ref = g[f"{variant}_Hv"]
    assert np.max(np.abs(out - ref)) <= 1e-13 * np.max(np.abs(ref))


@pytest.mark.gpu
@pytest.mark.parametrize("n,bits,tile", [(11, 1, 8), (12, 3, 8), (14, 3, 10)])
def test_sharded_evolve_matches_unsharded_and_expm(engine, n, bits, tile):
    import scipy.sparse as sp
    from scipy.sparse.linalg import expm_multiply
    from quantumsimulations_amd.dipolar_ensemble_with_rare import problem_to_csr
    prob = _random_problem(n, 4242 + n, rare_bit=n - 1)
    t = np.linspace(0.0, 4e-4, 5)
    engine.set_option("tile_bits", tile)
    try:
        engine.clear()
        p0 = engine.add(prob)
        ps = engine.add_sharded(prob, bits)
        other = engine.add(_random_problem(n - 1, 77, rare_bit=n - 2))   # batched alongside
        obs, st = engine.evolve(t)
        assert st["mode"] == 0
        s_ref, s_sh = engine.state(p0), engine.state(ps)
    finally:
        engine.clear()
        engine.set_option("tile_bits", 13)
    for i in range(1 << bits):          # every shard row holds the whole register's observables
        np.testing.assert_allclose(obs[ps + i], obs[p0], rtol=0, atol=1e-12)
    assert np.max(np.abs(s_sh - s_ref)) < 1e-12
    psi0 = np.zeros(1 << n, dtype=complex)
    psi0[prob.psi0_index] = 1.0
    ex = expm_multiply(-1j * t[-1] * sp.csr_matrix(problem_to_csr(prob)), psi0)
    assert np.max(np.abs(s_sh - ex)) < 1e-10
    assert other == ps + (1 << bits)


@pytest.mark.gpu
def test_sharded_argument_errors(engine):
    prob = _random_problem(8, 5)
    engine.clear()
    with pytest.raises(ValueError):
        engine.add_sharded(prob, 4)
    with pytest.raises(RuntimeError):        # a dist shard needs dse_dist_init first
        engine.add_sharded(prob, 1, rank=0)
    engine.clear()
