"""A register partitioned over PROCESSES (include/dse.h dse_add_problem_sharded, shard_rank >= 0):
world-size 2 and 4 on one MI355X, torch.distributed gloo as the transport through the library's host
exchange backend (dse_dist_init_exchange) instead of RCCL.  Everything of the multi-process path
runs for real -- each rank's shard, the index-swap all-to-all of the Walsh-Hadamard engine around
its MID pass, the per-term shard send/recv of the step kernels, the all-reduce of the observable
sums at the end, the partner masks -- only the transport differs from the RCCL one (several
ranks cannot share one GPU under RCCL).  Checked against the unsharded engine in the parent.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
T = np.linspace(0.0, 2e-4, 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _problem(n):
    from test_gpu_parity import _random_problem
    return _random_problem(n, 5150 + n, rare_bit=n - 1)


def _rank(rank, world, port, n, wht, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from quantumsimulations_amd.engine import Engine
    try:
        with Engine(0) as eng:
            eng.set_option("wht", wht)
            eng.dist_init_exchange(rank, world, dist)
            prob = _problem(n)
            bits = world.bit_length() - 1
            pid = eng.add_sharded(prob, bits, rank)
            rng = np.random.default_rng(77)
            v = rng.standard_normal(1 << n) + 1j * rng.standard_normal(1 << n)
            shard = v.reshape(1 << bits, -1)[rank].copy()
            hv = eng.apply_h(pid, shard)
            ov = eng.observables(pid, shard)
            obs, st = eng.evolve(T)
            out[rank] = {"hv": hv, "ov": ov, "obs": obs[pid], "state": eng.state(pid),
                         "mode": st["mode"], "xbytes": st["exchange_bytes"]}
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,world,wht", [(16, 2, 1), (16, 2, 0), (17, 4, 1), (15, 4, 0)])
def test_partitioned_over_processes_matches_unsharded(engine, n, world, wht):
    import torch.multiprocessing as mp
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rank, args=(world, _free_port(), n, wht, out), nprocs=world, join=True)
    prob = _problem(n)
    rng = np.random.default_rng(77)
    v = rng.standard_normal(1 << n) + 1j * rng.standard_normal(1 << n)
    engine.clear()
    engine.set_option("wht", wht)
    engine.set_option("span_tile", 0)  # the unsharded reference on the same engine family
    try:
        p0 = engine.add(prob)
        hv = engine.apply_h(p0, v)
        ov = engine.observables(p0, v)
        ref, st = engine.evolve(T)
        s_ref = engine.state(p0)
    finally:
        engine.set_option("wht", 1)
        engine.set_option("span_tile", -1)
        engine.clear()
    parts = np.split(hv, world)
    sparts = np.split(s_ref, world)
    for r in range(world):
        got = out[r]
        assert got["mode"] == st["mode"] == (2 if wht else 0)
        assert np.max(np.abs(got["hv"] - parts[r])) <= 1e-12 * np.max(np.abs(hv))
        np.testing.assert_allclose(got["ov"], ov, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(got["obs"], ref[p0], rtol=0, atol=1e-12)
        assert np.max(np.abs(got["state"] - sparts[r])) < 1e-12
        assert got["xbytes"] > 0.0
