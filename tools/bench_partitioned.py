#!/usr/bin/env python3
"""Config 5: one register partitioned over GPUs.

    torchrun --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_partitioned.py
    python tools/bench_partitioned.py --loopback 8        # all 8 shards on one GPU (test mode)

Rank r holds shard r of the N = n_sea + 1 qubit center_on register (top log2(world) qubits
global, the rare spin among them).  Walsh-Hadamard engine (default, --wht 1): every H application
index-swaps the X / Y vectors twice (RCCL all-to-all, 4 shard-sized transfers of which 1/world
stays local); step kernels (--wht 0): every term exchanges whole shards with the partner ranks the
terms couple (RCCL send/recv).  Rank 0 prints one JSON line: ms per H application, exchanged
bytes per H application and rank, the observables at t_final.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.partitioned import (join, shard_bits_for,  # noqa: E402
                                                simulate_rare_partitioned)
from quantumsimulations_amd.sweep import sweep_point_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-sea", type=int, default=29)
    ap.add_argument("--t-final", type=float, default=1e-5)
    ap.add_argument("--steps", type=int, default=11)
    ap.add_argument("--delta", type=float, default=50e3)
    ap.add_argument("--loopback", type=int, default=0, help="all shards on one GPU (2, 4 or 8)")
    ap.add_argument("--wht", type=int, default=1)
    ap.add_argument("--swap-overlap", type=int, default=1,
                    help="1: each vector's index swap on a second stream under the other's pass")
    ap.add_argument("--transport", choices=("rccl", "host"), default="rccl",
                    help="rccl: libdse's RCCL communicator (one GPU per rank); host: the library's host "
                         "exchange backend over torch.distributed gloo (several ranks may share a GPU)")
    a = ap.parse_args()
    p = sweep_point_params(a.n_sea, a.delta, "center_on", a.t_final, a.steps)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    prob = pb.build_problem(p)
    if a.loopback:
        bits = shard_bits_for(a.loopback)
        with Engine(0) as eng:
            eng.set_option("wht", a.wht)
            eng.set_option("swap_overlap", a.swap_overlap)
            pid = eng.add_sharded(prob, bits)
            t0 = time.perf_counter()
            obs, st = eng.evolve(np.linspace(0.0, a.t_final, a.steps))
            wall = time.perf_counter() - t0
        obs_d = {k: float(obs[pid, j, -1]) for j, k in enumerate(pb.OBS_NAMES)}
        shards, mode = a.loopback, "loopback (all shards on one GPU)"
        st = dict(st, h_applications=st["h_applications"] / shards)   # counted once per shard
    else:
        import torch
        import torch.distributed as dist
        dev = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo")       # bootstrap (rccl) or the data path itself (host)
        with Engine(dev) as eng:
            eng.set_option("wht", a.wht)
            eng.set_option("swap_overlap", a.swap_overlap)
            if a.transport == "rccl":
                join(eng, rank, world, dist)
            else:
                eng.dist_init_exchange(rank, world, dist)
            dist.barrier()
            print(f"[bench_partitioned] rank {rank}/{world} joined ({a.transport}), N={prob.n_qubits}",
                  file=sys.stderr, flush=True)
            t0 = time.perf_counter()
            _, obs, st = simulate_rare_partitioned(p, eng, rank, world)
            wall = time.perf_counter() - t0
            tt = torch.tensor([wall], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            wall = float(tt.item())
        obs_d = {k: float(v[-1]) for k, v in obs.items()}
        shards = world
        mode = "RCCL between ranks" if a.transport == "rccl" else "host exchange over gloo"
        dist.destroy_process_group()
    n = prob.n_qubits
    bits = shard_bits_for(shards)
    n_masks = 0
    hi = n - bits
    for m in range(1, 1 << bits):          # partner masks the terms need (as libdse computes)
        gbits = [hi + i for i in range(bits) if (m >> i) & 1]
        if len(gbits) == 1:
            b = gbits[0]
            n_masks += int(np.any(prob.flip[b] != 0) or np.any(prob.pair[:, b] != 0)
                           or np.any(prob.pair[b, :] != 0) or bool((prob.sea_mask >> b) & 1)
                           or b == prob.rare_bit)
        elif len(gbits) == 2:
            n_masks += int(prob.pair[min(gbits), max(gbits)] != 0)
    shard_bytes = (1 << (n - bits)) * 16
    wht = st.get("mode") == 2
    xbytes = 4 * shard_bytes * (shards - 1) // shards if wht else n_masks * shard_bytes
    measured = st.get("exchange_bytes", 0.0)   # libdse's count of this rank's off-device bytes
    happ = max(st["h_applications"], 1)
    links = max(shards - 1, 1)                 # fully connected xGMI: one link per peer
    if rank == 0:
        print(json.dumps({
            "config": f"config 5: N={n} center_on delta={a.delta:g} Hz, t_final={a.t_final}, "
                      f"{a.steps} outputs, {shards} shards ({mode})",
            "wall_s": wall, "h_applications": st["h_applications"],
            "ms_per_h_application": wall / max(st["h_applications"], 1) * 1e3,
            "shard_GiB": shard_bytes / 2**30, "engine_mode": st.get("mode"),
            "swap_overlap": a.swap_overlap,
            "exchange": "index-swap all-to-all of A, B (x2)" if wht else f"send/recv, {n_masks} partner masks",
            "exchange_bytes_per_h_per_rank": xbytes,
            "exchange_bytes_measured_per_rank": measured,
            "exchange_bytes_measured_per_h_per_rank": measured / happ,
            # the exchange's bytes per link over the whole call's wall time: a lower bound of the
            # per-link rate while the exchange runs (the passes run between exchanges)
            "xgmi_gbs_per_link_lower_bound": (measured / links / wall / 1e9) if not a.loopback else None,
            # the same bytes over the time the exchanges themselves took (HIP events around each
            # RCCL call on its stream; host wall time for the host transport)
            "exchange_ms": st.get("exchange_ms"),
            "xgmi_gbs_per_link": (measured / links / (st["exchange_ms"] * 1e-3) / 1e9)
            if (not a.loopback and st.get("exchange_ms")) else None,
            "obs_t_final": obs_d,
            # exact propagation conserves the norm: the end-to-end check of the exchanged path
            "norm_error": abs(obs_d["state_norm"] - 1.0),
            "ok": bool(abs(obs_d["state_norm"] - 1.0) < 1e-9),
        }), flush=True)


if __name__ == "__main__":
    main()
