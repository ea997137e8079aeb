#!/usr/bin/env python3
"""Benchmark: N = 14 sea-detuning sweep on MI355X (BASELINE.json metric, config 3).

One "step" = one full batch of the hot path: the 64-detuning x 3-variant sweep
(192 independent evolutions, n_sea = 13 + 1 rare = 14 qubits) propagated over the
head-to-head grid t_final = 1e-3 s, 101 output times, with all seven observable
traces computed.  Problem tables are uploaded before the timed region (inputs
resident in HBM); each timed step resets every state to psi0 and runs the whole
evolution (Chebyshev step kernels + observable reductions) to t_final.

value = detuning-points / hour over the whole job (points of all ranks / max rank time).
Multi-GPU (torchrun, one process per GPU): weak scaling; rank r of N takes the
detunings j = r (mod N) of linspace(0, 150 kHz, 64 N), i.e. 64 distinct points per
rank, no data-path collective (evolutions are independent).

Extra fields: "roofline" (dominant kernel: the Chebyshev step, HIP events around
each launch inside the timed region) and "cpu_baseline" (rank 0, N = 1 only: the
QuTiP-5 sesolve equivalent -- scipy ZVODE-Adams + CSR, oracle/propagate.py --
on a bounded sample, extrapolated linearly in simulated time) and "large_register"
(rank 0, N = 1 only: config 5 on one GPU, N = 30, the Walsh-Hadamard engine's passes
against the HBM roofline; --no-large skips it).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6         # MI355X FP64 vector spec
N_SEA = 13
N_DET = 64
T_FINAL = 1e-3
STEPS_T = 101
DELTA_MAX = 150_000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tile-bits", type=int, default=int(os.environ.get("DSE_TILE_BITS", "13")))
    ap.add_argument("--streams", type=int, default=int(os.environ.get("DSE_STREAMS", "4")))
    ap.add_argument("--cpu-budget", type=float, default=float(os.environ.get("DSE_CPU_BUDGET_S", "20")))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streaming", action="store_true", help="per-term streaming kernels instead of "
                    "the persistent interval kernel")
    ap.add_argument("--outputs-per-launch", type=int, default=int(os.environ.get("DSE_OUTPUTS_PER_LAUNCH", "2")),
                    help="persistent mode: output times propagated per launch from one Chebyshev series")
    ap.add_argument("--n-sea", type=int, default=N_SEA)
    ap.add_argument("--n-det", type=int, default=N_DET)
    ap.add_argument("--no-large", action="store_true", help="skip the config-5 single-GPU leg")
    return ap.parse_args()


PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01", "v7_pmc_traffic.json")


def pmc_traffic(kernel: str):
    """HBM-side bytes per launch of ``kernel`` from the committed rocprofv3 counter passes of this
    bench command (FETCH_SIZE doubled per the gfx950 correction, plus WRITE_SIZE), or None."""
    try:
        with open(PMC_TRAFFIC) as f:
            rec = json.load(f)["kernels"][kernel]
        return rec["traffic_bytes_per_launch"], os.path.relpath(PMC_TRAFFIC, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def flops_per_amp(prob) -> float:
    """Algorithmic flops per amplitude of one H application:
    diagonal 4, each drive flip 8, each pair 4 on half the rows (= 2 per amp)."""
    n_pairs = int(np.count_nonzero(np.triu(prob.pair, 1)))
    n_flips = int(np.count_nonzero(np.any(prob.flip != 0.0, axis=1)))
    return 4.0 + 8.0 * n_flips + 2.0 * n_pairs


def cpu_baseline(budget_s: float):
    """QuTiP-5 sesolve equivalent (oracle) on one detuning point, 3 variants, bounded sample."""
    from oracle import propagate, reference_model as rm
    import dataclasses
    from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params
    delta = 75_000.0
    per_var = budget_s / 3.0
    total_wall_full = 0.0
    reached = []
    for v in VARIANTS:
        p = sweep_point_params(N_SEA, delta, v, T_FINAL, STEPS_T)
        H, obs, psi0, _ = rm.build(dataclasses.asdict(p))
        t = np.linspace(0.0, T_FINAL, STEPS_T)
        _, info = propagate.zvode_trace(H, psi0, t, obs, atol=1e-10, rtol=1e-9, nsteps=10_000_000,
                                        max_step=1e-5, time_budget_s=per_var)
        frac = info["t_reached"] / T_FINAL
        total_wall_full += info["wall_s"] / max(frac, 1e-12)
        reached.append(info["t_reached"])
    pts_per_hour = 3600.0 / total_wall_full
    return {
        "value": pts_per_hour, "unit": "detuning-points/hour", "cores": 1, "kind": "port",
        "sample": (f"ZVODE-Adams (QuTiP-5 sesolve equivalent, oracle/propagate.py) + scipy CSR, "
                   f"atol 1e-10 rtol 1e-9, N=14, delta=75 kHz, 3 variants, first "
                   f"{[round(r * 1e6, 1) for r in reached]} us of the {T_FINAL * 1e6:.0f} us grid, "
                   f"extrapolated linearly in simulated time; 1 core"),
        "seconds_per_point_extrapolated": total_wall_full,
    }


WHT_PMC_N30 = os.path.join(ROOT, "profiles", "r01", "wht_n30_pmc_traffic.json")


def large_register(device: int, n_sea: int = 29):
    """Config 5 on one GPU (N = n_sea + 1 = 30, center_on, 50 kHz, t_final 5e-6 s, 6 outputs): the
    Walsh-Hadamard engine's H|psi> passes against the HBM roofline.  Bytes per amplitude and H
    application are the passes' algorithmic traffic (FIRST 48, FWD/MID/INV 64 each, FINAL 80 + acc
    32 every third term); "traffic" is the rocprofv3 FETCH/WRITE count of the same passes
    (profiles/r01/wht_n30_pmc_traffic.json).  Kernel time per H application from HIP events
    (excludes the first call's device allocation of 5 x 16 GiB)."""
    from quantumsimulations_amd import problem as pb
    from quantumsimulations_amd.engine import Engine
    from quantumsimulations_amd.sweep import sweep_point_params
    t_final, steps = 5e-6, 6
    p = sweep_point_params(n_sea, 50e3, "center_on", t_final, steps)
    prob = pb.build_problem(p)
    n = prob.n_qubits
    wl = 13
    groups = 1 + -(-(n - wl) // (wl - 2))
    bpa = 48.0 + 64.0 * (2 * groups - 3) + 80.0 + 32.0 / 3.0
    with Engine(device) as eng:
        eng.add(prob)
        t0 = time.perf_counter()
        _, st = eng.evolve(np.linspace(0.0, t_final, steps))
        wall = time.perf_counter() - t0
    per_term_ms = st["step_kernel_ms"] / max(st["timed_launches"], 1)
    gbs = bpa * (1 << n) / (per_term_ms * 1e-3) / 1e9
    traffic = None  # HBM-side bytes per H application (MODE_GEN passes) from the counter passes
    try:
        with open(WHT_PMC_N30) as f:
            k = json.load(f)["kernels"]
        if n == 30:
            traffic = sum(k[f"k_wht<13, {ps}, 2>"]["traffic_bytes_per_launch"] for ps in range(5))
    except (OSError, KeyError, ValueError):
        pass
    return {
        "workload": f"config 5 on one GPU: N={n} center_on, 50 kHz, t_final {t_final} s, {steps} outputs",
        "engine_mode": st["mode"], "tile_bits": wl, "passes_per_h": 2 * groups - 1,
        "h_applications": st["h_applications"],
        "kernel_ms_per_h_application": per_term_ms,
        "wall_ms_per_h_application_incl_setup": wall / st["h_applications"] * 1e3,
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": gbs / HBM_PEAK_GBS, "bytes_per_amp_per_h": bpa, "traffic": traffic,
                     "traffic_source": os.path.relpath(WHT_PMC_N30, ROOT)},
    }


def shard_detunings(n_det_per_rank: int, rank: int, world: int) -> np.ndarray:
    """Weak scaling: rank r takes detunings j = r (mod world) of linspace(0, 150 kHz, n*world)."""
    return np.linspace(0.0, DELTA_MAX, n_det_per_rank * world)[rank::world]


def timed_steps(step, steps: int, warmup: int, sync, dist=None) -> float:
    """W untimed steps, then K steps bracketed by barrier + device sync on both sides; returns
    the maximum over ranks of the timed wall time."""
    import torch

    def barrier():
        sync()
        if dist is not None:
            dist.barrier()
    for _ in range(warmup):
        step()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            tt = tt.cuda()
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    return dt


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # RCCL carries only the barrier and the max-time reduction: the evolutions are independent
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    from quantumsimulations_amd import problem as pb
    from quantumsimulations_amd.engine import Engine
    from quantumsimulations_amd.sweep import sweep_params

    my_det = shard_detunings(args.n_det, rank, world)
    params = sweep_params(args.n_sea, my_det, T_FINAL, STEPS_T)
    probs = [pb.build_problem(p) for p in params]
    t = np.linspace(0.0, T_FINAL, STEPS_T)

    eng = Engine(local, tile_bits=args.tile_bits)
    eng.set_option("streams", args.streams)
    eng.set_option("persistent", 0 if args.streaming else 1)
    eng.set_option("outputs_per_launch", args.outputs_per_launch)
    if os.environ.get("DSE_CORESIDENT"):  # diagnostics: workgroups per 2-tile interval launch chunk
        eng.set_option("coresident", float(os.environ["DSE_CORESIDENT"]))
    for p in probs:
        eng.add(p)

    stats = []
    warm = [args.warmup]

    def step():
        _, st = eng.evolve(t)
        if warm[0] > 0:
            warm[0] -= 1
        else:
            stats.append(st)
    dt = timed_steps(step, args.steps, args.warmup, torch.cuda.synchronize, dist)

    points = len(my_det) * world * args.steps
    value = points / dt * 3600.0
    h_apps = sum(s["h_applications"] for s in stats)
    mode = stats[-1]["mode"]
    k_ms = sum(s["step_kernel_ms"] for s in stats)            # HIP-event time of timed launches
    k_launches = sum(s["timed_launches"] for s in stats)
    k_flops = sum(s["timed_flops"] for s in stats)             # their algorithmic flops
    k_bytes = sum(s["timed_bytes"] for s in stats)             # their algorithmic HBM bytes (streaming)
    all_flops = sum(s["h_flops"] for s in stats)
    all_bytes = sum(s["step_bytes"] for s in stats)
    fpa = sum(flops_per_amp(p) * (1 << p.n_qubits) for p in probs) / sum(1 << p.n_qubits for p in probs)
    if mode == 1:
        # persistent interval kernel: the state stays in LDS/registers for all terms of an output
        # interval; HBM moves only psi (once per interval) -> bounded by FP64 VALU throughput
        achieved = k_flops / (k_ms * 1e-3) / 1e12 if k_ms > 0 else None
        traffic, traffic_src = pmc_traffic("k_interval<13, true>") if args.tile_bits == 13 else (None, None)
        roof = {
            "kernel": "k_interval<13> (persistent Chebyshev interval: all K terms on chip)",
            "bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "compute": "FP64 VALU (MI355X: FP64 vector peak = dense FP64 MFMA peak = 78.6 TF/s)",
            "frac": (achieved / FP64_PEAK_TFLOPS) if achieved else None, "traffic": traffic,
            "traffic_source": traffic_src,
            "traffic_rate_gbs": (traffic / (k_ms / k_launches * 1e-3) / 1e9) if (traffic and k_launches) else None,
            "algorithmic_flops_per_amp": fpa,
            "avg_launch_us": k_ms / k_launches * 1e3 if k_launches else None,
            "flops_per_launch": k_flops / k_launches if k_launches else None,
            "aggregate_fp64_tflops": all_flops / dt / 1e12,
            "note": ("the H terms stay on chip (LDS + registers) for a whole launch, so the bound is FP64 "
                     "issue (with LDS bandwidth close behind), not HBM; traffic = L2<->fabric bytes per "
                     "launch from rocprofv3 FETCH_SIZE/WRITE_SIZE passes, dominated by the 2-tile "
                     "problems' per-term hand-off; the streaming formulation would move 58.7 B per "
                     "amplitude per term, i.e. an HBM-equivalent rate of "
                     f"{all_flops / fpa * 58.7 / dt / 1e9:.0f} GB/s"),
        }
    else:
        achieved = k_bytes / (k_ms * 1e-3) / 1e9 if k_ms > 0 else None
        roof = {
            "kernel": ("k_wht passes (Walsh-Hadamard engine: one Chebyshev term = FIRST, MID, FINAL)"
                       if mode == 2 else
                       "k_step_rb<13,MODE_GEN> (Chebyshev step: H|w>, recurrence, accumulation)"),
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
            "algorithmic_bytes_per_amp": 58.7,
            "avg_launch_us": k_ms / k_launches * 1e3 if k_launches else None,
            "bytes_per_launch": k_bytes / k_launches if k_launches else None,
            "achieved_fp64_tflops": k_flops / (k_ms * 1e-3) / 1e12 if k_ms > 0 else None,
            "aggregate_step_gbs": all_bytes / dt / 1e9,
            "note": ("per-launch HIP-event durations; launches of different streams overlap, so "
                     "per-launch GB/s understates the aggregate (aggregate_step_gbs)"),
        }
    line = {
        "metric": "detuning-points/hour (N=14 sea-detuning sweep, 3 variants per point)",
        "value": value,
        "unit": "detuning-points/hour",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64 (complex128 state)",
        "data": "synthetic (reference physical constants, deterministic; no external data)",
        "config": {
            "workload": (f"config 3: n_sea={args.n_sea}+1 rare (N=14 qubits), {len(my_det)} detunings in "
                         f"[0,150 kHz] x 3 variants = {3 * len(my_det)} evolutions per GPU, "
                         f"t_final={T_FINAL}s, {STEPS_T} outputs, 7 observables"),
            "global_points_per_step": len(my_det) * world,
            "evolutions_per_step_per_gpu": len(probs),
            "propagator": "exact Chebyshev (tol 1e-14)",
            "engine_mode": {1: "persistent", 2: "walsh-hadamard"}.get(mode, "streaming"),
            "tile_bits": args.tile_bits,
            "streams": args.streams,
            "outputs_per_launch": stats[-1].get("outputs_per_launch"),
            "ms_per_ode_step": (dt / args.steps) / (h_apps / args.steps / len(probs)) * 1e3,
            "h_applications_per_step": h_apps / args.steps,
            "parallelism": f"evolution-sharded x{world} (no collectives)",
        },
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(args.cpu_budget)
        except Exception as exc:  # report, never hide
            line["cpu_baseline"] = {"value": None, "error": repr(exc)}
    eng.close()
    if rank == 0 and world == 1 and not args.no_large:
        try:
            line["large_register"] = large_register(local)
        except Exception as exc:  # report, never hide
            line["large_register"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
