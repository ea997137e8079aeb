"""CPU baseline of bench.py (TEST INFRASTRUCTURE: only bench.py's ``cpu_baseline`` leg runs it).

The reference's CPU path for one sweep point is three QuTiP 5 ``sesolve`` calls
(sweep_sea_detuning.py:694-702 -> dipolar_ensemble_with_rare.py:653-666), i.e. scipy ZVODE-Adams
on -iH psi with a CSR H at the sweep's tolerances (atol 1e-10, rtol 1e-9, nsteps 1e7, max_step
1e-5; sweep_sea_detuning.py:1247-1250), restated in ``propagate.zvode_trace``.  QuTiP itself is
absent (see propagate.py), so this times that restatement ("port").

Sample: detunings {0, 75, 150 kHz} x the 3 variants at N = 14 on the bench's 1 ms / 101-output
grid; each evolution integrates until its share of the budget is spent (at an output time) and is
extrapolated linearly in simulated time (ZVODE's work is linear in t: SURVEY.md P2).  The cost of
a point = the sum over its 3 variants; the sweep average = the mean over the 3 detunings (cost
grows with |delta| through ||H||).

  serial   one process, one core: the reference's real behaviour (a serial loop, :611)
  all      ``cores`` worker processes, one evolution each, all busy at once (the node's host
           cores; ``cores`` = the CPU share this process may use): the throughput of the
           multiprocessing sweep SURVEY.md §8(d) plans

    python -m oracle.cpu_bench --budget 20 --cores 16     # prints one JSON line

Run as its own process (bench.py starts it with subprocess before touching the GPU), so the
worker pool forks a process that never initialised a GPU.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

N_SEA = 13
T_FINAL = 1e-3
STEPS = 101
DELTAS = (0.0, 75_000.0, 150_000.0)


def one_evolution(job):
    """(delta, variant, budget_s) -> seconds for the whole 1 ms evolution (extrapolated)."""
    delta, variant, budget = job
    from oracle import propagate, reference_model as rm
    from quantumsimulations_amd.sweep import sweep_point_params
    p = sweep_point_params(N_SEA, delta, variant, T_FINAL, STEPS)
    H, obs, psi0, _ = rm.build(dataclasses.asdict(p))
    t = np.linspace(0.0, T_FINAL, STEPS)
    _, info = propagate.zvode_trace(H, psi0, t, obs, atol=1e-10, rtol=1e-9, nsteps=10_000_000,
                                    max_step=1e-5, time_budget_s=budget)
    frac = info["t_reached"] / T_FINAL
    return {"delta": delta, "variant": variant, "t_reached": info["t_reached"],
            "rhs": info["rhs"], "wall_s": info["wall_s"],
            "seconds_extrapolated": info["wall_s"] / max(frac, 1e-12)}


def point_seconds(rows):
    """Mean over detunings of the summed seconds of the 3 variants of a point."""
    per = {}
    for r in rows:
        per.setdefault(r["delta"], {}).setdefault(r["variant"], []).append(r["seconds_extrapolated"])
    return float(np.mean([sum(np.mean(v) for v in d.values()) for d in per.values()])), per


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=float, default=20.0, help="CPU seconds of the serial leg")
    ap.add_argument("--cores", type=int, default=0, help="workers of the all-core leg (0: all)")
    args = ap.parse_args(argv)
    from quantumsimulations_amd.sweep import VARIANTS
    host_cores = len(os.sched_getaffinity(0))
    cores = args.cores if args.cores > 0 else host_cores
    per_ev = args.budget / (len(DELTAS) * len(VARIANTS))
    jobs = [(d, v, per_ev) for d in DELTAS for v in VARIANTS]

    t0 = time.perf_counter()
    serial = [one_evolution(j) for j in jobs]
    serial_wall = time.perf_counter() - t0
    sec_serial, per_serial = point_seconds(serial)

    # all-core leg: every worker busy at once (jobs cycled so each of `cores` workers gets one)
    all_jobs = [jobs[i % len(jobs)] for i in range(max(cores, len(jobs)))]
    t1 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        loaded = pool.map(one_evolution, all_jobs, chunksize=1)
    all_wall = time.perf_counter() - t1
    sec_loaded, per_loaded = point_seconds(loaded)
    out = {
        "value": 3600.0 / sec_serial, "unit": "detuning-points/hour", "cores": 1, "kind": "port",
        "value_all_cores": cores * 3600.0 / sec_loaded, "cores_all": cores, "host_cores": host_cores,
        "sample": (f"ZVODE-Adams + scipy CSR (QuTiP-5 sesolve restated, oracle/propagate.py), atol 1e-10 "
                   f"rtol 1e-9, N=14, detunings {[d / 1e3 for d in DELTAS]} kHz x 3 variants on the "
                   f"1 ms / {STEPS}-output grid, each evolution run for ~{per_ev:.1f} s and extrapolated "
                   f"linearly in simulated time; point = sum of its 3 variants, averaged over the "
                   f"detunings; value: 1 core (serial, the reference's loop); value_all_cores: "
                   f"{cores} worker processes, one evolution each, all busy at once"),
        "seconds_per_point_serial": sec_serial,
        "seconds_per_point_loaded_core": sec_loaded,
        "per_delta_serial_s": {f"{d / 1e3:g}kHz": {v: float(np.mean(x)) for v, x in per.items()}
                               for d, per in per_serial.items()},
        "reached_us": [round(r["t_reached"] * 1e6, 1) for r in serial],
        "wall_s": {"serial": serial_wall, "all_cores": all_wall},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
