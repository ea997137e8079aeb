"""CPU baseline of bench.py (TEST INFRASTRUCTURE: only bench.py's ``cpu_baseline`` leg runs it).

The reference's CPU path for one sweep point is three QuTiP 5 ``sesolve`` calls
(sweep_sea_detuning.py:694-702 -> dipolar_ensemble_with_rare.py:653-666), i.e. scipy ZVODE-Adams
on -iH psi with a CSR H at the sweep's tolerances (atol 1e-10, rtol 1e-9, nsteps 1e7, max_step
1e-5; sweep_sea_detuning.py:1247-1250), restated in ``propagate.zvode_trace``.  QuTiP itself is
absent (see propagate.py), so this times that restatement ("port").

Sample: detunings {0, 75, 150 kHz} x the 3 variants at N = 14 on the bench's 1 ms / 101-output
grid.  Every sampled evolution integrates the first quarter of the grid (250 us, 25 outputs) and
is extrapolated linearly in simulated time (ZVODE's work is linear in t: SURVEY.md P2).  The cost
of a point = the sum over its 3 variants; the sweep average = the mean over the 3 detunings (cost
grows with |delta| through ||H||).

  serial   one process, one core: the reference's real behaviour (a serial loop, :611).  The
           three variants at 75 kHz run serially; the sweep average scales their point cost by
           the all-core leg's detuning profile (mean over detunings / 75 kHz point)
  all      ``cores`` worker processes, one evolution each, all nine busy at once (``cores`` = the
           CPU share this process may use; 16 on the GPU box).  The node-wide figure is that
           measured per-loaded-core rate times the machine's core count (labelled an estimate:
           the rest of the node is not this job's)

    python -m oracle.cpu_bench --cores 16     # prints one JSON line

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
    """(delta, variant, fraction) -> seconds for the whole 1 ms evolution, extrapolated from the
    first ``fraction`` of the grid (integrated to its last output time)."""
    delta, variant, fraction = job
    from oracle import propagate, reference_model as rm
    from quantumsimulations_amd.sweep import sweep_point_params
    p = sweep_point_params(N_SEA, delta, variant, T_FINAL, STEPS)
    H, obs, psi0, _ = rm.build(dataclasses.asdict(p))
    t = np.linspace(0.0, T_FINAL, STEPS)
    t = t[:max(2, int(round(fraction * (STEPS - 1))) + 1)]
    _, info = propagate.zvode_trace(H, psi0, t, obs, atol=1e-10, rtol=1e-9, nsteps=10_000_000,
                                    max_step=1e-5)
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
    ap.add_argument("--fraction", type=float, default=0.25, help="share of the 1 ms grid integrated")
    ap.add_argument("--cores", type=int, default=0, help="workers of the all-core leg (0: all)")
    ap.add_argument("--budget", type=float, default=None, help="(ignored; older interface)")
    args = ap.parse_args(argv)
    from quantumsimulations_amd.sweep import VARIANTS
    host_cores = os.cpu_count() or 1
    share = len(os.sched_getaffinity(0))
    cores = args.cores if args.cores > 0 else share
    jobs = [(d, v, args.fraction) for d in DELTAS for v in VARIANTS]

    t0 = time.perf_counter()
    mid = DELTAS[len(DELTAS) // 2]
    serial = [one_evolution((mid, v, args.fraction)) for v in VARIANTS]
    serial_wall = time.perf_counter() - t0
    sec_serial_mid, _ = point_seconds(serial)

    # all-core leg: every worker busy at once (jobs cycled so each of `cores` workers gets one)
    all_jobs = [jobs[i % len(jobs)] for i in range(max(cores, len(jobs)))]
    t1 = time.perf_counter()
    with mp.get_context("fork").Pool(cores) as pool:
        loaded = pool.map(one_evolution, all_jobs, chunksize=1)
    all_wall = time.perf_counter() - t1
    sec_loaded, per_loaded = point_seconds(loaded)
    sec_loaded_mid = sum(float(np.mean(x)) for x in per_loaded[mid].values())
    sec_serial = sec_serial_mid * sec_loaded / sec_loaded_mid   # sweep average, 1 core
    out = {
        "value": 3600.0 / sec_serial, "unit": "detuning-points/hour", "cores": 1, "kind": "port",
        "value_all_cores": cores * 3600.0 / sec_loaded, "cores_all": cores,
        "value_full_node_estimate": host_cores * 3600.0 / sec_loaded, "host_cores": host_cores,
        "sample": (f"ZVODE-Adams + scipy CSR (QuTiP-5 sesolve restated, oracle/propagate.py), atol 1e-10 "
                   f"rtol 1e-9, N=14, detunings {[d / 1e3 for d in DELTAS]} kHz x 3 variants on the "
                   f"1 ms / {STEPS}-output grid, each evolution integrated over the first "
                   f"{args.fraction:.0%} of the grid and extrapolated linearly in simulated time; point = "
                   f"sum of its 3 variants, averaged over the detunings; value: 1 core (the reference's "
                   f"serial loop; the 3 variants at {mid / 1e3:g} kHz timed serially, scaled to the sweep "
                   f"average by the all-core leg's detuning profile); value_all_cores: {cores} worker "
                   f"processes (this job's CPU share), one evolution each, all busy at once; "
                   f"value_full_node_estimate: that loaded-core rate x the machine's {host_cores} cores "
                   f"(not run: the rest of the node is not this job's)"),
        "seconds_per_point_serial": sec_serial,
        "seconds_per_point_serial_at_mid_delta": sec_serial_mid,
        "seconds_per_point_loaded_core": sec_loaded,
        "per_delta_loaded_s": {f"{d / 1e3:g}kHz": {v: float(np.mean(x)) for v, x in per.items()}
                               for d, per in per_loaded.items()},
        "reached_us": sorted({round(r["t_reached"] * 1e6, 1) for r in serial + loaded}),
        "wall_s": {"serial": serial_wall, "all_cores": all_wall},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
