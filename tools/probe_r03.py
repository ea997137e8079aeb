#!/usr/bin/env python3
"""Round-3 planning probe (one GPU call): timings that decide the round's work.

* config 2: one N = 12 center_on evolution (50 kHz, 2 ms / 201 outputs) through the drop-in
  simulate_rare, wall ms and the engine's counters;
* the unmodified caller's pattern at N = 14: three serial simulate_rare calls (1 ms / 101);
* the reference's default workload on k_small: n_sea = 6, 13 detunings x 3 variants on the
  30 s / 20 000-output grid, first K intervals;
* dense symmetric eigensolver times (torch.linalg.eigh on the device) for n = 128 (batched),
  1024, 4096, 8192, 16384.
Prints one JSON object per line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import dipolar_ensemble_with_rare as dse  # noqa: E402
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


what = sys.argv[1] if len(sys.argv) > 1 else "all"

if what in ("all", "config2"):
    p = sweep_point_params(11, 50e3, "center_on", 2e-3, 201)
    dse.simulate_rare(p)
    walls = []
    for _ in range(3):
        t0 = time.perf_counter()
        dse.simulate_rare(p)
        walls.append((time.perf_counter() - t0) * 1e3)
    prob = pb.build_problem(p)
    with Engine(0) as eng:
        eng.add(prob)
        t = pb.time_grid(p)
        eng.evolve(t)
        _, st = eng.evolve(t)
    emit(case="config2", wall_ms=walls, stats=st)

if what in ("all", "n14serial"):
    ps = [sweep_point_params(13, 50e3, v, 1e-3, 101) for v in VARIANTS]
    for q in ps:
        dse.simulate_rare(q)
    walls = []
    for _ in range(2):
        t0 = time.perf_counter()
        for q in ps:
            dse.simulate_rare(q)
        walls.append((time.perf_counter() - t0) * 1e3)
    emit(case="n14_three_serial", wall_ms=walls)

if what in ("all", "refdefault"):
    dets = np.linspace(0.0, 150e3, 13)
    t_full = np.linspace(0.0, 30.0, 20000)
    for K in (4, 20):
        t = t_full[:K + 1]
        probs = [pb.build_problem(sweep_point_params(6, float(d), v, 30.0, 20000)) for d in dets for v in VARIANTS]
        with Engine(0) as eng:
            for q in probs:
                eng.add(q)
            eng.evolve(t[:2])
            t0 = time.perf_counter()
            _, st = eng.evolve(t)
            wall = time.perf_counter() - t0
        emit(case="refdefault_k_small", intervals=K, wall_s=wall, s_per_interval=wall / K,
             full_extrapolated_s=wall / K * 19999, stats=st)

if what in ("all", "eigh"):
    import torch
    dev = torch.device("cuda:0")
    emit(case="linalg_backend", lib=str(torch.backends.cuda.preferred_linalg_library()))
    rng = np.random.default_rng(1)
    for n, batch in ((128, 39), (1024, 1), (4096, 1), (8192, 1), (16384, 1)):
        a = torch.tensor(rng.standard_normal((batch, n, n)), dtype=torch.float64, device=dev)
        a = a + a.transpose(1, 2)
        if batch == 1:
            a = a[0]
        reps = 3 if n <= 4096 else 1
        torch.linalg.eigh(a)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            w, v = torch.linalg.eigh(a)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        emit(case="eigh", n=n, batch=batch, s=ts)
        del a, w, v
        torch.cuda.empty_cache()
