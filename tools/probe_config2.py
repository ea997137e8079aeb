#!/usr/bin/env python3
"""Config 2 (one N = 12 center_on evolution, 2 ms / 201 outputs) through simulate_rare: wall time
per call for the engine modes (matrix = 1 default / 0 per-interval), for rocprofv3 kernel traces
of the matrix mode's phases (column build, zgemv chain, observables)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import dipolar_ensemble_with_rare as dse  # noqa: E402
from quantumsimulations_amd.sweep import sweep_point_params  # noqa: E402

p = sweep_point_params(11, 50e3, "center_on", 2e-3, 201)
for matrix in (1, 0):
    eng = dse._engine(0)
    eng.set_option("matrix", matrix)
    dse.simulate_rare(p)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        dse.simulate_rare(p)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"matrix={matrix}: wall ms {[round(x, 2) for x in ts]}", flush=True)
