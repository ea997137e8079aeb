#!/usr/bin/env python3
"""Config 2 (one N = 12 center_on evolution, 2 ms / 201 outputs) through simulate_rare: wall time
per call for the engine modes (matrix = 1 default / 0 per-interval; in matrix mode also the
products' reduction in a separate launch, option symv_fused = 0), for rocprofv3 kernel traces of the
matrix mode's phases (column build, product chain, observables)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import dipolar_ensemble_with_rare as dse  # noqa: E402
from quantumsimulations_amd.sweep import sweep_point_params  # noqa: E402

p = sweep_point_params(11, 50e3, "center_on", 2e-3, 201)
for matrix, fused in ((1, 1), (1, 0), (1, 1), (0, 1)):
    eng = dse._engine(0)
    eng.set_option("matrix", matrix)
    eng.set_option("symv_fused", fused)
    dse.simulate_rare(p)
    ts = []
    for _ in range(5 if matrix else 3):
        t0 = time.perf_counter()
        dse.simulate_rare(p)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(f"matrix={matrix} symv_fused={fused}: wall ms {[round(x, 2) for x in ts]}", flush=True)
eng.set_option("matrix", 1)
eng.set_option("symv_fused", 1)
