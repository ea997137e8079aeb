#!/usr/bin/env python3
"""Round-3 planning probe: per-term time of the persistent interval kernel on 12-bit tiles (the
tile of a four-tile N = 14 register) against 13-bit tiles.  One-tile registers only (no hand-off):
n = 12 (center_on at n_sea = 11, tile_bits 12: k_interval<12>, two workgroups per CU) and n = 13
(center_off at n_sea = 13: k_interval<13>), 256 and 512 problems, one launch of 2 outputs."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import sweep_point_params  # noqa: E402

t = np.linspace(0.0, 2e-5, 3)
for n_sea, variant, tb in ((11, "center_on", 12), (13, "center_off", 13)):
    for count in (256, 512):
        dets = np.linspace(0.0, 150e3, count)
        probs = [pb.build_problem(sweep_point_params(n_sea, float(d), variant, float(t[-1]), len(t)))
                 for d in dets]
        with Engine(0, tile_bits=tb) as eng:
            eng.set_option("streams", 1)
            for p in probs:
                eng.add(p)
            eng.evolve(t)
            best = None
            for _ in range(3):
                _, st = eng.evolve(t)
                ms = st["step_kernel_ms"] / max(st["timed_launches"], 1)
                best = ms if best is None else min(best, ms)
        print(json.dumps({"n": probs[0].n_qubits, "tile_bits": tb, "problems": count,
                          "mode": st["mode"], "max_degree": st["max_degree"],
                          "ms_per_launch": best, "us_per_term": best * 1e3 / st["max_degree"]}), flush=True)
