#!/usr/bin/env python3
"""One N = 14 evolution alone in a context (the reference's serial simulate_rare pattern, 1 ms / 101
outputs): wall ms per evolve on the persistent 2-tile kernel (default) against the streaming step
kernels with smaller tiles over the chip (option persistent = 0, tile_bits = T), and max |d obs|."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import sweep_point_params  # noqa: E402

t = np.linspace(0.0, 1e-3, 101)
variant = sys.argv[1] if len(sys.argv) > 1 else "center_on"
cfgs = [("persistent", {})] + [(f"stream_L{L}", {"persistent": 0, "tile_bits": L}) for L in (13, 12, 11, 10, 9, 8)]
ref = None
with Engine(0) as eng:
    for name, opts in cfgs:
        for k, v in opts.items():
            eng.set_option(k, v)
        ts = []
        for rep in range(3):
            eng.clear()
            eng.add(pb.build_problem(sweep_point_params(13, 75e3, variant, 1e-3, 101)))
            t0 = time.perf_counter()
            obs, st = eng.evolve(t)
            ts.append((time.perf_counter() - t0) * 1e3)
        if ref is None:
            ref = obs.copy()
        print(json.dumps({"config": name, "wall_ms": [round(x, 2) for x in ts], "mode": st["mode"],
                          "h_applications": st["h_applications"],
                          "max_diff": float(np.max(np.abs(obs - ref)))}), flush=True)
        eng.set_option("persistent", 1)
        eng.set_option("tile_bits", 13)
