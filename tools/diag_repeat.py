#!/usr/bin/env python3
"""Repeatability of the persistent path on the config-3 points: the same evolve several times in one
context (same allocations), under option variants given as name=value pairs."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params  # noqa: E402

t = np.linspace(0.0, 2e-4, 21)
probs = [pb.build_problem(sweep_point_params(13, float(d), v, float(t[-1]), len(t)))
         for v in VARIANTS for d in (0, 75000, 150000)]
variants = [a.split(",") for a in sys.argv[1:]] or [[""]]
with Engine(0) as eng:
    for var in variants:
        opts = dict(kv.split("=") for kv in var if kv)
        eng.clear()
        for k, v in opts.items():
            eng.set_option(k, float(v))
        for p in probs:
            eng.add(p)
        runs = [eng.evolve(t)[0] for _ in range(4)]
        d = [float(np.max(np.abs(r - runs[0]))) for r in runs[1:]]
        per = [float(np.max(np.abs(runs[1][i] - runs[0][i]))) for i in range(len(probs))]
        print(json.dumps({"opts": opts, "maxdiff_vs_first": d, "per_problem": [f"{x:.0e}" for x in per]}), flush=True)
        for k in opts:
            eng.set_option(k, {"coresident": 0, "xcd_pairs": 1, "outputs_per_launch": 2, "spin_limit": 1 << 22}.get(k, 0))
