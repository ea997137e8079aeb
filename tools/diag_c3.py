#!/usr/bin/env python3
"""Config-3 diagnostic: the production N = 14 sweep points vs the reference-H fixture for
outputs_per_launch 2 and 1 and the streaming kernels, each evolve twice (bitwise repeatability)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params  # noqa: E402

OBS = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")
g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "hpsi_traces_n14.npz"))
t = g["t"]
keys, probs = [], []
for v in VARIANTS:
    for d in (0, 75000, 150000):
        keys.append(f"{v}_{d}")
        probs.append(pb.build_problem(sweep_point_params(13, float(d), v, float(t[-1]), len(t))))
with Engine(0) as eng:
    runs_cfg = [("M2", {"outputs_per_launch": 2}), ("M1", {"outputs_per_launch": 1}),
                ("stream", {"persistent": 0, "outputs_per_launch": 2})]
    if len(sys.argv) > 1 and sys.argv[1] == "dbg":  # diagnostics switches of the runtime, M = 2
        runs_cfg = [(f"dbg{d}", {"outputs_per_launch": 2, "dbg": d}) for d in (0, 1, 2, 4, 7)]
    for name, opts in runs_cfg:
        runs = []
        for rep in range(2):
            eng.clear()
            for k, v in opts.items():
                eng.set_option(k, v)
            for p in probs:
                eng.add(p)
            obs, st = eng.evolve(t)
            runs.append(obs)
            eng.set_option("persistent", 1)
            eng.set_option("outputs_per_launch", 2)
            eng.set_option("dbg", 0)
        err = {k: max(float(np.max(np.abs(runs[0][i, j] - g[f"{k}_{o}"]))) for j, o in enumerate(OBS))
               for i, k in enumerate(keys)}
        worst_t = {k: int(np.argmax(np.max(np.abs(runs[0][i, :6] - np.stack([g[f"{k}_{o}"] for o in OBS])), axis=0)))
                   for i, k in enumerate(keys)}
        print(json.dumps({"run": name, "mode": st["mode"], "M": st["outputs_per_launch"],
                          "repeat_bitwise": bool(np.array_equal(runs[0], runs[1])),
                          "repeat_maxdiff": float(np.max(np.abs(runs[0] - runs[1]))),
                          "err": {k: f"{e:.1e}" for k, e in err.items()}, "worst_t_index": worst_t}), flush=True)
