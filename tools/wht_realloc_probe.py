#!/usr/bin/env python3
"""Is the N = 30 engine's fast/slow mode per process or per allocation?  One process, several
engine contexts in turn (each allocates its own 80 GiB and frees it), kernel ms per H application
of each (the bench_large measurement)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import sweep_point_params  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    opts = dict(kv.split("=") for kv in sys.argv[2:])  # engine options, e.g. wht_skew=4352
    t = np.linspace(0.0, 1e-5, 3)
    prob = pb.build_problem(sweep_point_params(29, 50e3, "center_on", float(t[-1]), len(t)))
    for i in range(reps):
        with Engine(0) as eng:
            for k, v in opts.items():
                eng.set_option(k, float(v))
            eng.add(prob)
            eng.evolve(t)
            t0 = time.perf_counter()
            _, st = eng.evolve(t)
            wall = time.perf_counter() - t0
        print(json.dumps({"context": i, "opts": opts, "wall_ms_per_h": 1e3 * wall / st["h_applications"],
                          "h_applications": st["h_applications"]}), flush=True)


if __name__ == "__main__":
    main()
