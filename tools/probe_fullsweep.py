#!/usr/bin/env python3
"""Diagnostic: the full-sweep dense point (bench.py full_sweep_dense) under engine options: the 3
variants of one detuning on the reference's 30 s / 20 000-output grid, evolved once per settings
string, wall time and the engine's eigensolver / dense times as one JSON line each.

    python3 tools/probe_fullsweep.py eig_streams=2 eig_streams=3,eig_impl=1 points=16 ...

points=K (not an engine option): K detunings of linspace(0, 150 kHz, K) in one evolve (3K
registers), as bench.py's full_sweep evolves the whole sweep.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params  # noqa: E402


def main():
    t_ref = np.linspace(0.0, 30.0, 20000)
    with Engine(0) as eng:
        for settings in sys.argv[1:] or [""]:
            opts = dict(kv.split("=") for kv in settings.replace("+", ",").split(",") if kv)
            npts = int(opts.pop("points", 0))
            dets = np.linspace(0.0, 150e3, npts) if npts else [50e3]
            probs = [pb.build_problem(sweep_point_params(13, float(d), v, 30.0, 20000)) for d in dets for v in VARIANTS]
            for k, v in opts.items():
                eng.set_option(k, float(v))
            eng.clear()
            for p in probs:
                eng.add(p)
            t0 = time.perf_counter()
            _, st = eng.evolve(t_ref)
            wall = time.perf_counter() - t0
            print(json.dumps({"settings": settings, "wall_s": wall, "s_per_point": wall / len(dets),
                              "dense_problems": st["dense_problems"],
                              "eig_ms": st["dense_eig_ms"], "dense_ms": st["dense_ms"]}), flush=True)


if __name__ == "__main__":
    main()
