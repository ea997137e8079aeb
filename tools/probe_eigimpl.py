#!/usr/bin/env python3
"""Dense engine on the reference grid (30 s / 20 000 outputs), one N = 14 sweep point (3 variants:
two registers of 2^14 amplitudes and one of 2^13): wall time per evolve by eigensolver (option
eig_impl: 0 rocSOLVER dsyevd, 1 the half-matrix tridiagonalisation) and solver streams, and the
largest output difference against the first configuration.
    probe_eigimpl.py impl:streams [impl:streams ...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params  # noqa: E402

cfgs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(0, 2), (1, 2), (0, 2), (1, 2), (1, 1), (1, 3)]
t = np.linspace(0.0, 30.0, 20000)
with Engine(0) as eng:
    for v in VARIANTS:
        eng.add(pb.build_problem(sweep_point_params(13, 75e3, v, 30.0, 20000)))
    eng.evolve(t)
    ref = None
    for impl, es in cfgs:
        eng.set_option("eig_impl", impl)
        eng.set_option("eig_streams", es)
        t0 = time.perf_counter()
        obs, st = eng.evolve(t)
        wall = time.perf_counter() - t0
        if ref is None:
            ref = obs.copy()
        print(json.dumps({"eig_impl": impl, "eig_streams": es, "wall_s": wall, "eig_ms": st["dense_eig_ms"],
                          "dense_ms": st["dense_ms"], "max_diff_vs_first": float(np.max(np.abs(obs - ref)))}),
              flush=True)
