#!/usr/bin/env python3
"""The bench's sweep (N = 14, 64 detunings x 3 variants, 1 ms / 101 outputs) evolved once with the
library DSE_LIB points to; observables saved to <out.npy> for a bitwise comparison of two builds."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import VARIANTS, sweep_point_params  # noqa: E402

t = np.linspace(0.0, 1e-3, 101)
with Engine(0) as eng:
    for d in np.linspace(0.0, 150e3, 64):
        for v in VARIANTS:
            eng.add(pb.build_problem(sweep_point_params(13, float(d), v, 1e-3, 101)))
    obs, st = eng.evolve(t)
np.save(sys.argv[1], obs)
print(sys.argv[1], obs.shape, st["mode"])
