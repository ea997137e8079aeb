#!/usr/bin/env python3
"""The reference's own default run end to end through the drop-in sweep driver
(sweep_sea_detuning.py:1201-1252: Ga/Al at 3 T, f1A = 50 kHz, 13 detunings in [0, 150 kHz],
n_sea = 6, t_final = 30 s, 20 000 outputs, 3 variants per point): evolutions (the dense engine by
libdse's cost model), per-point metrics and the output tree (npz / json), with --report the
figures too.  Prints one JSON line with the phase timings."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantumsimulations_amd.sweep_runner import run_sweep_sea_detuning  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--report", default="none", choices=("none", "png", "full"))
a = ap.parse_args()
gamma_sea, gamma_rare, b0, f1a = 8.1812e7, 6.976e7, 3.0, 50_000.0
kw = dict(f_Az=gamma_sea * b0 / (2 * np.pi), f1A=f1a, target_sea_detuning=f1a, gamma_sea=gamma_sea,
          gamma_rare=gamma_rare, sea_detunings_Hz=np.linspace(0.0, 3.0 * f1a, 13), n_sea=6,
          t_final=30.0, steps=20000, phi_sea=np.pi / 2, phi_rare=np.pi / 2, is_spin_three_half=False,
          solver_atol=1e-10, solver_rtol=1e-9, solver_nsteps=10_000_000, solver_max_step=1e-5,
          coarse_window=100, devices=[0], verbose=False)
with tempfile.TemporaryDirectory() as tmp:
    run_sweep_sea_detuning(out_root=tmp, report="none", **kw)   # warm-up (contexts, libraries)
    tm = {}
    t0 = time.perf_counter()
    base = run_sweep_sea_detuning(out_root=tmp + "/timed", report=a.report, timings=tm, **kw)
    wall = time.perf_counter() - t0
    pts = sorted(d for d in os.listdir(base) if d.startswith("delta_"))
    z = np.load(os.path.join(base, pts[-1], "time_and_obs_center_on.npz"), allow_pickle=False)
    print(json.dumps({"workload": "reference __main__ (sweep_sea_detuning.py:1201-1252): N=7, 13 detunings x "
                                  "3 variants, t_final 30 s, 20000 outputs, through run_sweep_sea_detuning",
                      "report": a.report, "wall_s": wall, "timings": tm, "points": len(pts),
                      "points_per_hour": len(pts) * 3600.0 / wall,
                      "samples_per_trace": int(z["t"].shape[0]),
                      "max_norm_error_last_point": float(np.max(np.abs(z["state_norm"] - 1.0)))}), flush=True)
