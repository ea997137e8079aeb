#!/usr/bin/env python3
"""Config 5: one large register on one GPU.

    python tools/bench_large.py [--n-sea 29] [--t-final 1e-5] [--steps 11] [--delta 50e3]

N = n_sea + 1 qubits, center_on (rare driven), the sweep's physical constants.  Evolves the
reference grid with the streaming Chebyshev kernels (2^13-amplitude tiles, cross-tile terms
through L2/HBM) and prints one JSON line: ms per H application, the step kernel's algorithmic
GB/s and FP64 rate against the MI355X roofline, the observables at t_final and the norm drift.
"""
from __future__ import annotations

import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-sea", type=int, default=29)
    ap.add_argument("--t-final", type=float, default=1e-5)
    ap.add_argument("--steps", type=int, default=11)
    ap.add_argument("--delta", type=float, default=50e3)
    ap.add_argument("--variant", default="center_on")
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--wht", type=int, default=1, help="Walsh-Hadamard engine (1) or step kernels (0)")
    ap.add_argument("--wht-group-bits", type=int, default=0)
    ap.add_argument("--wht-tile-bits", type=int, default=0)
    ap.add_argument("--wht-persist", type=int, default=0, help="option wht_persist (bit 1: persistent MID)")
    ap.add_argument("--wht-contiguous", type=int, default=-1, help="option wht_contiguous; -1 the default")
    ap.add_argument("--wht-fuse", type=int, default=-1, help="option wht_fuse (FINAL + next FIRST); -1 the default")
    ap.add_argument("--wht-mid-inpage", type=int, default=-1,
                    help="option wht_mid_inpage (MID group's high bits below the 2-MiB page); -1 the default")
    ap.add_argument("--wht-half", type=int, default=-1,
                    help="option wht_half (bits: 1 FIRST, 2 FWD/INV, 4 MID); -1 the library default")
    a = ap.parse_args()
    p = sweep_point_params(a.n_sea, a.delta, a.variant, a.t_final, a.steps)
    t0 = time.perf_counter()
    prob = pb.build_problem(p)
    t_build = time.perf_counter() - t0
    t = np.linspace(0.0, a.t_final, a.steps)
    with Engine(0) as eng:
        eng.set_option("streams", a.streams)
        eng.set_option("wht", a.wht)
        eng.set_option("wht_group_bits", a.wht_group_bits)
        eng.set_option("wht_tile_bits", a.wht_tile_bits)
        eng.set_option("wht_persist", a.wht_persist)
        if a.wht_half >= 0:
            eng.set_option("wht_half", a.wht_half)
        if a.wht_contiguous >= 0:
            eng.set_option("wht_contiguous", a.wht_contiguous)
        if a.wht_fuse >= 0:
            eng.set_option("wht_fuse", a.wht_fuse)
        if a.wht_mid_inpage >= 0:
            eng.set_option("wht_mid_inpage", a.wht_mid_inpage)
        eng.add(prob)
        t0 = time.perf_counter()
        eng.evolve(t)                  # first call: device allocation, tables, code objects
        t_setup = time.perf_counter() - t0
        t0 = time.perf_counter()
        obs, st = eng.evolve(t)
        wall = time.perf_counter() - t0
    n = prob.n_qubits
    h_apps = st["h_applications"]
    k_ms, k_launch = st["step_kernel_ms"], max(st["timed_launches"], 1)
    gbs = st["timed_bytes"] / (k_ms * 1e-3) / 1e9 if k_ms > 0 else None
    tfl = st["timed_flops"] / (k_ms * 1e-3) / 1e12 if k_ms > 0 else None
    norm = obs[0, 6]
    print(json.dumps({
        "config": f"config 5: N={n} ({a.variant}, delta={a.delta:g} Hz), t_final={a.t_final}, {a.steps} outputs",
        "qubits_engine": n, "amplitudes": 1 << n, "state_GiB": (1 << n) * 16 / 2**30,
        "host_table_build_s": t_build, "first_evolve_s": t_setup, "wall_s": wall, "h_applications": h_apps,
        "ms_per_h_application": wall / max(h_apps, 1) * 1e3,
        "step_kernel_avg_us": k_ms / k_launch * 1e3,
        "step_kernel_gbs_algorithmic": gbs, "hbm_peak_gbs": 8000.0,
        "step_kernel_fp64_tflops": tfl, "fp64_peak_tflops": 78.6,
        "mode": st["mode"], "wht_group_bits": a.wht_group_bits, "wht_tile_bits": a.wht_tile_bits,
        "wht_persist": a.wht_persist, "wht_half": a.wht_half, "wht_mid_inpage": a.wht_mid_inpage, "wht_fuse": a.wht_fuse, "wht_contiguous": a.wht_contiguous,
        "max_degree": st["max_degree"], "tile_bits": st["tile_bits"],
        "norm_drift": float(np.max(np.abs(norm - 1.0))),
        "obs_t_final": {k: float(obs[0, i, -1]) for i, k in enumerate(pb.OBS_NAMES)},
    }), flush=True)


if __name__ == "__main__":
    main()
