#!/usr/bin/env python3
"""Diagnostic: time the Chebyshev step kernel on the bench workload with kernel sections ablated.

    python tools/probe_step.py [--tile-bits 13] [--reps 20]

Prints one JSON line per configuration (mean launch time, GB/s of the algorithmic bytes).
Ablated runs compute wrong numbers on purpose; this never touches parity.

Ablation options (ablate, span_ablate, real_ablate) need a diagnostics build of the same ABI:
    DSE_EXTRA_FLAGS=-DDSE_DIAG python -m quantumsimulations_amd.build --out tools/bin/libdse_diag.so
    DSE_LIB=tools/bin/libdse_diag.so python3 tools/probe_step.py ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import sweep_params  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tile-bits", type=int, default=13)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n-sea", type=int, default=13)
    ap.add_argument("--n-det", type=int, default=64)
    ap.add_argument("--only", default=None, help="run a single named configuration")
    args = ap.parse_args()
    params = sweep_params(args.n_sea, np.linspace(0.0, 150e3, args.n_det), 1e-3, 101)
    eng = Engine(0, tile_bits=args.tile_bits)
    for p in params:
        eng.add(pb.build_problem(p))
    t = np.linspace(0.0, 1e-5, 2)
    configs = [("full", 0, 0), ("one_round_256", 0, 256), ("no_sweeps", 1, 0), ("no_tt_pairs", 2, 0),
               ("no_cross_tile", 4, 0), ("no_epilogue_reads", 8, 0), ("no_zz_table", 16, 0),
               ("no_tile_load", 32, 0), ("compute_only", 8 | 16 | 32 | 4, 0),
               ("memory_only", 1 | 2 | 4, 0), ("memory_only_256", 1 | 2 | 4, 256)]
    for name, mask, items in configs:
        if args.only and name != args.only:
            continue
        eng.set_option("ablate", 0)
        eng.set_option("probe_items", 0)
        eng.evolve(t)                     # coefficients + valid buffers
        eng.set_option("ablate", mask)
        eng.set_option("probe_items", items)
        eng.time_step_kernel(2)           # warm
        eng.set_option("ablate", 0)
        eng.evolve(t)
        eng.set_option("ablate", mask)
        ms, by = eng.time_step_kernel(args.reps)
        print(json.dumps({"config": name, "ablate": mask, "items": items or "all", "ms": ms,
                          "gbs_algorithmic": by / (ms * 1e-3) / 1e9}), flush=True)
    eng.set_option("ablate", 0)
    eng.close()


if __name__ == "__main__":
    main()
