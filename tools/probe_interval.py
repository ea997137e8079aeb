#!/usr/bin/env python3
"""Diagnostic: time the persistent interval kernel on the bench workload with sections ablated.

    python tools/probe_interval.py

One output interval (dt = 1e-5 s) of the 64-point N = 14 sweep per configuration; prints the
HIP-event time of each lane's k_interval launch.  Ablated runs compute wrong numbers on purpose.

Ablation options (ablate, span_ablate, real_ablate) need a diagnostics build of the same ABI:
    DSE_EXTRA_FLAGS=-DDSE_DIAG python -m quantumsimulations_amd.build --out tools/bin/libdse_diag.so
    DSE_LIB=tools/bin/libdse_diag.so python3 tools/probe_interval.py ...
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import sweep_params  # noqa: E402


def keep(p, which):
    if which == "all":
        return True
    if which in ("pairs", "singles"):
        return (which == "pairs") == (p.n_qubits == 14)
    # "center_on" / "shell_off": the 2-tile problems of one variant (raw / generated hand-off)
    return p.n_qubits == 14 and p.meta.get("_v") == which


def run(eng, probs, t, mask, which):
    eng.clear()
    for p in probs:
        if keep(p, which):
            eng.add(p)
    eng.set_option("ablate", 0)
    eng.evolve(t)
    eng.set_option("ablate", mask)
    best = None
    for _ in range(3):
        _, st = eng.evolve(t)
        ms = st["step_kernel_ms"] / max(st["timed_launches"], 1)
        best = ms if best is None else min(best, ms)
    eng.set_option("ablate", 0)
    return best, st


def main():
    params = sweep_params(13, np.linspace(0.0, 150e3, 64), 1e-3, 101)
    probs = []
    for p in params:
        pr = pb.build_problem(p)
        pr.meta["_v"] = "center_on" if (p.is_center_rare and pr.rare_bit >= 0) else (
            "center_off" if p.is_center_rare else "shell_off")
        probs.append(pr)
    sets = sys.argv[1].split(",") if len(sys.argv) > 1 else ["pairs", "singles", "all"]
    t = np.linspace(0.0, 1e-5, 2)
    eng = Engine(0, tile_bits=13)
    eng.set_option("streams", 1)
    for which in sets:
        for name, mask in (("full", 0), ("no_publish", 64), ("no_wait_read", 128),
                           ("no_exchange", 64 | 128), ("no_acc", 256), ("no_tile_terms", 512),
                           ("exchange_only", 256 | 512), ("no_register_terms", 4)):
            if which in ("singles", "all") and mask & (64 | 128):
                continue
            ms, st = run(eng, probs, t, mask, which)
            print(json.dumps({"set": which, "config": name, "ablate": mask, "ms_per_launch": ms,
                              "max_degree": st["max_degree"], "us_per_term": ms * 1e3 / st["max_degree"]}),
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
