#!/usr/bin/env python3
"""Config 5 correctness at full size on one MI355X (N = 30, center_on, 50 kHz; 16 GiB per state
vector) -- the checks a multi-GPU run of the partitioned register rests on:

  1. Walsh-Hadamard engine (the default) vs the per-term step kernels (wht = 0) over the first
     outputs (t = 0, 0.2, 0.4 us): all seven observables
  2. the register as 8 loopback shards (top 3 qubits global, index-swap exchange between shards
     around the MID pass: the data movement of the 8-GPU run, as device copies) vs unsharded, over
     the bench's 5 us / 6-output window: observables and the exact invariants (norm, energy)

    python tools/check_config5_n30.py > profiles/r02/config5_n30_check.json
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import sweep_point_params  # noqa: E402


def diag_energy(prob) -> float:
    x = prob.psi0_index
    s = np.array([0.5 - ((x >> b) & 1) for b in range(prob.n_qubits)])
    return float(prob.shift + prob.field @ s + np.sum(np.triu(prob.zz, 1) * np.outer(s, s)))


def main():
    n_sea = int(os.environ.get("N_SEA", "29"))
    prob = pb.build_problem(sweep_point_params(n_sea, 50e3, "center_on", 5e-6, 6))
    e0 = diag_energy(prob)
    out = {"config": f"config 5: N={prob.n_qubits} center_on 50 kHz", "energy_t0": e0}
    t_short = np.linspace(0.0, 4e-7, 3)
    t_long = np.linspace(0.0, 5e-6, 6)
    with Engine(0) as eng:
        res = {}
        for wht in (1, 0):
            eng.clear()
            eng.set_option("wht", wht)
            eng.add(prob)
            t0 = time.perf_counter()
            res[wht], st = eng.evolve(t_short)
            out[f"short_wht{wht}_s"] = time.perf_counter() - t0
            out[f"short_wht{wht}_mode"] = st["mode"]
            print(f"short window wht={wht}: {out[f'short_wht{wht}_s']:.1f} s", file=sys.stderr, flush=True)
        eng.set_option("wht", 1)
        out["wht_vs_step_max_abs_diff"] = float(np.max(np.abs(res[1] - res[0])))
        runs = {}
        for name in ("unsharded", "sharded8"):
            eng.clear()
            pid = eng.add(prob) if name == "unsharded" else eng.add_sharded(prob, 3)
            t0 = time.perf_counter()
            obs, st = eng.evolve(t_long)
            wall = time.perf_counter() - t0
            e, n2 = eng.energy(pid)
            runs[name] = obs[pid]
            out[name] = {"wall_s": wall, "mode": st["mode"], "h_applications": st["h_applications"],
                         "energy_rel_error": abs(e - e0) / abs(e0), "norm2": n2,
                         "max_norm_error": float(np.max(np.abs(obs[pid, 6] - 1.0)))}
            print(f"{name}: {wall:.1f} s", file=sys.stderr, flush=True)
        eng.clear()
    out["sharded_vs_unsharded_max_abs_diff"] = float(np.max(np.abs(runs["sharded8"] - runs["unsharded"])))
    out["ok"] = bool(out["wht_vs_step_max_abs_diff"] < 1e-11
                     and out["sharded_vs_unsharded_max_abs_diff"] < 1e-12
                     and all(out[k]["energy_rel_error"] < 1e-11 and out[k]["max_norm_error"] < 1e-12
                             for k in ("unsharded", "sharded8")))
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
