#!/usr/bin/env python3
"""Spanning-register timings (dse_span.hip): JSON lines of wall and kernel time.

    python3 tools/probe_span.py lone [reps]     one N = 14 register per evolve (center_on and
                                                shell_off at 75 / 150 kHz), whole / span_tile 11 / 10
    python3 tools/probe_span.py sweep [reps]    the bench's 192 evolutions with default / span_tile 11 / 10
    python3 tools/probe_span.py shard [reps]    one GPU's share of the 64-point sweep on 8 GPUs
                                                (8 points = 24 evolutions), default / span_tile 11 / 10;
                                                SHARD_WORLD=W (default 8) and SHARD_RANK=r (default 0)
                                                select rank r's share of the W-GPU split
Grid: config 3's 1 ms / 101 outputs.  Kernel time = HIP events around every interval launch.

Ablation options (ablate, span_ablate, real_ablate) need a diagnostics build of the same ABI:
    DSE_EXTRA_FLAGS=-DDSE_DIAG python -m quantumsimulations_amd.build --out tools/bin/libdse_diag.so
    DSE_LIB=tools/bin/libdse_diag.so python3 tools/probe_span.py ...
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import VARIANTS, sweep_params, sweep_point_params  # noqa: E402

T = np.linspace(0.0, 1e-3, 101)


def setting(span):
    """'+'-joined tokens: '0' whole registers (span_tile 0), 'a' the automatic policy (default),
    'tL' option span_tile L, 'sS' option span S, 'rX' option real X (e.g. '0+r0': k_interval),
    'bB' option span_rb B (2^B amplitudes per thread), 'mM' option span_outputs M, 'pP' option
    span_partial P, 'cC' option span_chunks C, 'qL' option span_partial_tile L"""
    opts = {}
    for tok in str(span).split("+"):
        if tok == "0":
            opts["span_tile"] = 0
        elif tok == "a":
            opts["span_tile"] = -1
        else:
            opts[{"t": "span_tile", "s": "span", "r": "real", "b": "span_rb", "m": "span_outputs",
                  "p": "span_partial", "c": "span_chunks", "q": "span_partial_tile"}[tok[0]]] = int(tok[1:])
    return opts


def run(eng, probs, span, reps, label, **opts):
    eng.clear()
    for k, v in setting(span).items():
        eng.set_option(k, v)
    for k, v in opts.items():
        eng.set_option(k, v)
    for p in probs:
        eng.add(p)
    eng.evolve(T)  # warm-up (tables, allocations)
    walls, kms = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        obs, st = eng.evolve(T)
        walls.append((time.perf_counter() - t0) * 1e3)
        kms.append(st["step_kernel_ms"])
    eng.set_option("span", 0)
    eng.set_option("span_tile", -1)
    eng.set_option("real", 0)
    eng.set_option("span_rb", 0)
    eng.set_option("span_outputs", 4)
    eng.set_option("span_partial", 1)
    eng.set_option("span_chunks", 2)
    eng.set_option("span_partial_tile", 11)
    eng.clear()
    terms = st["h_applications"]
    rec = {"case": label, "span": span, "n_probs": len(probs), "wall_ms": min(walls),
           "wall_ms_all": [round(w, 2) for w in walls], "kernel_ms": min(kms),
           "span_problems": st["span_problems"], "max_degree": st["max_degree"],
           "launches": st["step_launches"], "h_applications": terms,
           "us_per_term_chain": 1e3 * min(kms) / max(1, st["max_degree"] * st["n_intervals"] /
                                                      max(1, st["outputs_per_launch"])),
           "fallbacks": st["handoff_fallbacks"], "real_problems": st["real_problems"], **opts}
    print(json.dumps(rec), flush=True)
    return obs


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "lone"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    spans = sys.argv[3].split("/") if len(sys.argv) > 3 else ["0", "t11", "t10"]
    with Engine(0) as eng:
        if what == "lone":
            for variant in ("center_on", "shell_off"):
                for d in (75e3, 150e3):
                    p = pb.build_problem(sweep_point_params(13, d, variant, T[-1], len(T)))
                    ref = None
                    for s in spans:
                        obs = run(eng, [p], s, reps, f"{variant}_{int(d / 1e3)}k")
                        if ref is None:
                            ref = obs
                        else:
                            print(json.dumps({"check": f"{variant}_{int(d / 1e3)}k", "span": s,
                                              "max_abs_diff_vs_span0": float(np.max(np.abs(obs - ref)))}), flush=True)
        elif what == "rablate":  # probe_span.py rablate <reps> - <mask/...>: k_real sections off (lone N=14)
            p = pb.build_problem(sweep_point_params(13, 150e3, "shell_off", T[-1], len(T)))
            masks = [int(m) for m in (sys.argv[4].split("/") if len(sys.argv) > 4 else ["0"])]
            for m in masks:
                run(eng, [p], "0", reps, f"shell_off_150k_real_ablate{m}", real_ablate=m)
            eng.set_option("real_ablate", 0)
        elif what == "ablate":  # probe_span.py ablate <reps> <setting> <mask/mask/...>: k_span sections off
            p = pb.build_problem(sweep_point_params(13, 150e3, "center_on", T[-1], len(T)))
            masks = [int(m) for m in (sys.argv[4].split("/") if len(sys.argv) > 4 else ["0"])]
            for m in masks:
                run(eng, [p], spans[0], reps, f"center_on_150k_ablate{m}", span_ablate=m)
            eng.set_option("span_ablate", 0)
        else:
            world = int(os.environ.get("SHARD_WORLD", "8"))
            n_pts = 64 if what == "sweep" else 64 // world
            dets = np.linspace(0.0, 150e3, 64)
            if what == "shard":  # rank r of W under the strong split: detunings j = r mod W
                dets = dets[int(os.environ.get("SHARD_RANK", "0"))::world]
            params = sweep_params(13, dets[:n_pts], T[-1], len(T))
            probs = [pb.build_problem(p) for p in params]
            ref = None
            for s in spans:
                obs = run(eng, probs, s, reps, what if what == "sweep" else
                          f"shard{world}_r{os.environ.get('SHARD_RANK', '0')}")
                if ref is None:
                    ref = obs
                else:
                    print(json.dumps({"check": what, "span": s,
                                      "max_abs_diff_vs_span0": float(np.max(np.abs(obs - ref)))}), flush=True)


if __name__ == "__main__":
    main()
