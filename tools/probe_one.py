#!/usr/bin/env python3
"""Diagnostic driver for counter collection: one output interval of the N = 14 sweep set
("singles" = center_off 1-tile problems, "pairs" = 2-tile problems, "all"), evolved 3 times,
with engine options given as k=v (e.g. real=0,span_tile=0 for k_interval; the defaults pick k_real
or k_span).

    rocprofv3 --pmc SQ_WAVES ... -- python3 tools/probe_one.py singles real=0,span_tile=0
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from quantumsimulations_amd import problem as pb  # noqa: E402
from quantumsimulations_amd.engine import Engine  # noqa: E402
from quantumsimulations_amd.sweep import sweep_params  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "singles"
    params = sweep_params(13, np.linspace(0.0, 150e3, 64), 1e-3, 101)
    probs = [pb.build_problem(p) for p in params]
    t = np.linspace(0.0, 1e-5, 2)
    with Engine(0, tile_bits=13) as eng:
        eng.set_option("streams", 1)
        for kv in ",".join(sys.argv[2:]).split(",") if len(sys.argv) > 2 else []:
            k, v = kv.split("=")
            eng.set_option(k, float(v))
        for p in probs:
            if which == "all" or (which == "pairs") == (p.n_qubits == 14):
                eng.add(p)
        for _ in range(3):
            _, st = eng.evolve(t)
        print(which, st["max_degree"], st["step_kernel_ms"] / max(st["timed_launches"], 1),
              "real", st["real_problems"], "span", st["span_problems"], flush=True)


if __name__ == "__main__":
    main()
