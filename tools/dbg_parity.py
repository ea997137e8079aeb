"""Debug: run-to-run determinism of the persistent 2-tile path under kernel-section ablations.
Prints, per ablation mask, the largest deviation between repeated evolves of the same problems.
Ablation options (ablate, span_ablate, real_ablate) need a diagnostics build of the same ABI:
    DSE_EXTRA_FLAGS=-DDSE_DIAG python -m quantumsimulations_amd.build --out tools/bin/libdse_diag.so
    DSE_LIB=tools/bin/libdse_diag.so python3 tools/dbg_parity.py ...
"""
import sys, numpy as np
sys.path.insert(0, '.')
from quantumsimulations_amd import problem as pb
from quantumsimulations_amd.engine import Engine
from quantumsimulations_amd.sweep import sweep_point_params
t = np.linspace(0.0, 2e-5, 5)
params = [sweep_point_params(13, d, v, 2e-5, 5) for d in (0.0, 50e3, 100e3, 150000.0) for v in ("center_on", "shell_off")]
with Engine(0, tile_bits=13) as eng:
    for p in params: eng.add(pb.build_problem(p))
    for ab in [int(a) for a in sys.argv[1:]] or [0]:
        eng.set_option("ablate", ab)
        first, _ = eng.evolve(t)
        worst = np.zeros(len(params))
        for rep in range(5):
            o, st = eng.evolve(t)
            worst = np.maximum(worst, np.abs(o - first).max(axis=(1, 2)))
        print("ablate", ab, [f"{x:.1e}" for x in worst], flush=True)
    eng.set_option("ablate", 0)
