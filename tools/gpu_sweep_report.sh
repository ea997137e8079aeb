#!/bin/bash
# The single-sweep drop-in (run_sweep_sea_detuning, config 3 at N = 14: 32 detunings, 1 ms / 101
# outputs, 10-output coarse windows) with the reference's full report (PDF + per-point PNGs):
# PNGs drawn by worker processes while this process writes the PDF, against the serial report
# (DSE_REPORT_WORKERS=1).  Trees go to /tmp on the box; a ticker keeps the call from looking hung.
set -o pipefail
OUT=gpurun_out/r02/sweep_report
mkdir -p $OUT
cat > /tmp/sweep_report_run.py <<'PY'
import json, time, numpy as np
from quantumsimulations_amd.sweep import GAMMA_RARE, GAMMA_SEA, PHI, SWEEP_TOL, f_az_hz
from quantumsimulations_amd.sweep_runner import run_sweep_sea_detuning, writer_count
if __name__ == "__main__":
    tm = {}
    t0 = time.perf_counter()
    run_sweep_sea_detuning(f_Az=f_az_hz(), f1A=50e3, target_sea_detuning=50e3, gamma_sea=GAMMA_SEA,
                           gamma_rare=GAMMA_RARE, sea_detunings_Hz=np.linspace(0.0, 150e3, 32),
                           n_sea=13, t_final=1e-3, steps=101, phi_sea=PHI, phi_rare=PHI,
                           out_root="/tmp/sr", coarse_window=10, report="full", timings=tm,
                           verbose=False, **SWEEP_TOL)
    tm["wall_s"] = time.perf_counter() - t0
    tm["report_workers"] = writer_count()
    tm["points"] = 32
    print(json.dumps(tm), flush=True)
PY
( while sleep 30; do echo "tick $(date +%T)"; done ) &
TICK=$!
rc=0
for w in 0 1; do
  if [ $w = 1 ]; then export DSE_REPORT_WORKERS=1; else unset DSE_REPORT_WORKERS; fi
  PYTHONPATH=$PWD timeout -k 10 500 python -u /tmp/sweep_report_run.py > $OUT/workers$w.json 2> $OUT/workers$w.err || { rc=1; tail -20 $OUT/workers$w.err; break; }
  cat $OUT/workers$w.json
  rm -rf /tmp/sr
done
kill $TICK
exit $rc
