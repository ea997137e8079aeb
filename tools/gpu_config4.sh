#!/bin/bash
# BASELINE config 4 end to end on the box's GPU(s): 8 f1A sweeps (linspace 5..50 kHz) x 64
# detunings x 3 variants = 1536 N = 14 evolutions, per-point files + metrics, then the 2D report;
# once without per-point figures and once with the PNG figures written by the worker processes
# while the next group evolves.  1 ms / 101 outputs with 10-output coarse
# windows (the reference default, 100, leaves one window on this grid).  Trees go to /tmp on the box.
set -o pipefail
OUT=gpurun_out/r02/config4
mkdir -p $OUT
timeout -k 10 400 python -u -m quantumsimulations_amd.sweep2d_run --root /tmp/c4_none --report none --stable --coarse-window 10 > $OUT/none.log 2>&1 || { tail -20 $OUT/none.log; exit 1; }
tail -1 $OUT/none.log
timeout -k 10 700 python -u -m quantumsimulations_amd.sweep2d_run --root /tmp/c4_png --report png --stable --coarse-window 10 > $OUT/png.log 2>&1 || { tail -20 $OUT/png.log; exit 1; }
tail -1 $OUT/png.log
cp /tmp/c4_png/stable_region_stats.json $OUT/ 2>/dev/null; ls /tmp/c4_png | head -20
