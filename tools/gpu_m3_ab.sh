#!/bin/bash
# Three outputs per launch (DSE_MAX_OUT=3 build) against the default build, bench sweep leg.
set -o pipefail
OUT=gpurun_out/r02/m3
mkdir -p $OUT
DSE_LIB=quantumsimulations_amd/libdse_m3.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config3.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_variants.sh m3_bench "base:quantumsimulations_amd/libdse.so:" "m3b2:quantumsimulations_amd/libdse_m3.so:--outputs-per-launch 2" "m3:quantumsimulations_amd/libdse_m3.so:--outputs-per-launch 3"
