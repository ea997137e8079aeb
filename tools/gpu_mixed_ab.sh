#!/bin/bash
# A/B of the mixed 1-/2-tile interval launch (option mixed_launch): its GPU test, then the sweep leg
# of the bench with and without it, two rounds each.
set -o pipefail
OUT=gpurun_out/r02/mixed
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config3.py tests/test_gpu_handoff.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
tools/gpu_variants.sh mixed "mixed:quantumsimulations_amd/libdse.so:--mixed-launch 1" "base:quantumsimulations_amd/libdse.so:--mixed-launch 0"
