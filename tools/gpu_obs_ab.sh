#!/bin/bash
# Overlapped observables (option obs_overlap): the persistent-path GPU tests, then the bench's sweep
# leg with the option on and off, two rounds each.
set -o pipefail
OUT=gpurun_out/r02/obs
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config3.py tests/test_gpu_handoff.py tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_small.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
tools/gpu_variants.sh obs "ovl:quantumsimulations_amd/libdse.so:--obs-overlap 1" "inline:quantumsimulations_amd/libdse.so:--obs-overlap 0"
