#!/bin/bash
# A/B of the hand-off with and without agent-scope release/acquire fences (libdse_f.so), with the
# repeatability diagnostic of each; two bench rounds each.
set -o pipefail
OUT=gpurun_out/r02/fence
mkdir -p $OUT
DSE_LIB=quantumsimulations_amd/libdse_f.so timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_config3.py tests/test_gpu_handoff.py > $OUT/tests_f.log 2>&1 || { tail -20 $OUT/tests_f.log; exit 1; }
tail -1 $OUT/tests_f.log
DSE_LIB=quantumsimulations_amd/libdse_f.so timeout -k 10 300 python -u tools/diag_repeat.py "" "outputs_per_launch=1" > $OUT/rep_f.jsonl 2>&1 || exit 1
tools/gpu_variants.sh fence "base:quantumsimulations_amd/libdse.so:" "fences:quantumsimulations_amd/libdse_f.so:"
