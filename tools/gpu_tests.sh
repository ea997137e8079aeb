#!/bin/bash
# GPU test suite alone (tag argument names the output directory).
set -o pipefail
OUT=gpurun_out/r03/${1:-tests}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1; rc=$?
tail -4 $OUT/gpu_tests.log
exit $rc
