#!/bin/bash
# Targeted GPU tests + a probe script: bash tools/gpu_quick.sh "<pytest -k expr or file list>" [probe args...]
set -o pipefail
OUT=gpurun_out/r03/quick
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $1 > $OUT/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|passed|failed" $OUT/tests.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
shift
if [ $# -gt 0 ]; then timeout -k 10 300 python -u "$@" > $OUT/probe.txt 2>&1; rc2=$?; cat $OUT/probe.txt | tail -30; exit $rc2; fi
exit $rc
