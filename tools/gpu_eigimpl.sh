#!/bin/bash
# dense-engine tests, then the eigensolver A/B on one N = 14 point of the reference grid
set -o pipefail
OUT=gpurun_out/r03/eigimpl${TAG:-}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dense.py > $OUT/tests.log 2>&1; rc=$?; tail -12 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe_eigimpl.py "$@" > $OUT/probe.jsonl 2> $OUT/probe.err; rc=$?; cat $OUT/probe.jsonl; tail -3 $OUT/probe.err; exit $rc
