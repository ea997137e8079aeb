#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03/eigst
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dense.py > $OUT/tests.log 2>&1; rc=$?; tail -4 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_eigstreams.py > $OUT/probe.jsonl 2> $OUT/probe.err; rc=$?; cat $OUT/probe.jsonl; tail -3 $OUT/probe.err; exit $rc
