#!/bin/bash
# Dense-engine check: its GPU tests, the eigensolver A/B point on the 30 s grid, then the
# tridiagonalisation A/B of probe binaries (tools/gpu_sytrd_ab.sh) when any are given.
set -o pipefail
OUT=gpurun_out/r03/dense_round
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dense.py > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/probe_eigimpl.py 1:2 0:2 1:2 > $OUT/point.jsonl 2> $OUT/point.err; rc=$?; cat $OUT/point.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/point.err; exit $rc; }
[ $# -gt 0 ] && bash tools/gpu_sytrd_ab.sh "$@"
exit 0
