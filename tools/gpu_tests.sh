#!/bin/bash
# GPU test pass: the whole -m gpu suite (or the files given), one process, per-test timeout.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
exit $rc
