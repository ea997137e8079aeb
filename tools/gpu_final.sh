#!/bin/bash
# Round-end verification: GPU tests, smoke, bench (with CPU baseline and the config-5 leg), then
# the bench's kernel trace + stats and the FETCH_SIZE / WRITE_SIZE counter passes.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err && \
bash tools/gpu_profile.sh
