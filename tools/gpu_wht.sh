#!/bin/bash
# Walsh-Hadamard engine: parity tests, then config 5 timings (N = 24 and N = 30) against the
# step kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wht.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wht_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_large.py --n-sea 23 --wht 1 > gpurun_out/large24_wht.json 2> gpurun_out/large.err && \
timeout -k 10 300 python -u tools/bench_large.py --n-sea 23 --wht 0 > gpurun_out/large24_step.json 2>> gpurun_out/large.err && \
timeout -k 10 400 python -u tools/bench_large.py --n-sea 29 --wht 1 > gpurun_out/large30_wht.json 2>> gpurun_out/large.err
