#!/bin/bash
# Walsh-Hadamard engine and partitioned-register GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_wht.py tests/test_gpu_partitioned.py -x -v --timeout 120 --timeout-method thread > gpurun_out/wht_tests.log 2>&1
