#!/bin/bash
# Walsh-Hadamard engine tests, then per-pass kernel times for both tile sizes (kernel trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/whtvar
run() {  # name n_sea tile_bits group_bits
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/whtvar/$1 -o k --output-format csv -- python3 tools/bench_large.py --n-sea $2 --wht-tile-bits $3 --wht-group-bits $4 > gpurun_out/whtvar/$1.json 2> gpurun_out/whtvar/$1.err
}
timeout -k 10 400 python -u -m pytest tests/test_gpu_wht.py -x -q --timeout 120 --timeout-method thread > gpurun_out/whtvar/tests.log 2>&1 && \
run n24t13 23 13 0 && run n24t12 23 12 0 && run n22t12 21 12 0 && run n22t13 21 13 0 && run n30t12 29 12 0 && run n30t13 29 13 0
