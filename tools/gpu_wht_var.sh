#!/bin/bash
# Walsh-Hadamard engine tests, then per-pass kernel times for several group layouts (kernel trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/whtvar
run() {  # name n_sea group_bits
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/whtvar/$1 -o k --output-format csv -- python3 tools/bench_large.py --n-sea $2 --wht-group-bits $3 > gpurun_out/whtvar/$1.json 2> gpurun_out/whtvar/$1.err
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_wht.py -x -q --timeout 120 --timeout-method thread > gpurun_out/whtvar/tests.log 2>&1 && \
run n24g11 23 11 && run n24g6 23 6 && run n23g10 22 10 && run n22g9 21 9 && run n30g11 29 11
