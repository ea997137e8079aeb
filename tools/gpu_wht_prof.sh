#!/bin/bash
# Walsh-Hadamard engine profile at config 5 sizes: kernel trace + stats (N = 24), then FETCH_SIZE
# and WRITE_SIZE counter passes (separate runs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
N_SEA=${N_SEA:-23}
mkdir -p gpurun_out/whtprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/whtprof/trace -o wht --output-format csv -- python3 tools/bench_large.py --n-sea $N_SEA > gpurun_out/whtprof/large.json 2> gpurun_out/whtprof/trace.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/whtprof/fetch -o fetch --output-format csv -- python3 tools/bench_large.py --n-sea $N_SEA --t-final 2e-6 --steps 2 > gpurun_out/whtprof/fetch.json 2> gpurun_out/whtprof/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/whtprof/write -o write --output-format csv -- python3 tools/bench_large.py --n-sea $N_SEA --t-final 2e-6 --steps 2 > gpurun_out/whtprof/write.json 2> gpurun_out/whtprof/write.err
