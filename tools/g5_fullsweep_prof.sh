#!/bin/bash
# round-6 profile call: the full sweep's solver-stream A/B and kernel trace (NUFFT outputs), then
# the bench sweep leg's kernel trace and FETCH/WRITE counter passes (tools/gpu.sh trace, traffic)
set -o pipefail
mkdir -p gpurun_out/r06/g5
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probe_fullsweep.py points=8,eig_streams=3 points=8,eig_streams=2 points=8,eig_streams=4 points=8,eig_streams=3 > gpurun_out/r06/g5/streams_ab.jsonl 2> gpurun_out/r06/g5/streams_ab.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/g5/trace -o fs --output-format csv -- python3 tools/probe_fullsweep.py points=6 > gpurun_out/r06/g5/trace.out 2> gpurun_out/r06/g5/trace.err || exit 1
bash tools/gpu.sh g5 trace traffic
