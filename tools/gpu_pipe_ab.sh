#!/bin/bash
# Software-pipelined fused loop (DSE_PIPE=1 build) against the default build.
set -o pipefail
OUT=gpurun_out/r02/pipe
mkdir -p $OUT
DSE_LIB=quantumsimulations_amd/libdse_pipe.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config3.py tests/test_gpu_parity.py tests/test_gpu_handoff.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for v in libdse libdse_pipe; do
  DSE_LIB=quantumsimulations_amd/$v.so timeout -k 10 200 python -u tools/probe_interval.py singles,pairs > $OUT/probe_$v.jsonl 2> $OUT/probe.err || exit 1
done
bash tools/gpu_variants.sh pipe_bench "base:quantumsimulations_amd/libdse.so:" "pipe:quantumsimulations_amd/libdse_pipe.so:"
