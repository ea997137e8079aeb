#!/bin/bash
# A/B of LLVM scheduler knobs for the whole library (variant builds via DSE_EXTRA_FLAGS):
#   libdse_mc.so  -mllvm -amdgpu-sched-strategy=max-memory-clause
#   libdse_tr.so  -mllvm -amdgpu-use-amdgpu-trackers
# config-3 parity tests on each variant, then the bench's sweep leg, two rounds each.
set -o pipefail
OUT=gpurun_out/r02/sched
mkdir -p $OUT
for v in mc tr; do
  DSE_LIB=quantumsimulations_amd/libdse_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config3.py > $OUT/tests_$v.log 2>&1 || { tail -20 $OUT/tests_$v.log; exit 1; }
  tail -1 $OUT/tests_$v.log
done
tools/gpu_variants.sh sched "base:quantumsimulations_amd/libdse.so:" "mc:quantumsimulations_amd/libdse_mc.so:" "tr:quantumsimulations_amd/libdse_tr.so:"
