#!/bin/bash
# Interval-kernel change check: bitwise comparison of the bench sweep's observables between the
# in-tree library and tools/bin/libdse_base.so, the N = 14 GPU tests, then the sweep-leg A/B.
set -o pipefail
OUT=gpurun_out/r03/iv_ab
mkdir -p $OUT
timeout -k 10 200 python -u tools/dump_sweep_obs.py $OUT/new.npy > $OUT/dump.log 2>&1 && \
DSE_LIB=tools/bin/libdse_base.so timeout -k 10 200 python -u tools/dump_sweep_obs.py $OUT/base.npy >> $OUT/dump.log 2>&1 && \
python3 -c "
import numpy as np
a=np.load('$OUT/new.npy'); b=np.load('$OUT/base.npy')
print('bitwise equal:', np.array_equal(a,b), 'max diff', float(np.max(np.abs(a-b))))" || { cat $OUT/dump.log; exit 1; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_config3.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab3.sh dpp "new:quantumsimulations_amd/libdse.so" "base:tools/bin/libdse_base.so"
