#!/bin/bash
# Interval-kernel change check: bitwise comparison of the bench sweep's observables between a
# variant build ($1, default tools/bin/libdse_dpp.so) and the in-tree library, the N = 14 GPU
# tests on the variant, then the sweep-leg A/B.
set -o pipefail
OUT=gpurun_out/r03/iv_ab
mkdir -p $OUT
NEW=${1:-tools/bin/libdse_dpp.so}
DSE_LIB=$NEW timeout -k 10 200 python -u tools/dump_sweep_obs.py $OUT/new.npy > $OUT/dump.log 2>&1 && \
timeout -k 10 200 python -u tools/dump_sweep_obs.py $OUT/base.npy >> $OUT/dump.log 2>&1 && \
python3 -c "
import numpy as np
a=np.load('$OUT/new.npy'); b=np.load('$OUT/base.npy')
print('bitwise equal:', np.array_equal(a,b), 'max diff', float(np.max(np.abs(a-b))))" || { cat $OUT/dump.log; exit 1; }
DSE_LIB=$NEW timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_config3.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1; rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab3.sh dpp "new:$NEW" "base:quantumsimulations_amd/libdse.so"
