#!/bin/bash
# k_obs with unrolled in-tile bits: bitwise comparison with the previous build (libdse_old.so),
# the observable / parity GPU tests, then the bench's sweep leg, new vs old, two rounds each.
set -o pipefail
OUT=gpurun_out/r02/obsfast
mkdir -p $OUT
DSE_LIB=quantumsimulations_amd/libdse_old.so timeout -k 10 120 python -u tools/obs_compare.py $OUT/old.npy > $OUT/cmp_old.log 2>&1 || { tail $OUT/cmp_old.log; exit 1; }
timeout -k 10 120 python -u tools/obs_compare.py $OUT/new.npy > $OUT/cmp_new.log 2>&1 || { tail $OUT/cmp_new.log; exit 1; }
python -c "import numpy as np; a=np.load('$OUT/old.npy'); b=np.load('$OUT/new.npy'); print('bitwise equal:', np.array_equal(a,b), a.size, float(np.max(np.abs(a-b))))"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_config3.py tests/test_gpu_partitioned.py tests/test_gpu_wht.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
tools/gpu_variants.sh obsfast "new:quantumsimulations_amd/libdse.so:" "old:quantumsimulations_amd/libdse_old.so:"
