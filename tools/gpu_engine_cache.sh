#!/bin/bash
# evolve_many's per-device context cache: the GPU tests that go through evolve_many, then the full
# config-4 driver without figures with the cache on and off (DSE_ENGINE_CACHE=0).
set -o pipefail
OUT=gpurun_out/r02/ecache
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sweep.py tests/test_gpu_config4.py tests/test_gpu_small.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for c in 1 0 1 0; do
  DSE_ENGINE_CACHE=$c timeout -k 10 300 python -u -m quantumsimulations_amd.sweep2d_run --root /tmp/c4_$c --report none --stable --coarse-window 10 > $OUT/c4_cache$c.log 2>&1 || { tail -20 $OUT/c4_cache$c.log; exit 1; }
  tail -1 $OUT/c4_cache$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cache=$c', round(d['evolve_s'],3), round(d['wall_s'],3))"
  rm -rf /tmp/c4_$c
done
