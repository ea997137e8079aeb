#!/bin/bash
# Partitioned registers: parity of the overlapped index-swap schedule (WHT, dist and partitioned GPU
# tests), then loopback timings with and without the overlap.
set -o pipefail
OUT=gpurun_out/r02/swap
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wht.py tests/test_gpu_dist.py tests/test_gpu_partitioned.py tests/test_gpu_config5.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for ov in 0 1 0 1; do
  timeout -k 10 200 python -u tools/bench_partitioned.py --loopback 8 --n-sea 27 --swap-overlap $ov >> $OUT/loop_n28.jsonl 2>> $OUT/err.log || exit 1
done
for ov in 0 1; do
  timeout -k 10 300 python -u tools/bench_partitioned.py --loopback 8 --n-sea 29 --swap-overlap $ov >> $OUT/loop_n30.jsonl 2>> $OUT/err.log || exit 1
done
python -c "
import json
for f in ('$OUT/loop_n28.jsonl','$OUT/loop_n30.jsonl'):
    for l in open(f):
        d=json.loads(l); print(f.split('/')[-1], d['swap_overlap'], round(d['ms_per_h_application'],2), d.get('norm_check', d.get('max_norm_error')))
"
