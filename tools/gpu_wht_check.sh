#!/bin/bash
# Walsh-Hadamard engine check: its GPU tests, then the bench with the config-5 leg (N = 30).
set -o pipefail
OUT=gpurun_out/r02/whtcheck
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wht.py tests/test_gpu_dist.py tests/test_gpu_config5.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-full > $OUT/bench.json 2> $OUT/bench.err || exit 1
python -c "
import json; d=json.load(open('$OUT/bench.json')); lr=d['large_register']
print('sweep', round(d['value']), 'large ms/H', round(lr['kernel_ms_per_h_application'],2), 'frac', round(lr['roofline']['frac'],3), lr['check']['ok'])
"
