#!/bin/bash
# Persistent MID (option wht_persist = 2): bitwise test, then N = 30 A/B in one call (alternating),
# then a rocprofv3 kernel trace of each variant.
set -o pipefail
OUT=gpurun_out/r03/whtp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wht.py -k persistent > $OUT/tests.log 2>&1; rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for pm in 0 2 0 2; do
  timeout -k 10 150 python -u tools/bench_large.py --n-sea 29 --t-final 5e-6 --steps 6 --wht-persist $pm >> $OUT/ab.jsonl 2>> $OUT/ab.err || exit $?
  tail -1 $OUT/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['wht_persist'], round(d['ms_per_h_application'],2), 'ms/H')"
done
for pm in 0 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace$pm -o w --output-format csv -- python3 tools/bench_large.py --n-sea 29 --t-final 5e-6 --steps 6 --wht-persist $pm > $OUT/rp$pm.json 2> $OUT/rp$pm.err || exit $?
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$OUT/trace$pm/w_kernel_stats.csv')):
    if 'k_wht' in r['Name']: print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
" 
done
