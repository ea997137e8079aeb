#!/bin/bash
# A/B of two builds of libdse in one GPU call: parity tests of B first, then the bench (sweep leg
# only) alternately A, B, A, B.  A = quantumsimulations_amd/libdse_a.so, B = libdse.so.
#   tools/gpu_ab.sh <tag> [pytest files...]
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/r02/$TAG
mkdir -p $OUT
: > $OUT/ab.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${@:-tests/test_gpu_config3.py tests/test_gpu_parity.py tests/test_gpu_handoff.py} > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for v in a b; do
    if [ $v = a ]; then L=quantumsimulations_amd/libdse_a.so; else L=quantumsimulations_amd/libdse.so; fi
    DSE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-large --no-full > $OUT/ab_$v$i.json 2>> $OUT/ab.err || exit 1
    python -c "import json; d=json.load(open('$OUT/ab_$v$i.json')); r=d['roofline']; print(json.dumps({'variant':'$v','value':round(d['value']),'ms_per_step':round(d['ms_per_step'],1),'frac':round(r['frac'],3),'avg_launch_us':round(r['avg_launch_us'],1),'chip_frac':round(r['chip_level']['frac'],3)}))" | tee -a $OUT/ab.jsonl || exit 1
  done
done
DSE_LIB=quantumsimulations_amd/libdse.so timeout -k 10 300 python -u tools/probe_interval.py center_on,shell_off,pairs,singles > $OUT/probe.jsonl 2> $OUT/probe.err
exit 0
