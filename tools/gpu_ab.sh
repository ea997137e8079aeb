#!/bin/bash
# A/B of two builds of libdse in one GPU call: bench (no CPU leg) alternately A, B, A, B.
# A = quantumsimulations_amd/libdse_a.so, B = quantumsimulations_amd/libdse.so
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for i in 1 2; do
  for v in a b; do
    if [ $v = a ]; then L=quantumsimulations_amd/libdse_a.so; else L=quantumsimulations_amd/libdse.so; fi
    DSE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_tmp.json 2>> gpurun_out/ab.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_tmp.json')); print(json.dumps({'variant':'$v','value':d['value'],'ms_per_step':d['ms_per_step'],'frac':d['roofline']['frac']}))" >> gpurun_out/ab.jsonl || exit 1
  done
done
