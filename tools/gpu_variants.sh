#!/bin/bash
# Bench (sweep leg only) over library variants / options, two rounds each, one GPU call.
#   tools/gpu_variants.sh <tag> "<name>:<lib>:<extra bench args>" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/r02/$TAG
mkdir -p $OUT
: > $OUT/variants.jsonl
for i in 1 2; do
  for spec in "$@"; do
    IFS=: read name lib extra <<< "$spec"
    DSE_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-large --no-full $extra > $OUT/$name.$i.json 2>> $OUT/err.log || exit 1
    python -c "import json; d=json.load(open('$OUT/$name.$i.json')); r=d['roofline']; print(json.dumps({'variant':'$name','value':round(d['value']),'ms_per_step':round(d['ms_per_step'],1),'frac':round(r['frac'],3),'avg_launch_us':round(r['avg_launch_us'],1),'chip_frac':round(r['chip_level']['frac'],3),'h_per_step':d['config']['h_applications_per_step']}))" | tee -a $OUT/variants.jsonl || exit 1
  done
done
