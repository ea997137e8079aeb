#!/bin/bash
# A/B of bench options in one GPU call: the bench's sweep leg, alternating, three rounds each.
#   tools/gpu_abenv.sh <tag> "<name>:<VAR=value>[,VAR=value]" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/r03/ab_$TAG
mkdir -p $OUT
: > $OUT/variants.jsonl
for i in 1 2 3; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env ${envs//,/ } timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault > $OUT/$name.$i.json 2>> $OUT/err.log || exit 1
    python -c "import json; d=json.loads(open('$OUT/$name.$i.json').read().splitlines()[-1]); r=d['roofline']; print(json.dumps({'variant':'$name','value':round(d['value']),'ms_per_step':round(d['ms_per_step'],1),'frac':round(r['frac'],3),'avg_launch_us':round(r['avg_launch_us'],1),'chip_frac':round(r['chip_level']['frac'],3),'by_stream':[(round(x['avg_launch_us']),round(x['frac'],3)) for x in r.get('by_stream',[])]}))" | tee -a $OUT/variants.jsonl || exit 1
  done
done
