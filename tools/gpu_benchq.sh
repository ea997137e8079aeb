#!/bin/bash
# Quick bench check: smoke, then the sweep leg only (no CPU / full / large / config-2 legs).
set -o pipefail
OUT=gpurun_out/r03/benchq
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault > $OUT/bench.json 2> $OUT/bench.err && \
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]); r=d['roofline']
print(d['value'], r['frac'], r['chip_level']['frac']); print(json.dumps(r['by_stream'], indent=1))"
DSE_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault --steps 3 --warmup 1 > $OUT/bench_ht.json 2> $OUT/host_phases.txt && tail -40 $OUT/host_phases.txt
