#!/bin/bash
# The config-3 reference-grid GPU test, then the bench's sweep leg with DSE_HOST_TIMING=1: host time
# of each dse_evolve phase per step (what the step time holds besides the launch loop).
set -o pipefail
OUT=gpurun_out/r02/hg
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config3.py -k reference_grid -s > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
grep -E "reference grid|passed|failed" $OUT/test.log
DSE_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-large --no-full --steps 2 --warmup 1 > $OUT/bench.json 2> $OUT/host.err || exit 1
python - <<'PY'
import collections
d=collections.defaultdict(list)
for l in open('gpurun_out/r02/hg/host.err'):
    if l.startswith('[dse_evolve]'):
        d[l[len('[dse_evolve]'):].rsplit(None, 2)[0].strip()].append(float(l.split()[-2]))
for k,v in d.items(): print(k, len(v), ["%.2f"%x for x in v[-3:]])
PY
