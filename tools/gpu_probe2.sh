#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03/probe2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/refdefault_e2e.py --report none > $OUT/refdefault_e2e.json 2> $OUT/e2e.err && cat $OUT/refdefault_e2e.json && \
timeout -k 10 300 python -u tools/refdefault_e2e.py --report png > $OUT/refdefault_e2e_png.json 2>> $OUT/e2e.err && cat $OUT/refdefault_e2e_png.json && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c2 -o c2 --output-format csv -- python3 tools/probe_config2.py > $OUT/c2_probe.txt 2> $OUT/c2.err && cat $OUT/c2_probe.txt && \
for tb in 13 12 13 12; do timeout -k 10 200 python -u tools/bench_large.py --wht-tile-bits $tb >> $OUT/wht_tb.jsonl 2>> $OUT/wht.err || exit 1; done; cat $OUT/wht_tb.jsonl | cut -c1-300
