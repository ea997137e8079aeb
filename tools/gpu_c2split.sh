#!/bin/bash
# Config-2 kernel split: rocprofv3 kernel trace + stats of tools/probe_config2.py (matrix mode and
# the per-interval path), summarised by kernel.
set -o pipefail
OUT=gpurun_out/r03/c2split
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c2 --output-format csv -- python3 tools/probe_config2.py > $OUT/probe_rocprof.txt 2> $OUT/trace.err && \
cat $OUT/probe_rocprof.txt && head -20 $OUT/trace/c2_kernel_stats.csv
