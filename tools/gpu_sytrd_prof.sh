#!/bin/bash
# Kernel split of rocSOLVER dsyevd / dsytrd at dim 8192 (one solve after a warm-up).
set -o pipefail
OUT=gpurun_out/r03/sytrd
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o s --output-format csv -- tools/bin/probe_eig 8192 1 > $OUT/probe.jsonl 2> $OUT/err.txt && cat $OUT/probe.jsonl && \
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/trace/s_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print(r['Calls'].rjust(6), ('%.1f ms' % (float(r['TotalDurationNs'])/1e6)).rjust(10), ('%.1f us' % (float(r['AverageNs'])/1e3)).rjust(10), r['Name'][:110])
"
