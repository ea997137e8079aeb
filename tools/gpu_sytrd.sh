#!/bin/bash
# Half-matrix tridiagonalisation (dse_sytrd.hip) vs rocSOLVER: accuracy at 2^11..2^14 with timings,
# then the phases and kernel split of sytrd_lower at $PROF_DIM (default 16384).
set -o pipefail
OUT=gpurun_out/r03/sytrd${TAG:-3}
trap "rm -f $OUT/trace/s_kernel_trace.csv" EXIT  # too large to bring back; summarised on the box
mkdir -p $OUT
export TMPDIR=/tmp
for n in ${DIMS:-2048 4096 8192 16384}; do
  timeout -k 10 200 tools/bin/probe_sytrd $n check >> $OUT/probe.jsonl 2>> $OUT/err.txt || { echo "fail $n $?"; cat $OUT/err.txt; exit 1; }
done
cat $OUT/probe.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o s --output-format csv -- tools/bin/probe_sytrd ${PROF_DIM:-16384} split > $OUT/prof.jsonl 2>> $OUT/err.txt && cat $OUT/prof.jsonl && \
python3 -c "
import csv
rows=list(csv.DictReader(open('$OUT/trace/s_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:25]: print(r['Calls'].rjust(6), ('%.1f ms' % (float(r['TotalDurationNs'])/1e6)).rjust(10), ('%.1f us' % (float(r['AverageNs'])/1e3)).rjust(10), r['Name'][:110])
"
python3 tools/symv_curve.py $OUT/trace/s_kernel_trace.csv ${PROF_DIM:-16384}
