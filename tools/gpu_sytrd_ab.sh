#!/bin/bash
# A/B of tridiagonalisation builds (probe binaries) at 2^13 and 2^14, alternating; then the per-size
# symv bandwidth curve and column-kernel times of the first binary under rocprofv3.
#   tools/gpu_sytrd_ab.sh <probe binary> [<probe binary> ...]
set -o pipefail
OUT=gpurun_out/r03/sytrd_ab
mkdir -p $OUT
: > $OUT/ab.jsonl
trap "rm -f $OUT/trace/s_kernel_trace.csv" EXIT
export TMPDIR=/tmp
for n in 8192 16384; do
  timeout -k 10 200 $1 $n check 2>> $OUT/err.txt | grep check | tee -a $OUT/check.jsonl || { echo fail; cat $OUT/err.txt; exit 1; }
done
for i in 1 2; do
  for b in "$@"; do
    for n in 8192 16384; do
      timeout -k 10 200 $b $n 2>> $OUT/err.txt | sed "s#^{#{\"variant\": \"$(basename $b)\", #" >> $OUT/ab.jsonl || { echo fail; cat $OUT/err.txt; exit 1; }
    done
  done
done
grep -v dsyevd $OUT/ab.jsonl | grep -v rocsolver_dsytrd
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/trace -o s --output-format csv -- $1 16384 split > $OUT/prof.jsonl 2>> $OUT/err.txt && \
python3 tools/symv_curve.py $OUT/trace/s_kernel_trace.csv 16384
