#!/bin/bash
set -o pipefail
OUT=gpurun_out/r03/c2prof
mkdir -p $OUT
export TMPDIR=/tmp
DSE_HOST_TIMING=1 timeout -k 10 120 python -u tools/probe_config2.py > $OUT/probe.txt 2> $OUT/host_phases.txt && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c2 --output-format csv -- python3 tools/probe_config2.py > $OUT/probe_rocprof.txt 2> $OUT/trace.err && \
timeout -k 10 200 python -u tools/probe_tile12.py > $OUT/tile12.jsonl 2> $OUT/tile12.err
cat $OUT/probe.txt; tail -20 $OUT/host_phases.txt; cat $OUT/tile12.jsonl
