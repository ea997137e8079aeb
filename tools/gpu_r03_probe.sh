#!/bin/bash
# Round-3 opening call: GPU tests at HEAD (timed), then the planning probe (tools/probe_r03.py).
# pytest failures (rc 1) do not stop the call; a timeout, crash or fault (any other rc) does.
set -o pipefail
OUT=gpurun_out/r03/probe
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests
T0=$(date +%s)
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc wall=$(( $(date +%s) - T0 )) s"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step probe && \
timeout -k 10 240 python -u tools/probe_r03.py config2 > $OUT/probe.jsonl 2> $OUT/probe.err && \
timeout -k 10 120 python -u tools/probe_r03.py n14serial >> $OUT/probe.jsonl 2>> $OUT/probe.err && \
timeout -k 10 240 python -u tools/probe_r03.py refdefault >> $OUT/probe.jsonl 2>> $OUT/probe.err && \
timeout -k 10 400 python -u tools/probe_r03.py eigh >> $OUT/probe.jsonl 2>> $OUT/probe.err ; rc=$?
cat $OUT/probe.jsonl; tail -5 $OUT/probe.err
step done
exit $rc
