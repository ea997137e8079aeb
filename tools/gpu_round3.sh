#!/bin/bash
# Round-3 check on one MI355X: GPU tests, smoke, bench, rocprofv3 kernel trace + stats of the
# bench's sweep leg, then FETCH_SIZE / WRITE_SIZE counter passes (separate runs).  Steps are
# chained: the first failure ends the call.  Outputs under gpurun_out/r03/<tag>/.
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/r03/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step tests && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 ; rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] && \
step smoke && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log && \
step bench && \
timeout -k 10 800 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && head -c 400 $OUT/bench.json && echo && \
step trace && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --no-large --no-full --no-config2 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err && \
step fetch && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault --steps 1 --warmup 0 > $OUT/fetch.json 2> $OUT/fetch.err && \
step write && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault --steps 1 --warmup 0 > $OUT/write.json 2> $OUT/write.err && \
step done
