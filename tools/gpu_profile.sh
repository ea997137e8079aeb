#!/bin/bash
# Round profile of the bench: kernel trace + stats of the default bench command (no CPU leg), then
# one counter pass each for FETCH_SIZE and WRITE_SIZE (separate runs; MI355X_MICROARCH.md:
# FETCH_SIZE counts 1/2 of a wide streaming read on gfx950 -- corrected in bench.py / DESIGN.md).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof/bench_under_rocprof.json 2> gpurun_out/prof/trace.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o fetch --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/prof/fetch.json 2> gpurun_out/prof/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o write --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/prof/write.json 2> gpurun_out/prof/write.err
