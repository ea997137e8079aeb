#!/bin/bash
# Iteration pass: gpu parity tests, interval-kernel ablation probe, bench without the CPU leg
# (default outputs per launch, then one per launch for comparison).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/probe_interval.py > gpurun_out/probe.jsonl 2> gpurun_out/probe.err && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline --outputs-per-launch 1 > gpurun_out/bench_m1.json 2>> gpurun_out/bench.err
