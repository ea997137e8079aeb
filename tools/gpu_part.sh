#!/bin/bash
# Config 5 partitioned register in loopback (all shards on one GPU): WHT engine (index swap) vs
# step kernels at N = 24, then the WHT engine at N = 30 with 8 shards.
set -o pipefail
mkdir -p gpurun_out/part
timeout -k 10 300 python -u tools/bench_partitioned.py --n-sea 23 --loopback 8 --wht 1 > gpurun_out/part/n24_lb8_wht.json 2> gpurun_out/part/err && \
timeout -k 10 300 python -u tools/bench_partitioned.py --n-sea 23 --loopback 8 --wht 0 > gpurun_out/part/n24_lb8_step.json 2>> gpurun_out/part/err && \
timeout -k 10 400 python -u tools/bench_partitioned.py --n-sea 29 --loopback 8 --wht 1 > gpurun_out/part/n30_lb8_wht.json 2>> gpurun_out/part/err
