#!/bin/bash
# Experiment: N = 13 sweep as 1 tile of 2^13 (one 512-thread workgroup per CU) vs 2 tiles of 2^12
# (256-thread workgroups, two per CU) in the persistent kernel.
set -o pipefail
mkdir -p gpurun_out/l12
timeout -k 10 300 python -u bench.py --no-cpu-baseline --n-sea 12 --steps 2 --tile-bits 13 > gpurun_out/l12/n13_t13.json 2> gpurun_out/l12/err && \
DSE_CORESIDENT=512 timeout -k 10 300 python -u bench.py --no-cpu-baseline --n-sea 12 --steps 2 --tile-bits 12 > gpurun_out/l12/n13_t12.json 2>> gpurun_out/l12/err && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --n-sea 12 --steps 2 --tile-bits 12 > gpurun_out/l12/n13_t12_cap256.json 2>> gpurun_out/l12/err
