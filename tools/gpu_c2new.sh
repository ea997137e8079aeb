#!/bin/bash
# Matrix mode check: GPU tests of the propagator-matrix mode, host phases of one config-2 call,
# then the config-2 kernel split under rocprofv3.
set -o pipefail
OUT=gpurun_out/r03/c2new
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_matrix.py > $OUT/tests.log 2>&1; rc=$?; tail -8 $OUT/tests.log; [ $rc -eq 0 ] && \
DSE_HOST_TIMING=1 timeout -k 10 120 python -u tools/probe_config2.py > $OUT/probe.txt 2> $OUT/host_phases.txt && cat $OUT/probe.txt && tail -12 $OUT/host_phases.txt && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c2 --output-format csv -- python3 tools/probe_config2.py > $OUT/probe_rocprof.txt 2> $OUT/trace.err && \
cat $OUT/probe_rocprof.txt && head -8 $OUT/trace/c2_kernel_stats.csv
