# The N = 30 engine's strided passes run in a fast or a slow mode from process to process: three
# processes, each under one UTCL1 counter pass, to see whether translation misses follow the mode
# (per-dispatch durations from the same pass).
set -o pipefail
O=gpurun_out/r06/mode; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum -d $O/p$i -o p$i --output-format csv -- python3 tools/bench_large.py --steps 2 > $O/p$i.json 2> $O/p$i.err || exit 1
done
