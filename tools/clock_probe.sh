# GPU clock under the bench's full sweep against one GPU's 2-GPU share (k_interval only): one
# GRBM_GUI_ACTIVE pass each (cycles the GPU was busy, per dispatch), divided by the dispatch's
# duration from the same pass (tools/clock_summary.py).
set -o pipefail
O=gpurun_out/r06/clk; mkdir -p $O
export TMPDIR=/tmp
LEGS="--no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault --no-shard8"
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/full -o full --output-format csv -- python3 bench.py $LEGS --steps 1 --warmup 0 --detail $O/d.json > $O/full.json 2> $O/full.err || exit 1
SHARD_WORLD=2 SHARD_RANK=1 timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/share2 -o share2 --output-format csv -- python3 tools/probe_span.py shard 1 0 > $O/share2.out 2> $O/share2.err || exit 1
SHARD_WORLD=8 SHARD_RANK=7 timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/share8 -o share8 --output-format csv -- python3 tools/probe_span.py shard 1 0 > $O/share8.out 2> $O/share8.err || exit 1
