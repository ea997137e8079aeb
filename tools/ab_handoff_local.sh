# (round 6 A/B; the option handoff_local was removed after it: no change in time or traffic)
# A/B of option handoff_local on the bench's sweep leg (step time, k_interval launch time), then
# FETCH_SIZE passes per setting (tools/pmc_summary.py reads gpurun_out/r06/x2/<setting>/).
set -o pipefail
O=gpurun_out/r06/x2; mkdir -p $O
LEGS="--no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault --no-shard8"
for v in 2 1 0; do
  DSE_BENCH_SET=handoff_local=$v timeout -k 10 200 python bench.py $LEGS --steps 5 --warmup 1 --detail $O/d.json > $O/b_$v.json 2>> $O/b.err || exit 1
  python -c "import json,sys;d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]);print('local=$v', d['ms_per_step'], d['roofline']['avg_launch_us'])"
  DSE_BENCH_SET=handoff_local=$v timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $O/l$v/fetch -o fetch --output-format csv -- python3 bench.py $LEGS --steps 1 --warmup 0 --detail $O/d2.json > $O/fetch_$v.json 2> $O/fetch_$v.err || exit 1
done
