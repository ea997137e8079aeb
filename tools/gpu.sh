#!/bin/bash
# One parameterised GPU runner (replaces the per-experiment gpu_*.sh wrappers of rounds 1-3).
#
#   tools/gpu.sh <tag> <task>[:arg,arg...] [<task>...]
#
# Every task runs under its own time limit; the first failure ends the call (no GPU step after
# a fault, an abort or a time limit).  Outputs land in gpurun_out/r06/<tag>/.
#   tests[:pytest-path-or-k]   pytest -m gpu (whole suite, a file, or "-k expr" as k=expr)
#   smoke                      __graft_entry__.smoke()
#   bench[:args]               python bench.py <args>  (args: comma-separated)
#   trace                      rocprofv3 --kernel-trace --stats of the bench's sweep leg
#   traffic                    FETCH_SIZE and WRITE_SIZE passes of the same (one counter per run)
#   traffic_large              the same over tools/bench_large.py (N = 30, Walsh-Hadamard engine)
#   large_trace[:args]         rocprofv3 kernel trace of tools/bench_large.py <args> (per-pass times)
#   sq:<set>                   three SQ counter passes over tools/probe_one.py <set>
#   sqeig:<dim>                the same over tools/bin/probe_eig2 <dim> (PMC_FILTER: a kernel regex)
#   sytrd:<dim,...>            tools/bin/probe_sytrd <dim> check
#   eig2:<dim[/random],...>    tools/bin/probe_eig2 (two-stage eigensolver vs dsyevd)
#   py:<script>,<args...>      python -u <script> <args> > <tag>/<script-name>.out
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/r06/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
LEGS="--no-cpu-baseline --no-large --no-full --no-config2 --no-refdefault --no-shard8"
step() { echo "[$(date +%T)] $*"; }
fail() { echo "FAILED: $* (rc $rc)"; exit 1; }
pmc() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" ${PMC_FILTER:+--kernel-include-regex "$PMC_FILTER"} -d $OUT/pmc/$name -o $name --output-format csv -- "${PMC_CMD[@]}" > $OUT/pmc.$name.log 2>&1
}
for T in "$@"; do
  task=${T%%:*}; arg=""; [ "$task" != "$T" ] && arg=${T#*:}
  IFS=',' read -r -a A <<< "$arg"
  step "$task ${A[*]}"
  case $task in
    tests)
      sel=(tests); [ -n "$arg" ] && sel=("$arg")
      [[ "$arg" == k=* ]] && sel=(tests -k "${arg#k=}")
      log=$OUT/gpu_tests${arg:+_$(basename "${arg#k=}" .py)}.log
      DSE_TEST_RECORD=$OUT timeout -k 10 1100 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu "${sel[@]}" > $log 2>&1; rc=$?
      tail -3 $log; [ $rc -eq 0 ] || fail tests ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
      cat $OUT/smoke.log; [ $rc -eq 0 ] || fail smoke ;;
    bench)
      nb=$((nb + 1)); b=$OUT/bench$([ $nb -gt 1 ] && echo _$nb)
      DSE_BENCH_DETAIL=$b.detail.json timeout -k 10 900 python -u bench.py "${A[@]}" > $b.json 2> $b.err; rc=$?
      head -c 600 $b.json; echo; [ $rc -eq 0 ] || { tail -5 $b.err; fail bench; } ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py $LEGS "${A[@]}" > $OUT/bench_under_rocprof.json 2> $OUT/trace.err; rc=$?
      [ $rc -eq 0 ] || fail trace ;;
    traffic)
      timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py $LEGS --steps 1 --warmup 0 > $OUT/fetch.json 2> $OUT/fetch.err; rc=$?
      [ $rc -eq 0 ] || fail fetch
      timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py $LEGS --steps 1 --warmup 0 > $OUT/write.json 2> $OUT/write.err; rc=$?
      [ $rc -eq 0 ] || fail write ;;
    traffic_large)  # FETCH_SIZE / WRITE_SIZE passes over the N = 30 register (tools/bench_large.py)
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/large/fetch -o fetch --output-format csv -- python3 tools/bench_large.py --steps 3 > $OUT/large_fetch.json 2> $OUT/large_fetch.err; rc=$?
      [ $rc -eq 0 ] || fail fetch_large
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/large/write -o write --output-format csv -- python3 tools/bench_large.py --steps 3 > $OUT/large_write.json 2> $OUT/large_write.err; rc=$?
      [ $rc -eq 0 ] || fail write_large ;;
    large_trace)  # large_trace:<bench_large args>: kernel trace of the N = 30 register (per-pass times)
      nl=$((nl + 1))
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/large_trace_$nl -o large --output-format csv -- python3 tools/bench_large.py "${A[@]}" > $OUT/large_trace_$nl.json 2> $OUT/large_trace_$nl.err; rc=$?
      echo "${A[*]}" > $OUT/large_trace_$nl.args; tail -c 400 $OUT/large_trace_$nl.json; [ $rc -eq 0 ] || fail large_trace ;;
    sq|sqeig)  # sqeig:<dim>: the same passes over tools/bin/probe_eig2 <dim>
      PMC_CMD=(python3 tools/probe_one.py "${A[@]}"); q=$(echo "${A[*]}" | tr ' =' '__')_
      [ $task = sqeig ] && PMC_CMD=(tools/bin/probe_eig2 "${A[@]}") && q=eig2_${q}
      pmc ${q}p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU; rc=$?
      [ $rc -eq 0 ] || fail sq p1
      pmc ${q}p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE; rc=$?
      [ $rc -eq 0 ] || fail sq p2
      pmc ${q}p3 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE; rc=$?
      [ $rc -eq 0 ] || fail sq p3 ;;
    eig2)  # eig2:<dim>[/random],...  tools/bin/probe_eig2 (two-stage eigensolver) against dsyevd
      for a in "${A[@]}"; do
        timeout -k 10 ${EIG2_TIMEOUT:-120} tools/bin/probe_eig2 ${a%%/*} $([ "$a" != "${a#*/}" ] && echo ${a#*/}) >> $OUT/eig2.jsonl 2>> $OUT/eig2.err; rc=$?
        tail -1 $OUT/eig2.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/eig2.err; fail eig2 $a; }
      done ;;
    eig2prof)  # rocprofv3 kernel trace of probe_eig2 <dim>
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/eig2prof_$arg -o eig2 --output-format csv -- tools/bin/probe_eig2 $arg > $OUT/eig2prof_$arg.out 2> $OUT/eig2prof_$arg.err; rc=$?
      tail -2 $OUT/eig2prof_$arg.out; [ $rc -eq 0 ] || fail eig2prof ;;
    sytrd)
      for n in "${A[@]}"; do
        timeout -k 10 200 tools/bin/probe_sytrd $n check >> $OUT/sytrd.jsonl 2>> $OUT/sytrd.err; rc=$?
        [ $rc -eq 0 ] || { cat $OUT/sytrd.err; fail sytrd $n; }
      done
      cat $OUT/sytrd.jsonl ;;
    py)
      s=${A[0]}; name=$(basename $s .py)${A[1]:+_${A[1]}}
      timeout -k 10 ${PY_TIMEOUT:-600} python -u "${A[@]}" > $OUT/$name.out 2> $OUT/$name.err; rc=$?
      tail -c 1500 $OUT/$name.out; [ $rc -eq 0 ] || { tail -20 $OUT/$name.err; fail py $s; } ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
step done
