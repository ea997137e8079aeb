#!/bin/bash
# Counter passes over tools/probe_one.py (one rocprofv3 --pmc pass per run, each time-limited).
#   tools/gpu_pmc.sh <tag> [set...]       sets: singles pairs all
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-pmc}; shift
SETS=${@:-singles pairs}
OUT=gpurun_out/r02/$TAG
mkdir -p $OUT
run() {  # set name counters...
  local set=$1 name=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT/$set/$name -o $name --output-format csv -- python3 tools/probe_one.py $set > $OUT/$set.$name.log 2>&1
}
for S in $SETS; do
  run $S p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU && \
  run $S p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
  run $S p3 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE || exit 1
done
echo done
