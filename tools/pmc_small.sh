#!/bin/bash
# SQ counters of one 1-lane and one 5-lane 9-mer pass (tools/pass_once.py), one rocprofv3
# --pmc run per counter set.  usage: tools/pmc_small.sh OUTDIR
out=$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$R/$out/$name" -o run -- \
    python3 "$R/tools/pass_once.py" 1 5 > "$R/$out/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run sq3 SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_INSTS_VALU_TRANS_F32
