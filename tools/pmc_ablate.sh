#!/bin/bash
# SQ instruction counters of one bench step under KP_DEBUG_SKIP ablations (timing-only builds
# of the phases; see kp_dp_params.dbg).  usage: tools/pmc_ablate.sh OUTDIR v1 v2 ...
out=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  KP_DEBUG_SKIP=$v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$R/$out/d$v" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-full-cv > "$R/$out/d$v.log" 2>&1 || exit 1
  echo "pass $v done"
done
