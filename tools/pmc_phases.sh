#!/bin/bash
# SQ instruction counters of the 5-lane 9-mer pass with phases ablated (tool): one rocprofv3
# --pmc run of tools/ablate.py per KP_DEBUG_SKIP value, on the timing-ablation build
# (make -C kmerpapa_amd/csrc ablation).  The differences between runs attribute the VALU /
# LDS instructions to the gather (1), the level phase (2), the logs (4), the low split scan (8).
# usage: tools/pmc_phases.sh OUTDIR SKIP...
out=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  KMERPAPA_LIB="$R/kmerpapa_amd/libkmerpapa_hip_ablation.so" timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$R/$out/s$v" -o run -- python3 "$R/tools/ablate.py" "$v" > "$R/$out/s$v.log" 2>&1 || exit 1
  echo "skip $v done"
done
