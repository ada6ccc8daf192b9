#!/bin/bash
# PMC passes over one bench step (each pass its own run; <= 8 SQ / 4 TCC counters per pass).
# usage: tools/pmc_dp.sh OUTDIR [env assignments...]; writes OUTDIR/<pass>/*counter_collection.csv
# BENCH_ARGS: extra bench.py arguments (e.g. "--config 11mer")
out=$1; shift
for kv in "$@"; do export "$kv"; done
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$R/$out/$name" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-full-cv $BENCH_ARGS > "$R/$out/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc  # a failed GPU step ends the script
}
want() { [ -z "$PASSES" ] || [[ " $PASSES " == *" $1 "* ]]; }
want sq1 && run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
want sq2 && run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
want fetch && run fetch FETCH_SIZE
want write && run write WRITE_SIZE
want l2 && run l2 TCC_HIT_sum TCC_MISS_sum
true
