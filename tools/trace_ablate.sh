#!/bin/bash
# Per-launch kernel traces of one bench step: full, levels-only (KP_DEBUG_SKIP=1) and
# gather-only (KP_DEBUG_SKIP=2).  Extra VAR=value arguments are exported to every run.
set -o pipefail
R=$GRAFT_REPO_ROOT
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2; do
  KP_DEBUG_SKIP=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr$v -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-full-cv > $R/gpurun_out/tr$v.log 2>&1 || exit 1
  echo "trace $v done"
done
