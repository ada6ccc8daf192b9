#!/bin/bash
# The measurement set committed under profiles/<round>/ (run on the GPU box from the repo root):
#   bench.json            python bench.py (default arguments)
#   prof/                 rocprofv3 --kernel-trace --stats of the same command
#   pmc/                  FETCH_SIZE / WRITE_SIZE / SQ / L2 passes over one bench step
set -o pipefail
out=${1:-gpurun_out/round}
mkdir -p "$out"
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
echo "bench done"; tail -c 600 "$out/bench.json"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$out/prof" -o run -- python3 "$R/bench.py" > "$R/$out/prof_bench.json" 2> "$R/$out/prof.err" ) || exit $?
echo "kernel-trace done"
bash tools/pmc_dp.sh "$out/pmc" || exit $?
echo "pmc done"
