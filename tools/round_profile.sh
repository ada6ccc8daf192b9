#!/bin/bash
# The measurement set committed under profiles/<round>/ (run on the GPU box from the repo root):
#   pmc/ + pmc_9mer.json  FETCH_SIZE / WRITE_SIZE / SQ / L2 passes over one bench step, and
#                         the per-pass HBM traffic record bench.py reports (written into the
#                         box's profiles/r01 first, so the bench below picks it up)
#   bench.json            python bench.py (default arguments)
#   prof/                 rocprofv3 --kernel-trace --stats of the same command
set -o pipefail
out=${1:-gpurun_out/round}
mkdir -p "$out"
R=$GRAFT_REPO_ROOT
bash tools/pmc_dp.sh "$out/pmc" || exit $?
python3 tools/pmc_json.py "$out/pmc" profiles/r01/pmc_9mer.json 5 > "$out/pmc_9mer.json" || exit $?
cp profiles/r01/pmc_9mer.json "$out/pmc_9mer.json"
echo "pmc done"
timeout -k 10 300 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
echo "bench done"; tail -c 400 "$out/bench.json"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$out/prof" -o run -- python3 "$R/bench.py" > "$R/$out/prof_bench.json" 2> "$R/$out/prof.err" ) || exit $?
echo "kernel-trace done"
