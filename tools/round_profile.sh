#!/bin/bash
# The measurement set committed under profiles/<round>/ (run on the GPU box from the repo root):
#   pmc/ + pmc_9mer.json  FETCH_SIZE / WRITE_SIZE / L2 hit passes over one bench step: the
#                         per-pass L2-miss fabric traffic record bench.py reports (written
#                         into the box's profiles/<round> first, so the bench below uses it)
#   bench.json            python bench.py (default arguments)
#   prof/                 rocprofv3 --kernel-trace --stats of the same command
# usage: tools/round_profile.sh OUTDIR ROUND   (e.g. gpurun_out/r03 r03)
# The kernel-trace run skips the 2/4/8-GPU model legs (--model-worlds ''): their shadow rank
# processes would load the profiler too; the bench line itself comes from the plain run.
set -o pipefail
out=${1:-gpurun_out/round}
rnd=${2:-r03}
mkdir -p "$out" "profiles/$rnd"
R=$GRAFT_REPO_ROOT
PASSES="fetch write l2" bash tools/pmc_dp.sh "$out/pmc" || exit $?
python3 tools/pmc_json.py "$out/pmc" "profiles/$rnd/pmc_9mer.json" 5 > "$out/pmc_9mer.json" || exit $?
echo "pmc done"
timeout -k 10 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || exit $?
echo "bench done"; tail -c 600 "$out/bench.json"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$out/prof" -o run -- python3 "$R/bench.py" --model-worlds '' > "$R/$out/prof_bench.json" 2> "$R/$out/prof.err" ) || exit $?
echo "kernel-trace done"
