#!/bin/bash
# PMC traffic record of the 11-mer config (BASELINE configs[4], ANNNNMNNNNA, 5 lanes per
# step) for bench.py --config 11mer's roofline.traffic, plus its kernel-trace stats.
# usage: tools/profile_11mer.sh OUTDIR ROUND
set -o pipefail
out=${1:-gpurun_out/p11}
rnd=${2:-r03}
mkdir -p "$out" "profiles/$rnd"
R=$GRAFT_REPO_ROOT
PASSES="fetch write l2" BENCH_ARGS="--config 11mer" bash tools/pmc_dp.sh "$out/pmc" || exit $?
python3 tools/pmc_json.py "$out/pmc" "profiles/$rnd/pmc_11mer.json" 5 ANNNNMNNNNA > "$out/pmc_11mer.json" || exit $?
echo "pmc done"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$out/prof" -o run -- python3 "$R/bench.py" --config 11mer --no-cpu-baseline --no-full-cv \
    > "$R/$out/prof_bench.json" 2> "$R/$out/prof.err" ) || exit $?
echo "kernel-trace done"
