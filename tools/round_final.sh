#!/bin/bash
# The round's last measurement run on one GPU box, from the repo root (tool):
#   gpu_tests.txt   pytest -m gpu (the driver's round-end suite)
#   smoke.txt       __graft_entry__.smoke()
#   <round>/...     tools/round_profile.sh: PMC passes + pmc_9mer.json, bench.json, kernel trace
#   bench_11mer     bench.py --config 11mer (after its PMC record, tools/profile_11mer.sh)
#   cli_9mer.json   the whole CLI on the 9-mer counts (tools/cli_9mer.py)
# usage: tools/round_final.sh OUTDIR ROUND
set -o pipefail
out=${1:-gpurun_out/final}
rnd=${2:-r04}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 1500 --timeout-method thread > "$out/gpu_tests.txt" 2>&1 || exit $?
echo "gpu tests done"; tail -1 "$out/gpu_tests.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit $?
echo "smoke done"
bash tools/round_profile.sh "$out/p9" "$rnd" || exit $?
bash tools/profile_11mer.sh "$out/p11" "$rnd" || exit $?
timeout -k 10 500 python bench.py --config 11mer > "$out/bench_11mer.json" 2> "$out/bench_11mer.err" || exit $?
echo "bench 11mer done"
timeout -k 10 300 python tools/cli_9mer.py > "$out/cli_9mer.json" 2> "$out/cli_9mer.err" || exit $?
echo "cli done"
