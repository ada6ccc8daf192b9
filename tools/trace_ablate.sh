set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in 0 1 2; do
  KP_DEBUG_SKIP=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr$v -o run -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-full-cv > $R/gpurun_out/tr$v.log 2>&1 || exit 1
  echo "trace $v done"
done
