# Experiment: sweep-kernel time against threads per workgroup (KP_DP_THREADS) and lanes per
# workgroup (KP_LANES_PER_WG); run on the GPU box from the repo root.
mkdir -p gpurun_out/occ
for spec in "512 5" "1024 5" "256 5" "512 4" "512 3" "1024 3"; do
  set -- $spec
  KP_DP_THREADS=$1 KP_LANES_PER_WG=$2 timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-full-cv > gpurun_out/occ/t$1_l$2.json 2> gpurun_out/occ/t$1_l$2.err
  rc=$?
  case $rc in 0|1) ;; *) echo "stop rc=$rc"; exit $rc;; esac
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/occ/t$1_l$2.json').read().strip().splitlines()[-1]); print('$1 $2', d['ms_per_step'], d['dp_kernel_ms_per_step'], d['value'])" || tail -2 gpurun_out/occ/t$1_l$2.err
done
