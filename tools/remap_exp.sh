# Experiment: XCD run length (KP_XCD_REMAP) with the current sweep; run on the GPU box from the repo root.
mkdir -p gpurun_out/remap
for G in 8 4 16 0; do
  KP_XCD_REMAP=$G timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-full-cv > gpurun_out/remap/g$G.json 2> gpurun_out/remap/g$G.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/remap/g$G.json').read().strip().splitlines()[-1]); print('$G', d['ms_per_step'], d['dp_kernel_ms_per_step'])"
done
