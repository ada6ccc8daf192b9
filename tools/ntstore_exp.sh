# Experiment: non-temporal score-row stores (KP_NT_STORE); run on the GPU box from the repo root.
mkdir -p gpurun_out/nt
for v in 0 1 0 1; do
  KP_NT_STORE=$v timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-full-cv > gpurun_out/nt/nt$v.json 2> gpurun_out/nt/nt$v.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/nt/nt$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['dp_kernel_ms_per_step'], d['value'])"
done
