# Experiment: sweep-kernel time for tiled block orders (KP_BLOCK_TILE); run on the GPU box from the repo root.
mkdir -p gpurun_out/tiles
for T in 0 8 5 4 3 6; do
  KP_BLOCK_TILE=$T timeout -k 10 120 python3 bench.py > gpurun_out/tiles/t$T.json 2> gpurun_out/tiles/t$T.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/tiles/t$T.json').read().strip().splitlines()[-1]); print('$T', d['ms_per_step'], d['dp_kernel_ms_per_step'])"
done
