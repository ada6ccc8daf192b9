#!/bin/bash
# The persistent 1-lane sweep (kp_dp_ws.h) on the GPU box (tool): A/B against kp_dp_kernel
# with a sampled bit-for-bit comparison (tools/ws_ab.py), then the parity suite of small
# lattices.  usage: tools/ws_check.sh TAG [PATTERNS...]
tag=${1:-ws}
shift
out=gpurun_out/r06
mkdir -p $out
timeout -k 10 500 python tools/ws_ab.py "$@" > $out/ws_ab_$tag.txt 2>&1
rc=$?
cat $out/ws_ab_$tag.txt | tail -5
[ $rc -eq 0 ] || exit $rc
KP_WS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $out/ws_parity_$tag.txt 2>&1
rc=$?
tail -3 $out/ws_parity_$tag.txt
[ $rc -eq 0 ] || exit $rc
# every device group 1 lane wide: the sweep of every lattice above high level 0 on kp_dp_ws.h
KP_WS=1 KP_LANES_PER_WG=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 \
    --timeout-method thread > $out/ws_parity1lane_$tag.txt 2>&1
tail -8 $out/ws_parity1lane_$tag.txt
