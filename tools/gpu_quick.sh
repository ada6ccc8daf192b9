#!/bin/bash
# Quick GPU check of a kernel change: the parity suites that compare every cell with the
# oracle, then the lane-composition timing (tools/lanes_exp.py).  usage: tools/gpu_quick.sh TAG
tag=${1:-quick}
out=gpurun_out/r02
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_bruteforce.py -m gpu -x -q \
    --timeout 600 --timeout-method thread > $out/gpu_tests_$tag.txt 2>&1
rc=$?
tail -2 $out/gpu_tests_$tag.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/lanes_exp.py > $out/lanes_$tag.txt 2>&1 || exit $?
cat $out/lanes_$tag.txt
