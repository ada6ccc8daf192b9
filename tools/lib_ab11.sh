#!/bin/bash
# One box, two library builds, alternating (tool): the 11-mer and 9-mer bench steps of
# kmerpapa_amd/libkmerpapa_hip_r05.so (round 5's sources) and of the current build.
out=gpurun_out/r06
mkdir -p $out
for rep in 1 2; do
  for lib in kmerpapa_amd/libkmerpapa_hip_r05.so kmerpapa_amd/libkmerpapa_hip.so; do
    for cfg in 11mer 9mer; do
      KMERPAPA_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 5 --no-cpu-baseline --no-full-cv \
          > $out/lib_ab.tmp 2>/dev/null || exit $?
      python -c "import json,sys; d=json.loads(open('$out/lib_ab.tmp').read().strip().splitlines()[-1]); print('$rep', '$lib', '$cfg', round(d['ms_per_step'], 2), round(d['roofline']['kernel_ms_per_pass'], 2))" >> $out/lib_ab11.txt
    done
  done
done
cat $out/lib_ab11.txt
