#!/bin/bash
# Shapes of the persistent 1-lane sweep (tool): tools/ws_ab.py on each prebuilt variant
# library (kmerpapa_amd/libkmerpapa_hip_ws<V>.so), then the phase ablation of the sweep
# with KP_WS=1 (timing-ablation build).  usage: tools/ws_variants.sh TAG VARIANTS...
tag=${1:-v}
shift
out=gpurun_out/r06
mkdir -p $out
for v in "$@"; do
    echo "== variant $v" >> $out/ws_variants_$tag.txt
    KMERPAPA_LIB=kmerpapa_amd/libkmerpapa_hip_ws$v.so timeout -k 10 300 python tools/ws_ab.py NNNNMNNNN \
        >> $out/ws_variants_$tag.txt 2>&1 || exit $?
done
KP_WS=1 ABLATE_LANES=1 KMERPAPA_LIB=kmerpapa_amd/libkmerpapa_hip_ablation.so timeout -k 10 300 \
    python tools/ablate.py 0 1 2 3 > $out/ws_ablate_$tag.txt 2>&1 || exit $?
cat $out/ws_variants_$tag.txt $out/ws_ablate_$tag.txt
