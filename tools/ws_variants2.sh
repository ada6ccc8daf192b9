#!/bin/bash
# tools/ws_variants.sh with a per-variant ablation build (kmerpapa_amd/libkmerpapa_hip_abl_ws<V>.so)
tag=${1:-v}
shift
out=gpurun_out/r06
mkdir -p $out
for v in "$@"; do
    echo "== variant $v" >> $out/ws_variants_$tag.txt
    KMERPAPA_LIB=kmerpapa_amd/libkmerpapa_hip_ws$v.so timeout -k 10 300 python tools/ws_ab.py NNNNMNNNN \
        >> $out/ws_variants_$tag.txt 2>&1 || exit $?
    if [ -f kmerpapa_amd/libkmerpapa_hip_abl_ws$v.so ]; then
        KP_WS=1 ABLATE_LANES=1 KMERPAPA_LIB=kmerpapa_amd/libkmerpapa_hip_abl_ws$v.so timeout -k 10 300 \
            python tools/ablate.py 0 1 2 3 >> $out/ws_variants_$tag.txt 2>&1 || exit $?
    fi
done
cat $out/ws_variants_$tag.txt
