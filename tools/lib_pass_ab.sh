#!/bin/bash
# Library builds' 1-lane passes, alternating (tool): tools/lib_pass_ab.py under each build
# of the comma list LIBS, two rounds, lines appended to $out/lib_pass_ab.txt.
# usage: tools/lib_pass_ab.sh LIB[,LIB...] LANES GEN_PAT [GEN_PAT ...]
out=gpurun_out/r06
mkdir -p $out
LIBS=$1; NL=$2; shift 2
for rep in 1 2; do
  for lib in ${LIBS//,/ }; do
    KMERPAPA_LIB=$lib timeout -k 10 300 python tools/lib_pass_ab.py $NL "$@" >> $out/lib_pass_ab.txt || exit $?
  done
done
cat $out/lib_pass_ab.txt
