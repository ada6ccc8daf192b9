#!/bin/bash
# Pass times of alternative builds of the library (KMERPAPA_LIB) on the same compositions
# (tools/lanes_exp.py).  usage: tools/libs_exp.sh OUTDIR lib1.so lib2.so ... -- comp1 comp2 ...
out=$1; shift
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done; shift
mkdir -p "$out"
for lib in "${libs[@]}"; do
  echo "== $lib"
  KMERPAPA_LIB=$PWD/$lib timeout -k 10 150 python3 tools/lanes_exp.py "$@" > "$out/$(basename $lib .so).txt" 2>&1 || { cat "$out/$(basename $lib .so).txt"; exit 1; }
  cat "$out/$(basename $lib .so).txt"
done
