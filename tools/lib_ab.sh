#!/bin/bash
# A/B of library builds with tools/lanes_exp.py (tool): ROUNDS rounds, each library in turn
# in a fresh process.  usage: tools/lib_ab.sh ROUNDS "LIB1 LIB2 ..." COMP...
rounds=$1; libs=$2; shift 2
for r in $(seq "$rounds"); do
  for lib in $libs; do
    echo "== $lib"
    KMERPAPA_LIB=$lib timeout -k 10 150 python3 tools/lanes_exp.py "$@" || exit $?
  done
done
