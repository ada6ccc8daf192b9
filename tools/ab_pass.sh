#!/bin/bash
# A/B pass timing of library builds (tool): for each round, every library in turn runs
# tools/pass_once.py with the given lane compositions in a fresh process.
# usage: tools/ab_pass.sh ROUNDS "LIB1 LIB2 ..." COMP...   (e.g. 2 "a.so b.so" 5 5 5 1 1)
rounds=$1; libs=$2; shift 2
for r in $(seq "$rounds"); do
  for lib in $libs; do
    echo "== $lib"
    KMERPAPA_LIB=$lib timeout -k 10 120 python3 tools/pass_once.py "$@" || exit $?
  done
done
