#!/bin/bash
# A/B pass timing of launch-knob settings of one library build (tool): for each round,
# every setting in turn runs tools/pass_once.py with the given lane compositions in a
# fresh process.  usage: tools/env_ab.sh ROUNDS "K=V[,K=V] K=V ..." COMP...
#   (e.g. 3 "KP_HPD=0 KP_HPD=1" 5 1)
rounds=$1; sets=$2; shift 2
for r in $(seq "$rounds"); do
  for st in $sets; do
    echo "== $st"
    env $(echo "$st" | tr ',' ' ') timeout -k 10 120 python3 tools/pass_once.py "$@" || exit $?
  done
done
