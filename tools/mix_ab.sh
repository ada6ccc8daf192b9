#!/bin/bash
for r in 1 2; do
for lib in kmerpapa_amd/libkmerpapa_hip.so kmerpapa_amd/libkp_mixhz.so kmerpapa_amd/libkp_mixmerged.so; do
  echo "== $lib"
  KMERPAPA_LIB=$lib timeout -k 10 120 python3 tools/lanes_exp.py 5 m2,3 m4,1 || exit $?
done; done
