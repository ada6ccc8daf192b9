#!/bin/bash
# Each mode of tools/async_oom in a fresh process; records its output and exit status.
# usage: tools/async_oom.sh OUTFILE
out=${1:-gpurun_out/async_oom.txt}
for mode in ${MODES:-malloc oom after grown regrown}; do
  timeout -k 10 60 tools/async_oom "$mode" 400 >> "$out" 2>&1
  rc=$?
  echo "{\"mode\": \"$mode\", \"exit_status\": $rc}" >> "$out"
  case $rc in 0|134|6) ;; *) exit $rc;; esac  # an abort is the finding; anything else stops
done
