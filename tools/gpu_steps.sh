#!/bin/bash
# Run "name|seconds|command" steps in order; each under its own time limit.  Stop at the
# first step that crashed, aborted or timed out (124/134/137/139 or signals); a plain
# test failure (exit 1) does not stop later steps.
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  case $rc in 0|1|2|5) ;; *) echo "stopping after $name (rc=$rc)"; exit $rc;; esac
done
