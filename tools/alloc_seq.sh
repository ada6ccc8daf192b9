#!/bin/bash
# How long does a large allocation wait right after another process freed (exited with)
# 200 GB of written HBM, by its own size; and after a pause?  (tool; one GPU box)
set -e
A="timeout -k 5 60 ./tools/alloc_once"
for gb in 20 80 150; do
  echo "# after a 200 GB process exit: $gb GB"; $A 200 w; $A $gb
  sleep 8
  echo "# after a 200 GB process exit and 4 s: $gb GB"; $A 200 w; sleep 4; $A $gb
  sleep 8
done
