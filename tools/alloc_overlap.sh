#!/bin/bash
# tools/alloc_overlap right after a 200 GB process exit (tool; one GPU box)
set -e
timeout -k 5 60 ./tools/alloc_once 200 w
timeout -k 5 60 ./tools/alloc_overlap 40 150
