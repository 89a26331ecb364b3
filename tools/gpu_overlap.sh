#!/bin/bash
# tools/overlap.py at several grid splits.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/overlap.log
for cfg in "1 2 staged" "2 1 staged" "1 1 staged" "5 0 staged" "0 3 staged" "1 1 split"; do
  set -- $cfg
  timeout -k 10 120 python3 tools/overlap.py --small-per-cu $1 --big-per-cu $2 --big-kernel $3 >> gpurun_out/overlap.log 2>&1 || { tail -5 gpurun_out/overlap.log; exit 11; }
done
grep '^{' gpurun_out/overlap.log
