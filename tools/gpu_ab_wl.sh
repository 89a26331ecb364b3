#!/bin/bash
# Interleaved A/B of build/variants/*.so on several workloads (GPU box). usage: tools/gpu_ab_wl.sh "<grids>" wl1 wl2 ...
set -o pipefail
mkdir -p gpurun_out
G=$1; shift
for wl in "$@"; do
  timeout -k 10 240 python3 tools/abtest.py --workload $wl --grids $G build/variants/*.so > gpurun_out/ab_$wl.log 2>&1 || { echo "FAIL $wl"; tail -5 gpurun_out/ab_$wl.log; exit 12; }
  cat gpurun_out/ab_$wl.log
done
