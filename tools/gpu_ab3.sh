#!/bin/bash
# A/B of build/variants/*.so on C3, C4 and C2 (no tests).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab3.log
for wl in ${WLS:-c3_udp64 c4_imix c2_tcp1500}; do
  rot=1; [ $wl = c3_udp64 ] && rot=8
  timeout -k 10 300 python3 tools/abtest.py --workload $wl --grids 0 --rotate $rot --iters 16 --reps ${REPS:-9} build/variants/*.so >> gpurun_out/ab3.log 2>&1 || { tail -5 gpurun_out/ab3.log; exit 12; }
done
grep '^{' gpurun_out/ab3.log
