#!/bin/bash
# Interleaved A/B of build/variants/*.so on C3 (8 rotating batches), C2, IMIX and C5 (no tests).
set -o pipefail
mkdir -p gpurun_out
for w in ${WORKLOADS:-c3_udp64 c2_tcp1500 c4_imix c5_tcp1500_10k}; do
  rot=1; [ $w = c3_udp64 ] && rot=8
  it=10; [ $w = c3_udp64 ] && it=16
  timeout -k 10 300 python3 tools/abtest.py --workload $w --grids 0 --rotate $rot --iters $it --reps ${REPS:-7} build/variants/*.so > gpurun_out/ab_$w.log 2>&1 || { tail -5 gpurun_out/ab_$w.log; exit 12; }
  grep '^{' gpurun_out/ab_$w.log
done
