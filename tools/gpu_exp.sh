#!/bin/bash
# Interleaved A/B of build/variants/*.so (no tests): C3 (8 rotating batches), then IMIX / C5 / C2; an optional
# KNOB=NAME=v1,v2 interleaves values of one env knob on every workload (e.g. DK_RX_LDS_TABLE=0,1).
set -o pipefail
mkdir -p gpurun_out
K=""; [ -n "$KNOB" ] && K="--knob $KNOB"
[ "$SKIP_C3" = 1 ] || timeout -k 10 300 python3 tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --iters 16 --reps ${REPS:-9} $K build/variants/*.so > gpurun_out/ab_c3.log 2>&1 || { tail -5 gpurun_out/ab_c3.log; exit 12; }
[ "$SKIP_C3" = 1 ] || grep "^{" gpurun_out/ab_c3.log
for wl in ${WLS:-c4_imix c5_tcp1500_10k c2_tcp1500}; do
  timeout -k 10 300 python3 tools/abtest.py --workload $wl --grids 0 --iters 10 --reps ${REPS:-7} $K build/variants/*.so > gpurun_out/ab_$wl.log 2>&1 || { tail -5 gpurun_out/ab_$wl.log; exit 13; }
  grep '^{' gpurun_out/ab_$wl.log
done
