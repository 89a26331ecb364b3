#!/bin/bash
# TX (and RX C2) A/B of build/variants/*.so.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/abtest.py --workload c2_tcp1500 --tx --grids 0 --iters 10 --reps ${REPS:-9} build/variants/*.so > gpurun_out/tx_ab.log 2>&1 || { tail -5 gpurun_out/tx_ab.log; exit 12; }
[ -n "$TXONLY" ] || timeout -k 10 300 python3 tools/abtest.py --workload c2_tcp1500 --grids 0 --iters 10 --reps ${REPS:-9} build/variants/*.so >> gpurun_out/tx_ab.log 2>&1 || { tail -5 gpurun_out/tx_ab.log; exit 13; }
grep '^{' gpurun_out/tx_ab.log
