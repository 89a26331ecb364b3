#!/bin/bash
# C3 A/B of build/variants/*.so (no tests).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --iters 16 --reps ${REPS:-9} build/variants/*.so > gpurun_out/ab_c3.log 2>&1 || { tail -5 gpurun_out/ab_c3.log; exit 12; }
grep '^{' gpurun_out/ab_c3.log
