#!/bin/bash
# Interleaved A/B of build/variants/*.so: C3 (8 rotating batches), then the other workloads given as args.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --iters 16 build/variants/*.so > gpurun_out/abq_c3.log 2>&1 || { tail -5 gpurun_out/abq_c3.log; exit 12; }
grep '^{' gpurun_out/abq_c3.log
for wl in "$@"; do
  timeout -k 10 200 python3 tools/abtest.py --workload $wl --grids 0 build/variants/*.so > gpurun_out/abq_$wl.log 2>&1 || { tail -5 gpurun_out/abq_$wl.log; exit 13; }
  grep '^{' gpurun_out/abq_$wl.log
done
