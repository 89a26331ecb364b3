#!/bin/bash
# GPU parity suite (receive path) then an interleaved A/B of build/variants/*.so on C3, IMIX, C5, C2.
set -o pipefail
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 11; }
  tail -2 gpurun_out/tests.log
fi
timeout -k 10 300 python3 tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --iters 16 --reps 9 build/variants/*.so > gpurun_out/ab_c3.log 2>&1 || { tail -5 gpurun_out/ab_c3.log; exit 12; }
grep '^{' gpurun_out/ab_c3.log
for wl in ${WLS:-c4_imix c5_tcp1500_10k c2_tcp1500}; do
  timeout -k 10 300 python3 tools/abtest.py --workload $wl --grids 0 --iters 10 --reps 7 build/variants/*.so > gpurun_out/ab_$wl.log 2>&1 || { tail -5 gpurun_out/ab_$wl.log; exit 13; }
  grep '^{' gpurun_out/ab_$wl.log
done
