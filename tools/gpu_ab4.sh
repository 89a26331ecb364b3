#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or kernel_variants or full_size or c5 or random_batches or golden or corpus or options or small or misaligned or nic" > gpurun_out/s_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/s_tests.log; exit 11; }
tail -2 gpurun_out/s_tests.log
for wl in "$@"; do
  timeout -k 10 200 python3 tools/abtest.py --workload $wl --grids 0 --reps 9 build/variants/*.so > gpurun_out/ab4_$wl.log 2>&1 || { tail -5 gpurun_out/ab4_$wl.log; exit 13; }
  grep '^{' gpurun_out/ab4_$wl.log
done
