#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "small or kernel_variants or full_size_c3 or random_batches or counter or golden or corpus" > gpurun_out/c3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/c3_tests.log; exit 11; }
tail -2 gpurun_out/c3_tests.log
timeout -k 10 300 python3 tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --iters 16 build/variants/*.so > gpurun_out/ab_c3.log 2>&1 || { tail -5 gpurun_out/ab_c3.log; exit 12; }
grep '^{' gpurun_out/ab_c3.log
