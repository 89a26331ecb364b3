#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or kernel_variants or full_size or c5 or random_batches or golden or corpus or options or small or misaligned or nic" > gpurun_out/s_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/s_tests.log; exit 11; }
tail -2 gpurun_out/s_tests.log
timeout -k 10 300 python3 tools/abtest.py --workload c4_imix --grids 0 --knob DK_RX_SPLIT=0,1 --reps 7 build/variants/cur.so > gpurun_out/abis.log 2>&1 || exit 13
grep '^{' gpurun_out/abis.log
timeout -k 10 300 python3 tools/abtest.py --workload c2_tcp1500 --grids 0 --reps 7 build/variants/cur.so > gpurun_out/abis2.log 2>&1 || exit 14
grep '^{' gpurun_out/abis2.log
