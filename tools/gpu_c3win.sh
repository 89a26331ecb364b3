#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "small or kernel_variants or full_size_c3 or random_batches or counter or golden or corpus or nic_offsets or aligned_traffic or misaligned" > gpurun_out/w_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/w_tests.log; exit 11; }
tail -2 gpurun_out/w_tests.log
bash tools/gpu_ab_quick.sh
