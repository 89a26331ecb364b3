#!/bin/bash
# Small-frame stream/finish kernel: parity with it forced on, then C3 A/B.
set -o pipefail
mkdir -p gpurun_out
DK_RX_SMALL=${SMALL:-2} timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or random or corpus or options or fuzz or full_size_c3 or small or counter or empty" > gpurun_out/ss_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/ss_tests.log; exit 11; }
tail -2 gpurun_out/ss_tests.log
timeout -k 10 300 python3 tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --iters 16 --reps 11 --knob DK_RX_SMALL=${KNOB:-1,2} build/variants/*.so > gpurun_out/ss_ab.log 2>&1 || { tail -5 gpurun_out/ss_ab.log; exit 12; }
grep '^{' gpurun_out/ss_ab.log
