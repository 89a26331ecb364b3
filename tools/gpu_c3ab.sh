#!/bin/bash
# C3 work: small-kernel parity tests on the default build, then an interleaved C3 A/B of build/variants/*.so.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "${TESTK:-small or udp64 or c3 or variants or fuzz or corpus or golden or offload or misaligned or counter or streams}" > gpurun_out/c3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/c3_tests.log; exit 11; }
tail -2 gpurun_out/c3_tests.log
timeout -k 10 300 python3 tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --iters 16 --reps ${REPS:-9} build/variants/*.so > gpurun_out/ab_c3.log 2>&1 || { tail -5 gpurun_out/ab_c3.log; exit 12; }
grep '^{' gpurun_out/ab_c3.log
