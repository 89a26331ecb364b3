#!/bin/bash
# Development check: targeted parity tests (TESTK) on the default build, then the A/B of build/variants/*.so.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tcp.py -m gpu -x -v --timeout 250 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/dev_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/dev_tests.log; exit 11; }
tail -2 gpurun_out/dev_tests.log
tools/gpu_ab_all.sh
