#!/bin/bash
# Split kernel with 2 finishers per stream wave: parity with it forced on, then IMIX/C2 A/B against staged / split-1.
set -o pipefail
mkdir -p gpurun_out
DK_RX_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "golden or random or full_size or imix or corpus or options" > gpurun_out/s2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/s2_tests.log; exit 11; }
tail -2 gpurun_out/s2_tests.log
timeout -k 10 300 python3 tools/abtest.py --workload c4_imix --grids 0 --iters 16 --reps 11 --knob DK_RX_SPLIT=0,1,2 build/variants/cur.so > gpurun_out/s2_ab.log 2>&1 || { tail -5 gpurun_out/s2_ab.log; exit 12; }
timeout -k 10 300 python3 tools/abtest.py --workload c2_tcp1500 --grids 0 --iters 16 --reps 7 --knob DK_RX_SPLIT=1,2 build/variants/cur.so >> gpurun_out/s2_ab.log 2>&1 || { tail -5 gpurun_out/s2_ab.log; exit 13; }
grep '^{' gpurun_out/s2_ab.log
