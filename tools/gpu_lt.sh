#!/bin/bash
# LDS Active table: parity tests, then interleaved A/B of the table on/off (DK_RX_LDS_TABLE) on IMIX, C2 and C5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 250 --timeout-method thread -k "${TESTK:-lds_active or kernel_variants or random_batches or full_size or c5 or corpus}" > gpurun_out/lt_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/lt_tests.log; exit 11; }
tail -2 gpurun_out/lt_tests.log
for wl in ${WORKLOADS:-c4_imix c2_tcp1500 c5_tcp1500_10k}; do
  timeout -k 10 200 python3 tools/abtest.py --workload $wl --grids 0 --iters 10 --reps ${REPS:-9} --knob DK_RX_LDS_TABLE=-1,0 demikernel_amd/libdk_rx.so > gpurun_out/ab_lt_$wl.log 2>&1 || { tail -5 gpurun_out/ab_lt_$wl.log; exit 12; }
  grep '^{' gpurun_out/ab_lt_$wl.log
done
