#!/bin/bash
# GPU box: the receive parity tests against a tuning build (VARIANT=build/variants/<name>.so copied over the in-tree
# library of this scratch copy), then an interleaved A/B of build/variants/*.so on IMIX / C2 / C5 / C3.
set -o pipefail
mkdir -p gpurun_out
cp "$VARIANT" demikernel_amd/libdk_rx.so || exit 2
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "${TESTK:-not full_size}" > gpurun_out/vt_tests.log 2>&1 || { tail -30 gpurun_out/vt_tests.log; exit 11; }
tail -2 gpurun_out/vt_tests.log
WLS=${WLS:-c4_imix c2_tcp1500 c5_tcp1500_10k} REPS=${REPS:-7} SKIP_C3=1 bash tools/gpu_exp.sh
