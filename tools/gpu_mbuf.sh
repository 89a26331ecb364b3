#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mbuf" > gpurun_out/mbuf_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/mbuf_tests.log; exit 11; }
tail -2 gpurun_out/mbuf_tests.log
timeout -k 10 200 python -c "
import sys, json, torch
sys.path.insert(0, '.')
import bench
torch.cuda.set_device(0)
print(json.dumps(bench.mbuf_zero_copy_rate(0, torch.cuda.current_stream(0))))
" > gpurun_out/mbuf_rate.log 2>&1 || { tail -5 gpurun_out/mbuf_rate.log; exit 12; }
tail -1 gpurun_out/mbuf_rate.log
