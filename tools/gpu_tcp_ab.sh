#!/bin/bash
# TCP walk A/B (GPU box): tests with the in-tree library, then tcpbench with it and with build/old.so swapped in.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tcp.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tcp_tests.log 2>&1 || { tail -20 gpurun_out/tcp_tests.log; exit 11; }
tail -1 gpurun_out/tcp_tests.log
timeout -k 10 300 python3 tools/tcpbench.py --nseg 1048576 --nconns 1 16 64 256 1024 16384 --iters 5 --cpu-seconds 0.02 > gpurun_out/tcp_new.log 2>&1 || { tail -5 gpurun_out/tcp_new.log; exit 12; }
cp build/old.so demikernel_amd/libdk_rx.so
timeout -k 10 300 python3 tools/tcpbench.py --nseg 1048576 --nconns 1 16 64 256 1024 16384 --iters 5 --cpu-seconds 0.02 > gpurun_out/tcp_old.log 2>&1 || { tail -5 gpurun_out/tcp_old.log; exit 13; }
echo NEW; cat gpurun_out/tcp_new.log; echo OLD; cat gpurun_out/tcp_old.log
