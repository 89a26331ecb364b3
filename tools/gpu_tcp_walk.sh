mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tcp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_tests.log 2>&1 &&
DK_TCP_WALK=lane timeout -k 10 200 python -u tools/tcpbench.py --nseg 1048576 --nconns 16384 4096 1024 256 64 1 --cpu-seconds 0.2 > gpurun_out/t_lane.log 2>&1 &&
DK_TCP_WALK=wave timeout -k 10 200 python -u tools/tcpbench.py --nseg 1048576 --nconns 16384 4096 1024 256 64 1 --cpu-seconds 0.2 > gpurun_out/t_wave.log 2>&1
