mkdir -p gpurun_out
DK_TCP_WALK=lane timeout -k 10 200 python -u tools/tcpbench.py --nseg 1048576 --nconns 32768 65536 262144 --cpu-seconds 0.1 > gpurun_out/th_lane.log 2>&1 &&
DK_TCP_WALK=wave timeout -k 10 200 python -u tools/tcpbench.py --nseg 1048576 --nconns 32768 65536 262144 --cpu-seconds 0.1 > gpurun_out/th_wave.log 2>&1
