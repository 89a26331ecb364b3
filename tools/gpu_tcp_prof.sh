mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
DK_TCP_WALK=wave timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof_wave -o run -- python3 tools/tcpbench.py --nseg 1048576 --nconns 256 --iters 3 --cpu-seconds 0.1 > gpurun_out/tprof_wave.log 2>&1 &&
DK_TCP_WALK=lane timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof_lane -o run -- python3 tools/tcpbench.py --nseg 1048576 --nconns 256 --iters 3 --cpu-seconds 0.1 > gpurun_out/tprof_lane.log 2>&1
