set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/abtest.py --workload c2_tcp1500 --grids 2,3,4,5 build/variants/*.so > gpurun_out/ab_s1.log 2>&1 &&
DK_RX_SCHED=0 timeout -k 10 200 python3 tools/abtest.py --workload c2_tcp1500 --grids 2,3,4,5 build/variants/*.so > gpurun_out/ab_s0.log 2>&1 &&
timeout -k 10 200 python3 tools/kbench.py --workload c2_tcp1500 --iters 20 --probe --no-rx > gpurun_out/probe.log 2>&1
