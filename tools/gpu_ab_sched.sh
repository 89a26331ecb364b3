#!/bin/bash
# Schedule A/B (GPU box): parity under sched 2, then interleaved timing of sched 0/1/2 x grids on the big-frame workloads.
set -o pipefail
mkdir -p gpurun_out
DK_RX_SCHED=2 timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/par_s2.log 2>&1 || exit 11
for wl in c2_tcp1500 c5_tcp1500_10k c4_imix; do
  timeout -k 10 240 python3 tools/abtest.py --workload $wl --grids 2,3,4 --scheds 0,1,2 build/variants/*.so > gpurun_out/ab_$wl.log 2>&1 || exit 12
done
echo done
