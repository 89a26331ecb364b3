#!/bin/bash
# The current GPU session's measurement steps (rewritten per gpurun call; each step has its own time limit and the
# script stops at the first failure). Run from the repo root on the GPU box: bash tools/gpu_session.sh <tag>
set -o pipefail
TAG=${1:-s}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stdout+stderr to $O/<name>.log
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -h '^{' $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -20 $O/$name.log; exit 10; fi
}
export TMPDIR=/tmp

# r06h: medium frames of <= 640 B streamed by 8 lanes, 8 per step (med8.so) vs 16 lanes, 4 per step
step ab_imix 300 python tools/abtest.py --workload c4_imix --rotate 2 --defer --grids 0 --check --iters 10 --reps 9 demikernel_amd/libdk_rx.so build/variants/med8.so
step ab_imix1 300 python tools/abtest.py --workload c4_imix --rotate 1 --defer --grids 0 --iters 10 --reps 7 demikernel_amd/libdk_rx.so build/variants/med8.so
step ab_c1 300 python tools/abtest.py --workload c1_tcp1078 --rotate 3 --defer --grids 0 --check --iters 20 --reps 9 demikernel_amd/libdk_rx.so build/variants/med8.so
step ab_c2 300 python tools/abtest.py --workload c2_tcp1500 --defer --grids 0 --check --iters 10 --reps 7 demikernel_amd/libdk_rx.so build/variants/med8.so
step ab_tx 300 python tools/abtest.py --workload c2_tcp1500 --tx --grids 0 --iters 10 --reps 7 demikernel_amd/libdk_rx.so build/variants/med8.so
echo done
