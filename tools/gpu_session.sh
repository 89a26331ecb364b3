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

# r06c: staging kernel with the first chunk's descriptors loaded before the LDS init / table copy / barrier (ed.so)
step ab_c1 300 python tools/abtest.py --workload c1_tcp1078 --rotate 3 --defer --grids 0 --check --iters 20 --reps 11 demikernel_amd/libdk_rx.so build/variants/ed.so
step ab_imix 300 python tools/abtest.py --workload c4_imix --rotate 2 --defer --grids 0 --check --iters 10 --reps 9 demikernel_amd/libdk_rx.so build/variants/ed.so
echo done
