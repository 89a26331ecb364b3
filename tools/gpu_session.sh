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

# r05zh: IMIX (2 rotating batches) on the split kernel (stream + finish waves) vs the staging kernel, and the
# contiguous schedule (sched 1) vs round-robin tiles
step ab_imix 300 python tools/abtest.py --workload c4_imix --rotate 2 --defer --grids 0 --scheds 0,1 --knob DK_RX_SPLIT=0,1 --iters 10 --reps 7 demikernel_amd/libdk_rx.so
echo done
