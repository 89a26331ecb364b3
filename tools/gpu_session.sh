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

# r05zw: the bench's TCP lines' shapes (reordered streams, 16 MiB windows) per walk: 64 and 16 connections
step w64 300 env DK_TCP_WALK=wave python tools/tcpbench.py --nconns 64 16 --cpu-seconds 0.2
step r64 300 env DK_TCP_WALK=relay python tools/tcpbench.py --nconns 64 16 --cpu-seconds 0.2
step s64 300 env DK_TCP_WALK=scan python tools/tcpbench.py --nconns 64 16 --cpu-seconds 0.2
echo done
