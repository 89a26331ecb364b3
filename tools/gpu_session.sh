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

# r06u: reordered runs resolved from the arrival order (chain_run) with a DPP / swizzle bitonic sort
step tcptest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py
step probe 300 python tools/tcp_walk_probe.py --nconns 1 16 64 256 --walks scan wave --streams clean default bench --iters 7
echo done
