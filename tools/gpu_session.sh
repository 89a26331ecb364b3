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

# r06a: scan walk in one loop: batches resume once the state is the call-start one again; the slow window's next
# batch loading behind it. TCP GPU tests, the probe, the bench's reordered shapes (scan vs wave)
step tcptest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tcp.py
step probe 300 python tools/tcp_walk_probe.py --nconns 1 16 64 256 --walks scan --iters 7
step s64 300 env DK_TCP_WALK=scan python tools/tcpbench.py --nconns 64 16 --cpu-seconds 0.2
step w64 300 env DK_TCP_WALK=wave python tools/tcpbench.py --nconns 64 16 --cpu-seconds 0.2
echo done
