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

# r05l: the wave walk streams few-connection batches through LDS rings (LDS-DMA); partial retransmissions on the
# parallel check. TCP GPU tests, the 1 / 64 / 16k connection rates, kernel stats of the 1-connection case
step tcptest 600 python -u -m pytest tests/test_gpu_tcp.py -m gpu -x -q --timeout 300 --timeout-method thread
step tcp1 300 python tools/tcpbench.py --nconns 1 --buffer-size 1073741824 --reorder 0 --iters 10
step tcpn 300 python tools/tcpbench.py --nconns 64 16384 --iters 10 --cpu-seconds 0.5
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $O/prof1 -o run --output-format csv -- \
  python3 $R/tools/tcpbench.py --nconns 1 --buffer-size 1073741824 --reorder 0 --iters 10 --cpu-seconds 0.2 > $O/prof1.log 2>&1 || exit 11
echo done
