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

# TPACKET_V3 path: the next block group's scan overlapped with the current group's pipeline
V=build/variants
H=demikernel_amd/libdk_rx.so
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step t_ring 300 $PYT tests/test_gpu_parity.py -k tpacket3
step gputest 900 $PYT -m gpu tests
step ring_ab 400 python3 tools/ring_ab.py --lib $H --lib $V/ringprev.so --reps 5 --frames 262144
step ring_ab2 400 python3 tools/ring_ab.py --lib $H --lib $V/ringprev.so --reps 5 --frames 1048576
echo done
