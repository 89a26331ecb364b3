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

# r06f: rocPRIM onesweep configs for the TCP sort (s8b: 8 bits/pass 256x24; s6a: 6 bits/pass 512x16) vs the default
step probe 300 python tools/tcp_walk_probe.py --nconns 16384 1 --walks wave scan --iters 7 --libs demikernel_amd/libdk_rx.so build/variants/s8b.so build/variants/s6a.so
echo done
