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

# r05zj: grids that give every wave the same number of chunks (C3: 16,384 chunks; 683 workgroups x 8 waves = 3
# chunks each, 512 x 8 = 4 each; the rule's 768 leaves a third of the waves a chunk short) and for IMIX
step ab_c3 300 python tools/abtest.py --workload c3_udp64 --rotate 8 --defer --grids 0 --knob DK_RX_GRID=-1,683,640,512,768 --iters 20 --reps 9 demikernel_amd/libdk_rx.so
step ab_c3r 300 python tools/abtest.py --workload c3_udp64_random_ports --rotate 8 --defer --grids 0 --knob DK_RX_GRID=-1,683,512 --iters 20 --reps 9 demikernel_amd/libdk_rx.so
step ab_imix 300 python tools/abtest.py --workload c4_imix --rotate 2 --defer --grids 0 --knob DK_RX_GRID=-1,745,683,640 --iters 10 --reps 7 demikernel_amd/libdk_rx.so
echo done
