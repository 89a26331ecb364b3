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

# r05w: the small kernel with 8 waves per workgroup as the default build: GPU suite, then C3 A/B against the 4-wave
# build (results compared)
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step ab_c3 300 python tools/abtest.py --workload c3_udp64 --rotate 8 --defer --grids 0 --iters 20 --reps 15 --check build/variants/sw4.so demikernel_amd/libdk_rx.so
step ab_c3r 300 python tools/abtest.py --workload c3_udp64_random_ports --rotate 8 --defer --grids 0 --iters 20 --reps 15 build/variants/sw4.so demikernel_amd/libdk_rx.so
echo done
