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

# 1. the bench line exactly as the driver runs it, then the collective-overlap check (1-rank RCCL communicator)
step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
step overlap 300 python3 tools/overlap_collective.py --out $O/r04_overlap.json
# 2. SQ counter passes (3 runs each, <= 8 SQ counters per run) of the C1 / C3 / C4 kernels, deferred counters
step sq_c1 300 bash tools/pmc_kernel.sh c1_tcp1078 ${TAG}_c1 --rotate 3 --defer
step sq_c3 300 bash tools/pmc_kernel.sh c3_udp64 ${TAG}_c3 --rotate 8 --defer
step sq_c4 300 bash tools/pmc_kernel.sh c4_imix ${TAG}_c4 --defer
echo done
