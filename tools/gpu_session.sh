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

# 1. the GPU suite, smoke() and the bench line at this build
step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python3 bench.py --gpus 1 --steps 20 --warmup 5
# 2. rocprofv3 evidence: kernel stats of the bench, FETCH/WRITE traffic per workload, C1/C3/TX/TCP kernel stats
step profile 1000 bash tools/profile_bench.sh $TAG
# 3. SQ counters of the kernels changed this round: C1 (staged now), C3 (priority + early descriptors)
step sq_c1 300 bash tools/pmc_kernel.sh c1_tcp1078 ${TAG}_c1 --defer --rotate 3
step sq_c3 300 bash tools/pmc_kernel.sh c3_udp64 ${TAG}_c3 --defer --rotate 8
echo done
