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

# grid shape re-check after this round's changes (deferred counters, priorities)
step imix 300 python3 tools/tune_ab.py --workload c4_imix --reps 7 "defer=1" "defer=1,grid_per_cu=2" "defer=1,sched=1"
step c3 300 python3 tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 9 "defer=1" "defer=1,grid_per_cu=4"
step c1 300 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 9 "defer=1" "defer=1,grid_per_cu=1" "defer=1,sched=1"
echo done
