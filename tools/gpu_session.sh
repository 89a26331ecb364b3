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

# r06i: per-wave timelines of the staging kernel at the final sources (-DDK_DIAG_STAMPS build): IMIX with 2 rotating
# batches, the default dynamic tail and without it; C1
step st_imix 120 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2
step st_imix_t0 120 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2 --tuning tail=0
step st_c1 120 python tools/stamps_staged.py build/variants/stamps.so --workload c1_tcp1078 --rotate 3
echo done
