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

# r05c: the dynamic tail without stealing (own-XCD pool only)
# deferred counters as the bench runs them), then per-wave exit timelines with and without the tail
step parity 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "dynamic_tail or kernel_variants or full_size_c4 or packed_layouts or deferred or golden"
step ab_imix 600 python tools/tune_ab.py --workload c4_imix --rotate 2 --reps 7 --iters 20 "defer=1,tail=0" "defer=1,tail=1" "defer=1,tail=2" "defer=1,tail=3" "defer=1,tail=4"
step ab_imix1 600 python tools/tune_ab.py --workload c4_imix --rotate 1 --reps 5 --iters 20 "defer=1,tail=0" "defer=1,tail=2"
step stamps 600 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2 --tuning tail=0
step stamps_t2 600 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2 --tuning tail=2
echo done
