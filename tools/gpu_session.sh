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

# init barrier moved past the first chunk: small kernel (bar1/bar2, + wave-uniform verdict check wchk), staged
# kernel (stgbar1), split kernel (splitbar); GPU suite at the tree's build first
V=build/variants
H=demikernel_amd/libdk_rx.so
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step parity 900 python3 -u tools/variant_parity.py --lib $V/bar1.so --lib $V/bar2.so --lib $V/wchk.so --lib $V/bar1w.so \
  --lib $V/stgbar1.so --lib $V/splitbar.so
step ab_c3 400 python3 tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 11 --iters 16 --lib $H --lib $V/bar1.so \
  --lib $V/bar2.so --lib $V/wchk.so --lib $V/bar1w.so "defer=1"
step ab_c1 300 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 9 --iters 20 --lib $H --lib $V/stgbar1.so "defer=1"
step ab_c2 300 python3 tools/tune_ab.py --workload c2_tcp1500 --reps 9 --iters 10 --lib $H --lib $V/splitbar.so "defer=1"
step ab_c4 300 python3 tools/tune_ab.py --workload c4_imix --reps 9 --iters 10 --lib $H --lib $V/stgbar1.so "defer=1"
step ab_c5 300 python3 tools/tune_ab.py --workload c5_tcp1500_10k --reps 5 --iters 8 --lib $H --lib $V/splitbar.so "defer=1"
echo done
