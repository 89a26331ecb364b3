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

# 1. parity: the changed paths first, then the whole GPU suite
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step t_defer 400 $PYT tests/test_gpu_parity.py -k "deferred_counts or counter_rows or kernel_variants or full_size_c1 or full_size_c2"
step t_multi 300 $PYT tests/test_gpu_multiproc.py
step t_all 900 $PYT -m gpu tests
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
# 2. A/B: deferred counters (defer=1, static block assignment) x builds (sr3/sr4: 3/4 rounds per split-kernel step)
V=build/variants
H=demikernel_amd/libdk_rx.so
step ab_c1 300 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 7 --iters 20 --lib $H --lib $V/sr3.so \
  --lib $V/sr4.so "" "defer=1"
step ab_c3 300 python3 tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 9 --iters 16 --lib $H --lib $V/kargs0.so "" "defer=1"
step ab_c2 300 python3 tools/tune_ab.py --workload c2_tcp1500 --reps 7 --iters 10 --lib $H --lib $V/sr3.so --lib $V/sr4.so \
  "" "defer=1"
step ab_c4 300 python3 tools/tune_ab.py --workload c4_imix --reps 7 --iters 10 --lib $H --lib $V/kargs0.so "" "defer=1"
step ab_c5 300 python3 tools/tune_ab.py --workload c5_tcp1500_10k --reps 5 --iters 8 --lib $H --lib $V/sr3.so --lib $V/sr4.so \
  "" "defer=1"
echo done
