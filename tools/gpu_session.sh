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

L=demikernel_amd/libdk_rx.so
V=build/variants
# 0. variants' results against the oracle (their timings count only if they are bit-exact)
echo "== vparity"
timeout -k 10 300 python3 tools/variant_parity.py --lib $V/tiny.so --lib $V/fewsched1.so --lib $V/stprio1.so > $O/vparity.log 2>&1
rc=$?; grep -h '^{' $O/vparity.log | cut -c1-300
if [ $rc -gt 1 ]; then echo "vparity rc=$rc"; tail -20 $O/vparity.log; exit 10; fi  # 1 = a mismatch: keep going
# 1. the GPU suite at this build
step gpu_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
# 2. C3: priority / early descriptors, each on and off
step c3 300 python3 tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 11 --lib $L --lib $V/noprio.so --lib $V/prio2.so --lib $V/noearly.so --lib $V/none.so "defer=1"
# 3. C1 by the host rule (staged now) vs the split kernel
step c1 300 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 4 --reps 9 --lib $L --lib $V/fewsched1.so "defer=1" "defer=1,split=1"
# 4. IMIX: priority for the staged kernel's waves with one chunk more
step imix 300 python3 tools/tune_ab.py --workload c4_imix --rotate 2 --reps 9 --lib $L --lib $V/stprio1.so --lib $V/nosmall.so --lib $V/tiny.so "defer=1"
echo done
