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
echo "== vparity"
timeout -k 10 300 python3 tools/variant_parity.py --lib $V/dyn.so --frames 1048576 > $O/vparity.log 2>&1
rc=$?; grep -h '^{' $O/vparity.log | cut -c1-200
if [ $rc -gt 1 ]; then echo "vparity rc=$rc"; tail -20 $O/vparity.log; exit 10; fi
# staged kernel: dynamic tail (the last rounds grabbed from 8 counters) vs static round-robin
step imix 300 python3 tools/tune_ab.py --workload c4_imix --reps 9 --lib $L --lib $V/dyn.so --lib $V/nodyn.so "defer=1"
step imix_r2 300 python3 tools/tune_ab.py --workload c4_imix --rotate 2 --reps 7 --lib $L --lib $V/dyn.so "defer=1"
step c1x8 300 python3 tools/tune_ab.py --workload c1_tcp1078 --frames 1048576 --rotate 2 --reps 5 --lib $L --lib $V/dyn.so "defer=1"
echo done
