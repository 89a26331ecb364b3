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
timeout -k 10 300 python3 tools/variant_parity.py --lib $V/aos.so --lib $V/stg8.so > $O/vparity.log 2>&1
rc=$?; grep -h '^{' $O/vparity.log | cut -c1-200
if [ $rc -gt 1 ]; then echo "vparity rc=$rc"; tail -20 $O/vparity.log; exit 10; fi
# LDS Active table as 16-byte slots (one ds_read_b128 per lookup); staged kernel with 8 staged chunks
step imix 300 python3 tools/tune_ab.py --workload c4_imix --reps 9 --lib $L --lib $V/aos.so --lib $V/stg8.so "defer=1"
step c2 300 python3 tools/tune_ab.py --workload c2_tcp1500 --reps 7 --lib $L --lib $V/aos.so "defer=1"
step c5 300 python3 tools/tune_ab.py --workload c5_tcp1500_10k --reps 5 --lib $L --lib $V/aos.so "defer=1"
echo done
