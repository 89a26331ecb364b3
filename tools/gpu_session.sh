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

# small-frame kernel workgroup size (DK_SMALL_WAVES 4 -> 5 / 8 / 10: fewer counter rows per launch)
V=build/variants
H=demikernel_amd/libdk_rx.so
step parity 900 python3 -u tools/variant_parity.py --lib $V/sw5.so --lib $V/sw8.so --lib $V/sw10.so
step ab_c3 400 python3 tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 11 --iters 16 --lib $H --lib $V/sw5.so \
  --lib $V/sw8.so --lib $V/sw10.so "defer=1"
step ab_c3r 400 python3 tools/tune_ab.py --workload c3_udp64_random_ports --rotate 8 --reps 9 --iters 16 --lib $H \
  --lib $V/sw5.so --lib $V/sw8.so --lib $V/sw10.so "defer=1"
echo done
