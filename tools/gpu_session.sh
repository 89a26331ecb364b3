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

# s1 (round 6): GPU suite at the env-free tuning; C3 / IMIX fixed-vs-per-frame sweeps and phase totals; C3 at 8
# waves/SIMD (2 chunks per wave) as an A/B
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
step c3_sweep 400 python tools/sweep.py --workload c3_udp64 --frames 1M,2M,4M,8M --rotate 8 --tag base
step c3_sweep_w8 400 python tools/sweep.py --workload c3_udp64 --frames 1M,2M,4M,8M --rotate 8 --tag w8 --lib build/variants/w8.so
step c3_sweep_w8b16 400 python tools/sweep.py --workload c3_udp64 --frames 1M,2M,4M,8M --rotate 8 --tag w8b16 --lib build/variants/w8b16.so
step c3_stamps 300 python tools/stamps.py build/variants/stamps.so --workload c3_udp64
step imix_sweep 500 python tools/sweep.py --workload c4_imix --frames 512K,1M,2M,4M --rotate 2 --tag base
step imix_stamps 300 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2
echo done
