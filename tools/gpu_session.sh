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

# r05zi: the staging kernel's tail with 32-frame halves at the end of each pool (DK_RX_TAIL_HALF, % of a pool's
# waves): parity of the dynamic-tail test, IMIX A/B at 2 rotating batches and 1, the exit spread
step parity 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "dynamic_tail or full_size_c4 or kernel_variants"
step ab_imix 300 python tools/abtest.py --workload c4_imix --rotate 2 --defer --grids 0 --knob DK_RX_TAIL_HALF=0,25,50,100,200 --check --iters 10 --reps 7 demikernel_amd/libdk_rx.so
step ab_imix1 300 python tools/abtest.py --workload c4_imix --rotate 1 --defer --grids 0 --knob DK_RX_TAIL_HALF=0,50,100 --iters 10 --reps 7 demikernel_amd/libdk_rx.so
step st_h0 120 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2 --tuning tail_half=0
step st_h50 120 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2 --tuning tail_half=50
step st_h100 120 python tools/stamps_staged.py build/variants/stamps.so --workload c4_imix --rotate 2 --tuning tail_half=100
echo done
