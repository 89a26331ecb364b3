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

# 1. parity
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step t_part 400 $PYT tests/test_gpu_parity.py -k "full_size_c2 or deferred_counts or kernel_variants or tcp_fields or options"
step t_multi 300 $PYT tests/test_gpu_multiproc.py
step t_all 900 $PYT -m gpu tests
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
# 2. A/B: the LibOS record staged by the split kernel (head) vs stored between the frame reads (prev)
V=build/variants
H=demikernel_amd/libdk_rx.so
step ab_libos 300 python3 tools/tune_ab.py --workload c2_tcp1500 --tcp-fields --reps 7 --iters 10 --lib $H --lib $V/prev.so "defer=1"
step ab_c2 300 python3 tools/tune_ab.py --workload c2_tcp1500 --reps 7 --iters 10 --lib $H --lib $V/prev.so "defer=1"
step ab_c5 300 python3 tools/tune_ab.py --workload c5_tcp1500_10k --reps 5 --iters 8 --lib $H --lib $V/prev.so "defer=1"
step ab_c4 300 python3 tools/tune_ab.py --workload c4_imix --reps 7 --iters 10 --lib $H --lib $V/prev.so "defer=1"
# 3. the collective beside the kernels: every step, every 8 steps, 8 CUs left free
step overlap 400 python3 tools/overlap_collective.py --out $O/r04_overlap.json
echo done
