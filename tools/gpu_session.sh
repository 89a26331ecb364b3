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
step t_part 400 $PYT tests/test_gpu_parity.py -k "deferred_counts or kernel_variants or full_size_c4 or tx"
step t_all 900 $PYT -m gpu tests
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
# 2. A/B with deferred counters (what bench.py runs); early0: next descriptors waited for at the top of the chunk
V=build/variants
H=demikernel_amd/libdk_rx.so
step ab_c4 300 python3 tools/tune_ab.py --workload c4_imix --reps 9 --iters 10 --lib $H --lib $V/early0.so --lib $V/kargs0.so \
  --lib $V/prev.so "defer=1"
step ab_c3 300 python3 tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 11 --iters 16 --lib $H --lib $V/kargs0.so \
  --lib $V/prev.so "defer=1"
step ab_c2 300 python3 tools/tune_ab.py --workload c2_tcp1500 --reps 7 --iters 10 --lib $H --lib $V/early0.so --lib $V/prev.so "defer=1"
step ab_c5 300 python3 tools/tune_ab.py --workload c5_tcp1500_10k --reps 5 --iters 8 --lib $H --lib $V/early0.so --lib $V/prev.so "defer=1"
step ab_c1 300 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 7 --iters 20 --lib $H --lib $V/early0.so \
  --lib $V/kargs0.so --lib $V/prev.so "defer=1"
# 3. TX split kernel: separate role loops + descriptors ahead (head) vs before (prev)
step ab_tx 300 python3 tools/abtest.py --workload c2_tcp1500 --grids 0 --tx --reps 7 $H $V/prev.so
# 4. C1 shape at 1x, 2x, 4x, 8x the frames: the per-launch fixed cost (intercept) vs the per-byte rate
for F in 131072 262144 524288 1048576; do
  step c1_n$F 300 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 5 --iters 10 --frames $F "defer=1"
done
echo done
