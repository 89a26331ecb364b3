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
# the in-tree library must be the checked-out tree's build (a stale library fails every GPU test)
python -c "import __graft_entry__ as g; assert g.lib_build_id() == g.tree_build_id(), (g.lib_build_id(), g.tree_build_id())" || exit 9

# s11: 128-byte line rewrites in the probe (flags 4, 5); the TX kernels rewriting a frame's whole first 128-byte line
# (DK_TX_LINE128, in-tree default for this session): GPU suite, interleaved A/B against the 64-byte rewrite
step patch_probe 400 python tools/patch_probe.py --lates 0 --flags 0,1,4,5 --grids 1024,2048
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step tx_ab 400 python tools/abtest.py --workload c2_tcp1500 --grids 0 --tx --reps 11 --iters 20 build/variants/tx64.so build/variants/tx128.so
step tx_bench 300 python tools/kbench.py --workload c2_tcp1500 --iters 20 --no-rx --tx --tx-fields
echo done
