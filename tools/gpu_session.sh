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

# s6: the small-frame kernel with the next window's DMA in flight through a chunk's stores and counts (DK_SMALL_PIPE,
# now the default): GPU suite, interleaved A/B against the previous loop, C3 sweep at the new default
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
step c3_ab 400 python tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --defer --reps 11 --iters 20 build/variants/nopipe.so build/variants/pipe.so
step c3r_ab 400 python tools/abtest.py --workload c3_udp64_random_ports --grids 0 --rotate 8 --defer --reps 7 --iters 20 build/variants/nopipe.so build/variants/pipe.so
# the staged kernel's tail grabs committed half a round ahead (DK_TAIL_LATE) against 1.5, tail slack 1-3 rounds
step imix_tail_ab 500 python tools/abtest.py --workload c4_imix --grids 0 --rotate 2 --defer --reps 7 --iters 10 --knob DK_RX_TAIL=1,2,3 --check build/variants/tbase.so build/variants/tlate.so
step c3_sweep 400 python tools/sweep.py --workload c3_udp64 --frames 1M,1536K,2M,3M,4M --rotate 8 --tag pipe
echo done
