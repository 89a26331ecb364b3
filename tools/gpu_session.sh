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

# s2: GPU suite (TX fields form); the C3 read/write-mix ceiling; C3 sweep at sizes near the bench's and a
# no-counters ablation; interleaved A/B of merged counting and the late barrier on C3, IMIX, C2
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
step rw_probe 200 python tools/rw_probe.py
step c3_sweep 400 python tools/sweep.py --workload c3_udp64 --frames 1M,1536K,2M,3M,4M --rotate 8 --tag base
step c3_sweep_nocnt 400 python tools/sweep.py --workload c3_udp64 --frames 1M,2M,4M --rotate 8 --tag nocounts --no-counts
step c3_ab 400 python tools/abtest.py --workload c3_udp64 --grids 0 --rotate 8 --defer --reps 9 --iters 20 build/variants/base.so build/variants/cnt2.so build/variants/lateb.so build/variants/both.so
step imix_ab 400 python tools/abtest.py --workload c4_imix --grids 0 --rotate 2 --defer --reps 7 --iters 10 build/variants/base.so build/variants/cnt2.so
step c2_ab 400 python tools/abtest.py --workload c2_tcp1500 --grids 0 --defer --reps 7 --iters 10 build/variants/base.so build/variants/cnt2.so
step imix_sweep 400 python tools/sweep.py --workload c4_imix --frames 256K,512K,1M,1536K,2M --rotate 2 --tag base
step tcp_walks 400 python tools/tcp_walk_probe.py --nconns 16 64 256 --streams bench clean --walks rule wave scan --iters 6
step ring_numa 300 python tools/ring_numa.py
echo done
