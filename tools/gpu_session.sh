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

# s19: C3 re-check (s18's box ran the small kernel 26 µs under rocprofv3 against 20.7 the session before, same ISA)
step c3k 200 python tools/kbench.py --workload c3_udp64 --iters 20 --rotate 8 --defer
step c3rk 200 python tools/kbench.py --workload c3_udp64_random_ports --iters 20 --rotate 8 --defer
step c3sweep 300 python tools/sweep.py --workload c3_udp64 --frames 1M,2M,4M --rotate 8 --tag s19
step c3prof 200 rocprofv3 --kernel-trace --stats -T -d $O/c3 -o run --output-format csv -- python3 tools/kbench.py --workload c3_udp64 --iters 20 --rotate 8 --defer
echo done
