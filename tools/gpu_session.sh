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

# s29: the scan walk with each window's frame indices and records copied by the pre kernel (one round trip for the
# slow path and the post kernel) and the next batches loaded under the slow path: GPU suite, A/B, step attribution
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step scan_ab 400 python tools/tcp_ab.py build/variants/scanhead.so build/variants/scannopf.so build/variants/scanpf.so --nconns 1,16,64,256 --reorder 0 --buffer-size 1073741824 --walk scan
step scan_ab3 300 python tools/tcp_ab.py build/variants/scanhead.so build/variants/scanpf.so --nconns 16,64 --reorder 3 --buffer-size 16777216 --walk scan
step scan1 200 python tools/tcp_scan_stats.py build/variants/tcpstats.so --nconns 1 --reorder 0 --buffer-size 1073741824
echo done
