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

# s28: the TCP key pass with 1 / 2 / 4 frames a thread (every load before the first store) against the committed one
step key_ab 400 python tools/tcp_ab.py build/variants/keyold.so build/variants/key1.so build/variants/key2.so build/variants/key4.so --nconns 16384,64 --reorder 3 --buffer-size 16777216
step key_ab1 300 python tools/tcp_ab.py build/variants/keyold.so build/variants/key1.so build/variants/key2.so build/variants/key4.so --nconns 1 --reorder 0 --buffer-size 1073741824
step keyprof 200 rocprofv3 --kernel-trace --stats -T -d $O/k4 -o run --output-format csv -- python3 tools/tcp_ab.py build/variants/key4.so --nconns 16384 --reorder 3 --buffer-size 16777216 --reps 2
echo done
