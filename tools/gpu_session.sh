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

# r05a: the new GPU tests (tests.rs IPv4 vectors + UDP KAT through the HIP path, the 1 GiB-window TCP stream, the
# two-rank bench line's scaling fields), then the default bench line
step refvec 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k reference
step newtests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tcp.py::test_one_stream_gigabyte_window tests/test_gpu_multiproc.py
step bench 600 python bench.py
echo done
