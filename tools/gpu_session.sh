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

# r05zp: the LDS bind table as its own small-frame kernel instantiation (the port-table one as HEAD's): the parity
# file, then C3 / C3 on random ports, HEAD's library vs this build (rule, table forced off)
step parity 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py
step ab_c3 300 python tools/abtest.py --workload c3_udp64 --rotate 8 --defer --grids 0 --knob DK_RX_UDP_TABLE=-1,0 --check --iters 20 --reps 11 build/variants/head.so demikernel_amd/libdk_rx.so
step ab_c3r 300 python tools/abtest.py --workload c3_udp64_random_ports --rotate 8 --defer --grids 0 --knob DK_RX_UDP_TABLE=-1,0 --check --iters 20 --reps 11 build/variants/head.so demikernel_amd/libdk_rx.so
echo done
