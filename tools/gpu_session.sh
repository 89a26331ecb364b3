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

# r05h: (1) small_fast branch-free common path + leader atomics without the optimizer expansion + priority split on
# the host (prev.so = the commit before); (2) line-aligned quarter-wave spans (pre_la.so = without them): the whole
# receive parity file, A/B on C3 / IMIX / C2, the ring/layout PCIe experiment for both builds, C3 SQ counters
step parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py
step ab_c3 600 python tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 9 --iters 40 --lib demikernel_amd/libdk_rx.so --lib build/variants/pre_la.so --lib build/variants/prev.so "defer=1"
step ab_c3r 600 python tools/tune_ab.py --workload c3_udp64_random_ports --rotate 8 --reps 7 --iters 40 --lib demikernel_amd/libdk_rx.so --lib build/variants/prev.so "defer=1"
step ab_imix 600 python tools/tune_ab.py --workload c4_imix --rotate 2 --reps 5 --iters 20 --lib demikernel_amd/libdk_rx.so --lib build/variants/pre_la.so "defer=1"
step ab_c2 600 python tools/tune_ab.py --workload c2_tcp1500 --reps 5 --iters 20 --lib demikernel_amd/libdk_rx.so --lib build/variants/pre_la.so "defer=1"
step ring_new 600 python tools/ring_bytes.py
step ring_pre 600 env DK_RX_LIB_VARIANT=build/variants/pre_la.so python tools/ring_bytes.py
step pmc6 600 bash tools/pmc_kernel.sh c3_udp64 r05h_c3 --rotate 8 --defer
echo done
