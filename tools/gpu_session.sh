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

# r05i: line-aligned spans and the branch-free small_fast reverted (no gain, C3 +8 %: session r05h); kept: leader
# atomics without the optimizer expansion + the priority split on the host (prev.so = without them). C3 A/B, the ring
# experiment extended to the memory registration (ring layout in hipHostMalloc memory, packed layout in registered
# mmap memory), C3 SQ counters of the kept build
step ab_c3 600 python tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 9 --iters 40 --lib demikernel_amd/libdk_rx.so --lib build/variants/prev.so "defer=1"
step ab_c3r 600 python tools/tune_ab.py --workload c3_udp64_random_ports --rotate 8 --reps 7 --iters 40 --lib demikernel_amd/libdk_rx.so --lib build/variants/prev.so "defer=1"
step ring 600 python tools/ring_bytes.py
step pmc6 600 bash tools/pmc_kernel.sh c3_udp64 r05i_c3 --rotate 8 --defer
step smallparity 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "small or udp64 or kernel_variants or corpus or golden or reference"
echo done
