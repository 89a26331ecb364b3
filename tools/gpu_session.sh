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

# r05f: small-frame kernel with a uniform wave index and an unrolled window DMA (83 VGPRs at 5 waves/SIMD; 80 at 6):
# parity of the 6-wave build, C3 A/B 5 vs 6 waves, SQ counter passes of both
step parity6 600 python tools/variant_parity.py --lib /root/repo/build/variants/sm6.so
step ab_c3 600 python tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 9 --iters 40 --lib demikernel_amd/libdk_rx.so --lib /root/repo/build/variants/sm6.so "defer=1"
step ab_c3r 600 python tools/tune_ab.py --workload c3_udp64_random_ports --rotate 8 --reps 7 --iters 40 --lib demikernel_amd/libdk_rx.so --lib /root/repo/build/variants/sm6.so "defer=1"
step pmc5 600 bash tools/pmc_kernel.sh c3_udp64 r05f_c3_w5 --rotate 8 --defer
step pmc6 600 bash tools/pmc_kernel.sh c3_udp64 r05f_c3_w6 --rotate 8 --defer --lib /root/repo/build/variants/sm6.so
step trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05f/trace -o run --output-format csv -- python3 tools/kbench.py --workload c3_udp64 --iters 40 --rotate 8 --defer
echo done
