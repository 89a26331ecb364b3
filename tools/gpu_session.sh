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

# r05za: receive_batch's per-call Python cost (ABI structs cached, no record_stream for the same pending arrays): the
# GPU suite, then bench.py's C3 / C1 extras (HIP-event region vs the kernel's own duration)
step gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
step c3 300 python -c "
import json, torch, bench
torch.cuda.set_device(0); s = torch.cuda.current_stream(0)
for name, rot in (('c3_udp64', 8), ('c1_tcp1078', 3)):
    out = bench.rx_extra(name, 0, s, steps=40, warmup=4, rotate=rot)[0]
    print(json.dumps({'name': name, 'kernel_ms_avg': out['kernel_ms_avg'], 'frac': out['roofline']['frac'], 'gbps': out['gbps']}), flush=True)
"
echo done
