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

# r05zd: the bench's ring_path_rate vs ring_bytes' ring path on the same frames and engine (which factor costs ~5 %)
step ringq 400 python -c "
import json, time, numpy as np, torch, bench
from demikernel_amd import Config, RxEngine, RxResults, synth
from demikernel_amd import ring as RG
torch.cuda.set_device(0)
n = 1 << 19
flows = synth.make_flows(1024)
tr = synth.traffic(n, np.full(n, 1486, np.uint16), flows, seed=synth.SEED + 5)
packed, poff, lens = synth.build_numpy(tr)
eng = RxEngine(Config(synth.BOB_IPV4)); eng.set_sockets(flows)
def tool_like(reps=5):
    ring, used, _, elen = RG.build_tpacket3(packed, poff.astype(np.int64), lens, 1 << 22)
    r = RG.TpacketRing(ring, 1 << 22)
    res = RxResults(n, len(flows), host=True)
    nbytes = int(lens.astype(np.int64).sum()); rates = []
    for _ in range(reps + 1):
        t = time.perf_counter(); r.receive(eng, 0, used, res); rates.append(nbytes / (time.perf_counter() - t) / 1e9)
    r.close()
    return round(float(np.median(rates[1:])), 2), [round(x, 1) for x in rates]
batch = synth.build_device(tr, eng, seed=synth.SEED + 5)
for rep in range(3):
    print(json.dumps({'rep': rep, 'tool_like': tool_like(), 'bench_ring': bench.ring_path_rate(eng, batch, flows, n)}), flush=True)
"
echo done
