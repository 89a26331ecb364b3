#!/bin/bash
# TPACKET_V3 ring path: staged (DK_RX_HOST_ZC=0) vs zero-copy (default), same box, same process.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -c "
import os, sys, json, torch
sys.path.insert(0, '.')
import bench
from demikernel_amd import Config, RxEngine, synth
torch.cuda.set_device(0)
os.environ['DK_RX_HOST_ZC'] = '0'
e0 = RxEngine(Config(synth.BOB_IPV4), device=0)
os.environ.pop('DK_RX_HOST_ZC')
e1 = RxEngine(Config(synth.BOB_IPV4), device=0)
b, f, _ = bench.make_batch(e1, 'c2_tcp1500', 0, synth.SEED, 1)
e0.set_sockets(f)
out = {}
for rep in range(2):
    out[f'staged{rep}'] = bench.ring_path_rate(e0, b, f, 1 << 19)['gbps']
    out[f'zc{rep}'] = bench.ring_path_rate(e1, b, f, 1 << 19)['gbps']
print(json.dumps(out))
" > gpurun_out/ringzc.log 2>&1 || { tail -5 gpurun_out/ringzc.log; exit 12; }
tail -1 gpurun_out/ringzc.log
