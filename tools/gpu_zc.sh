#!/bin/bash
# C5 shard end to end: dk_rx_process_host staged (DK_RX_HOST_ZC=0) vs zero-copy (default on mapped memory), and the
# bench's direct zero-copy leg, in one process on one box.
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
e5 = RxEngine(Config(synth.BOB_IPV4), device=0)
b5, f5, _ = bench.make_batch(e5, 'c5_tcp1500_10k', 0, synth.SEED, 1)
e0.set_sockets(f5)
out = {}
for rep in range(2):
    out[f'staged{rep}'] = bench.host_path_rate(e0, b5, f5, b5.n)['gbps']
    out[f'zc_api{rep}'] = bench.host_path_rate(e5, b5, f5, b5.n)['gbps']
    out[f'zc_direct{rep}'] = bench.zero_copy_rate(e5, b5, f5, b5.n)['gbps']
print(json.dumps(out))
" > gpurun_out/zc.log 2>&1 || { tail -5 gpurun_out/zc.log; exit 12; }
tail -1 gpurun_out/zc.log
