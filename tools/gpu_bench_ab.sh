#!/bin/bash
# Same-box A/B of whole bench lines: bench.py --workload $WL --no-extras --no-cpu with each build/variants/*.so copied
# over the in-tree library of this scratch copy, twice in alternation.
set -o pipefail
mkdir -p gpurun_out
WL=${WL:-c4_imix}
for rep in 1 2; do
  for v in build/variants/*.so; do
    cp $v demikernel_amd/libdk_rx.so || exit 2
    timeout -k 10 200 python3 bench.py --workload $WL --no-extras --no-cpu --steps 50 > gpurun_out/bab_$(basename $v .so)_$rep.json 2> gpurun_out/bab.err || { tail -5 gpurun_out/bab.err; exit 3; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])" gpurun_out/bab_$(basename $v .so)_$rep.json $(basename $v .so) $rep
  done
done
