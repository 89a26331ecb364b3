#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/abtest.py --workload c4_imix --grids ${GRIDS:-0,4} --iters 16 --reps ${REPS:-9} build/variants/*.so > gpurun_out/imix_ab.log 2>&1 || { tail -5 gpurun_out/imix_ab.log; exit 12; }
grep '^{' gpurun_out/imix_ab.log
