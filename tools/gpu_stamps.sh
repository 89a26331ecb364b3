#!/bin/bash
# Per-wave timeline of the small-frame kernel (C3) from stamp builds under build/diag.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/stamps.log
for lib in ${LIBS:-build/diag/stamps.so}; do
  echo "{\"lib\": \"$lib\"}" >> gpurun_out/stamps.log
  timeout -k 10 240 python -u tools/stamps.py $lib --workload c3_udp64 --grids ${GRIDS:-1,5} >> gpurun_out/stamps.log 2>&1 || exit 1
done
