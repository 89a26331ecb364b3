#!/bin/bash
# A/B all build/variants/*.so on the standard workloads (GPU box).
R=$(cd "$(dirname "$0")/.." && pwd)
GRIDS=${1:-2,3,4}
for wl in ${2:-c2_tcp1500 c3_udp64 c4_imix c5_tcp1500_10k}; do
  timeout -k 10 300 python3 $R/tools/abtest.py --workload $wl --grids $GRIDS $R/build/variants/*.so 2>/dev/null || exit 1
done
