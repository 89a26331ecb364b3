#!/bin/bash
# Sweep build/variants x grid-per-CU x workloads (GPU box). usage: tools/sweep.sh "1 2 3 4" "c2_tcp1500 c3_udp64" [iters]
GRIDS=${1:-"1 2 3 4"}; WLS=${2:-c2_tcp1500}; IT=${3:-20}
R=$(cd "$(dirname "$0")/.." && pwd)
for so in $R/build/variants/*.so; do
  n=$(basename $so .so)
  for g in $GRIDS; do
    for wl in $WLS; do
      DK_RX_GRID_PER_CU=$g DK_RX_LIB_VARIANT=$so timeout -k 10 120 python3 $R/tools/kbench.py --workload $wl --iters $IT 2>/dev/null \
        | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$n', 'g=$g', '$wl', d['ms'], d['algo_GBps'], d['mpkt_s'])" || exit 1
    done
  done
done
