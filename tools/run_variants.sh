#!/bin/bash
# Time every build/variants/*.so on a workload (GPU box). usage: tools/run_variants.sh <workload> [iters]
WL=${1:-c2_tcp1500}; IT=${2:-30}; EXTRA=${3:-}
R=$(cd "$(dirname "$0")/.." && pwd)
for so in $R/build/variants/*.so; do
  n=$(basename $so .so)
  DK_RX_LIB_VARIANT=$so timeout -k 10 120 python3 $R/tools/kbench.py --workload $WL --iters $IT $EXTRA 2>/dev/null | sed "s/^/$n $WL /" || exit 1
done
