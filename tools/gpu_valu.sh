#!/bin/bash
# SQ instruction counts per wave for every build/variants/*.so on one workload (one --pmc pass each).
set -o pipefail
WL=${WL:-c3_udp64}
R=$(pwd); export TMPDIR=/tmp
for v in build/variants/*.so; do
  n=$(basename $v .so); OUT=$R/gpurun_out/valu_$n; mkdir -p $OUT
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "dk_rx" -d $OUT/p1 -o run --output-format csv -- python3 $R/tools/kbench.py --workload $WL --iters 4 --rotate 8 --lib $R/$v > $OUT/log.txt 2>&1) || { echo "$n failed"; tail -5 $OUT/log.txt; exit 11; }
done
echo ok
