#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/pmc_c3; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
for sm in 0 1; do
DK_RX_SMALL=$sm timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "dk_rx" -T -d $OUT/sq$sm -o run --output-format csv -- python3 $R/tools/kbench.py --workload c3_udp64 --iters 5 > $OUT/log$sm.txt 2>&1 || exit 11
DK_RX_SMALL=$sm timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE --kernel-include-regex "dk_rx" -T -d $OUT/sqb$sm -o run --output-format csv -- python3 $R/tools/kbench.py --workload c3_udp64 --iters 5 > $OUT/logb$sm.txt 2>&1 || exit 12
done
echo ok
