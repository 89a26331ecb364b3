#!/bin/bash
# PMC passes (one rocprofv3 run per pass, SQ counters only: <= 8 SQ + 1 GRBM each) over tools/kbench.py for one
# workload. usage (repo root, GPU box): tools/pmc_kernel.sh <workload> <tag> [kbench args...]
set -o pipefail
WL=$1; TAG=$2; shift 2
R=$(pwd); OUT=$R/gpurun_out/pmc_$TAG; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P3="SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
k=0
for P in "$P1" "$P2" "$P3"; do
  k=$((k+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex "dk_rx" -T -d $OUT/p$k -o run --output-format csv -- python3 $R/tools/kbench.py --workload $WL --iters 8 "$@" > $OUT/log$k.txt 2>&1 || { echo "pass $k failed"; tail -5 $OUT/log$k.txt; exit 11; }
done
echo ok
