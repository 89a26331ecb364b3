#!/bin/bash
# Profile the receive kernel on the GPU box (run from the repo root under gpurun).
# Writes rocprofv3 outputs under gpurun_out/prof_<tag>/ ; summaries are copied into profiles/ by hand.
set -o pipefail
TAG=${1:-r01}
WL=${2:-c2_tcp1500}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload $WL --iters 20 --probe > $OUT/kbench_trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dk_rx_kernel|read_probe" -T -d $OUT/pmc_fetch -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload $WL --iters 5 --probe > $OUT/kbench_fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dk_rx_kernel|read_probe" -T -d $OUT/pmc_write -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload $WL --iters 5 --probe > $OUT/kbench_write.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex "dk_rx_kernel" -T -d $OUT/pmc_sq -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload $WL --iters 5 > $OUT/kbench_sq.log 2>&1 || exit 14
echo done
