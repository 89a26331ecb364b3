#!/bin/bash
# The current GPU session's measurement steps (rewritten per gpurun call; each step has its own time limit and the
# script stops at the first failure). Run from the repo root on the GPU box: bash tools/gpu_session.sh <tag>
set -o pipefail
TAG=${1:-s}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
step() {  # step <name> <seconds> <cmd...>: stdout+stderr to $O/<name>.log
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  grep -h '^{' $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -20 $O/$name.log; exit 10; fi
}
export TMPDIR=/tmp

# 1. rocprofv3 evidence: kernel stats of the bench, FETCH/WRITE traffic per workload, C1/C3/TX/TCP kernel stats
step profile 1000 bash tools/profile_bench.sh $TAG
# 2. the collective beside the kernels (side stream / same stream, every 1 / 8 / 16 steps)
step overlap 300 python3 tools/overlap_collective.py --out $O/r04_overlap.json
# 3. IMIX LDS bank conflicts by structure: as run / socket table probed in global memory (no LDS table) / no counters
cd /tmp
SQ="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_LDS_ATOMIC SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE"
step lds_asis 120 rocprofv3 --pmc $SQ --kernel-include-regex "dk_rx_kernel" -T -d $O/lds_asis -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload c4_imix --iters 8 --defer
DK_RX_LDS_TABLE=0 step lds_notable 120 rocprofv3 --pmc $SQ --kernel-include-regex "dk_rx_kernel" -T -d $O/lds_notable -o run \
  --output-format csv -- python3 $R/tools/kbench.py --workload c4_imix --iters 8 --defer
step lds_nocount 120 rocprofv3 --pmc $SQ --kernel-include-regex "dk_rx_kernel" -T -d $O/lds_nocount -o run --output-format csv \
  -- python3 $R/tools/kbench.py --workload c4_imix --iters 8 --no-counts
cd $R
echo done
