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

# C1 (tcp-echo shape): kernel family and grid, counters on / off
step c1_fam 240 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 9 "" "split=0" "split=0,stage=0" \
  "split=0,grid_per_cu=2" "split=0,stage=0,grid_per_cu=2" "split=0,stage=0,grid_per_cu=8"
step c1_nocount 240 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 9 --no-counts "" "split=0" \
  "split=0,stage=0"
# rocprofv3 kernel stats and HBM traffic of C1 at the host rule
cd /tmp
step c1_stats 200 rocprofv3 --kernel-trace --stats -T -d $O/c1_stats -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload c1_tcp1078 --rotate 3 --iters 20
step c1_fetch 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dk_rx_split_kernel|read_probe" -T \
  -d $O/fetch_c1_tcp1078 -o run --output-format csv -- python3 $R/tools/kbench.py --workload c1_tcp1078 --iters 5 --probe-one
step c1_write 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dk_rx_split_kernel|read_probe" -T \
  -d $O/write_c1_tcp1078 -o run --output-format csv -- python3 $R/tools/kbench.py --workload c1_tcp1078 --iters 5 --probe-one
cd $R
step c1_sq 300 bash tools/pmc_kernel.sh c1_tcp1078 ${TAG}_c1 --rotate 3
echo done
