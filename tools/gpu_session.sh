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

# 1. parity: the changed paths first, then the whole GPU suite
PYT="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
step t_defer 400 $PYT tests/test_gpu_parity.py -k "deferred_counts or counter_rows or flow_counter or two_streams or streams_destroyed"
step t_multi 300 $PYT tests/test_gpu_multiproc.py
step t_all 900 $PYT -m gpu tests
step smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()"
# 2. deferred counters and the family choice on C1, and deferral on the other configs
step c1_fam 300 python3 tools/tune_ab.py --workload c1_tcp1078 --rotate 3 --reps 9 "" "defer=1" "split=0" "split=0,defer=1" \
  "split=0,stage=0" "split=0,stage=0,defer=1" "split=0,stage=0,grid_per_cu=8,defer=1"
for wl in c2_tcp1500 c4_imix c5_tcp1500_10k; do
  step ${wl}_defer 300 python3 tools/tune_ab.py --workload $wl --reps 7 --iters 10 "" "defer=1"
done
step c3_defer 300 python3 tools/tune_ab.py --workload c3_udp64 --rotate 8 --reps 9 --iters 16 "" "defer=1"
# 3. flow-count aggregation A/B (variant without it)
for wl in c1_tcp1078 c2_tcp1500 c5_tcp1500_10k; do
  step ${wl}_agg 300 python3 tools/tune_ab.py --workload $wl --rotate 3 --reps 7 --iters 10 --lib demikernel_amd/libdk_rx.so \
    --lib build/variants/aggoff.so "defer=1"
done
# 3b. end-only kernel arguments read at their use (DK_KARGS, default 1) vs through the by-value parameter
for wl in c3_udp64 c4_imix c2_tcp1500; do
  R8=1; [ $wl = c3_udp64 ] && R8=8
  step ${wl}_kargs 300 python3 tools/tune_ab.py --workload $wl --rotate $R8 --reps 7 --iters 10 \
    --lib demikernel_amd/libdk_rx.so --lib build/variants/kargs0.so "" "defer=1"
done
# 4. rocprofv3 kernel stats and HBM traffic of C1 at the host rule
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
