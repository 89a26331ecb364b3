#!/bin/bash
# rocprofv3 evidence for one round (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command itself (profiles/<tag>_bench_kernel_stats.csv)
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes over kbench (deferred counters, as the bench runs) (dk_rx_kernel + the read probe, whose byte count
#      is known: it calibrates the FETCH_SIZE unit for this access pattern on gfx950)
# then tools/summarize_profile.py <tag> writes profiles/<tag>_summary.md and profiles/pmc_traffic.json.
set -o pipefail
TAG=${1:-r01}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $OUT/bench -o run --output-format csv -- \
  python3 $R/bench.py --steps 50 --warmup 5 --cpu-seconds 2 --no-extras > $OUT/bench.json 2> $OUT/bench.err || exit 11
# traffic passes: one FETCH_SIZE and one WRITE_SIZE run per workload (name[:variant]: libos = the 36-byte LibOS record)
for SPEC in c2_tcp1500 c3_udp64 c4_imix c5_tcp1500_10k c1_tcp1078 c3_udp64_random_ports c2_tcp1500:libos c2_tcp1500:txf; do
  WL=${SPEC%%:*}; VAR=${SPEC#*:}; [ "$VAR" = "$SPEC" ] && VAR=""
  KEY=$WL${VAR:+_$VAR}
  TX=""; [ $KEY = c2_tcp1500 ] && TX=--tx
  EXTRA=""; [ "$VAR" = libos ] && EXTRA=--tcp-fields
  [ "$VAR" = txf ] && EXTRA=--tx-fields  # the fields form of the TX kernel (dk_tx_checksum_fields) alone
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "dk_rx_kernel|dk_rx_split_kernel|dk_rx_small_kernel|dk_tx_kernel|dk_tx_split_kernel|read_probe" -T -d $OUT/fetch_$KEY -o run --output-format csv -- \
    python3 $R/tools/kbench.py --workload $WL --iters 5 --probe-one --defer $TX $EXTRA > $OUT/fetch_$KEY.log 2>&1 || exit 12
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "dk_rx_kernel|dk_rx_split_kernel|dk_rx_small_kernel|dk_tx_kernel|dk_tx_split_kernel|read_probe" -T -d $OUT/write_$KEY -o run --output-format csv -- \
    python3 $R/tools/kbench.py --workload $WL --iters 5 --probe-one --defer $TX $EXTRA > $OUT/write_$KEY.log 2>&1 || exit 13
done
# kernel stats of the 64-byte-frame kernel (C3) and the TX checksum kernel (C2 batch)
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/c3 -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload c3_udp64 --iters 20 --rotate 8 --defer > $OUT/c3.log 2>&1 || exit 15
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/c1 -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload c1_tcp1078 --iters 20 --rotate 3 --defer > $OUT/c1.log 2>&1 || exit 17
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/tx -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload c2_tcp1500 --iters 20 --tx > $OUT/tx.log 2>&1 || exit 16
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/txf -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload c2_tcp1500 --iters 20 --no-rx --tx-fields > $OUT/txf.log 2>&1 || exit 18
# the TCP receive pipeline's kernels (1M segments, 16k connections)
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT/tcp -o run --output-format csv -- \
  python3 $R/tools/tcpbench.py --nconns 16384 --iters 10 --cpu-seconds 0.5 > $OUT/tcp.json 2> $OUT/tcp.err || exit 14
cd $R && python3 tools/summarize_profile.py $TAG
