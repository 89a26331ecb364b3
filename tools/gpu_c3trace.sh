#!/bin/bash
# Kernel trace of the C3 workload (8 rotating batches): per-launch durations and gaps of the small-frame kernel and
# the counter reduce. usage: tools/gpu_c3trace.sh [lib]
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/c3trace; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
LIB=${1:+--lib $R/$1}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $OUT -o run --output-format csv -- \
  python3 $R/tools/kbench.py --workload c3_udp64 --iters 40 --rotate 8 $LIB > $OUT/c3.log 2>&1 || { tail -5 $OUT/c3.log; exit 15; }
python3 - <<'PY'
import csv, glob
f = glob.glob('/root/repo/gpurun_out/c3trace/**/run_kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'dk_' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
prev = None
out = []
for r in rows[-40:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    out.append((r['Kernel_Name'].split('(')[0][-40:], (e - s) / 1e3, (s - prev) / 1e3 if prev else 0))
    prev = e
for o in out[-12:]: print('%-42s dur %.2f us gap %.2f us' % o)
PY
