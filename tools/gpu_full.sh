#!/bin/bash
# GPU box: parity tests, smoke, the default bench line (from the repo root under gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/f_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/f_tests.log; exit 11; }
tail -3 gpurun_out/f_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f_smoke.log 2>&1 || { echo SMOKE_FAILED; exit 12; }
SECONDS=0; timeout -k 10 400 python bench.py > gpurun_out/f_bench.log 2> gpurun_out/f_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/f_bench.err; exit 13; }
echo "bench seconds: $SECONDS"
cat gpurun_out/f_bench.log
