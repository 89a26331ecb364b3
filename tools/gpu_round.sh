#!/bin/bash
# GPU box: the whole -m gpu suite, smoke, and the full default bench line (from the repo root under gpurun).
# usage: tools/gpu_round.sh TAG
set -o pipefail
tag=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/${tag}_tests.log; exit 11; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { echo SMOKE_FAILED; cat gpurun_out/${tag}_smoke.log; exit 12; }
cat gpurun_out/${tag}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/${tag}_bench.err; exit 13; }
cat gpurun_out/${tag}_bench.json
