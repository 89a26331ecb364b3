#!/bin/bash
# GPU box: parity tests, smoke, and a short bench of the headline and C3 workloads (from the repo root under gpurun).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/t_tests.log; exit 11; }
tail -3 gpurun_out/t_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t_smoke.log 2>&1 || { echo SMOKE_FAILED; exit 12; }
timeout -k 10 200 python bench.py --no-extras --no-cpu > gpurun_out/t_bench_c2.log 2>&1 || { echo BENCH_FAILED; exit 13; }
timeout -k 10 200 python bench.py --no-extras --no-cpu --workload c3_udp64 > gpurun_out/t_bench_c3.log 2>&1 || exit 14
timeout -k 10 200 python bench.py --no-extras --no-cpu --workload c4_imix > gpurun_out/t_bench_c4.log 2>&1 || exit 15
cat gpurun_out/t_bench_c*.log
