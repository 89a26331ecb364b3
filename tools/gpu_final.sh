# Round-end evidence on the GPU box (from the repo root under gpurun): GPU tests, smoke, bench, and rocprofv3 kernel
# stats of the bench and of the TCP walk at 64 and 16,384 connections.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/f_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/f_smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/f_bench.log 2>&1 &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/f_prof_bench -o run --output-format csv -- python3 $R/bench.py --steps 20 > $R/gpurun_out/f_prof_bench.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $R/gpurun_out/f_prof_tcp -o run --output-format csv -- python3 $R/tools/tcpbench.py --nseg 1048576 --nconns 64 16384 --iters 10 --cpu-seconds 0.1 > $R/gpurun_out/f_prof_tcp.log 2>&1 &&
echo done
