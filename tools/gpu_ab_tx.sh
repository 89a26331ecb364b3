set -o pipefail
mkdir -p gpurun_out
DK_RX_LIB_VARIANT=$PWD/build/variants/tx3.so timeout -k 10 300 python3 -m pytest tests -m gpu -x -q -k "tx" > gpurun_out/t_tx3.log 2>&1 &&
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q > gpurun_out/t_gpu.log 2>&1 &&
timeout -k 10 200 python3 tools/abtest.py --tx --workload c2_tcp1500 --grids 2,3 build/variants/tx0.so build/variants/tx2.so build/variants/tx3.so > gpurun_out/ab_tx.log 2>&1 &&
timeout -k 10 200 python3 tools/abtest.py --tx --workload c4_imix --grids 3,4 build/variants/tx0.so build/variants/tx3.so >> gpurun_out/ab_tx.log 2>&1 &&
timeout -k 10 200 python3 tools/abtest.py --workload c2_tcp1500 --grids 3 build/variants/tx0.so >> gpurun_out/ab_tx.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/bench.log 2>&1
