#!/bin/bash
# SQ counter passes (tools/pmc_kernel.sh) for each named variant on one workload. usage: tools/gpu_pmc_ab.sh WL v1 v2 ...
set -o pipefail
WL=$1; shift
for v in "$@"; do
  tools/pmc_kernel.sh $WL ${WL}_$v --lib $(pwd)/build/variants/$v.so --rotate ${ROT:-1} || exit 11
  python3 tools/pmc_summary.py gpurun_out/pmc_${WL}_$v gpurun_out/pmc_${WL}_$v.json > /dev/null || exit 12
done
echo ok
