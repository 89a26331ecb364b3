#!/bin/bash
# Build tuning variants of libdk_rx.so into build/variants/<name>.so (same sources, different -D knobs).
# usage: tools/variants.sh "name1:-DX=1 -DY=2" "name2:..."
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/build/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -o $R/build/variants/$name.so \
    $R/demikernel_amd/csrc/rx_kernels.hip $R/demikernel_amd/csrc/rx_host.cpp $R/demikernel_amd/csrc/diag.hip &
done
wait
ls $R/build/variants
