#!/bin/bash
# Build tuning variants of libdk_rx.so into build/variants/<name>.so (same sources, different -D knobs).
# usage: tools/variants.sh "name1:-DX=1 -DY=2" "name2:..."      (SRC=<dir> builds from another source tree)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=${SRC:-$R}
mkdir -p $R/build/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  srcs=""
  for f in rx_kernels.hip rx_host.cpp diag.hip ring_host.cpp tcp_kernels.hip demi_host.cpp comm_host.cpp; do
    [ -f $S/demikernel_amd/csrc/$f ] && srcs="$srcs $S/demikernel_amd/csrc/$f"
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $flags -o $R/build/variants/$name.so \
    $srcs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done
wait
ls $R/build/variants
