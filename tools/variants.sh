#!/bin/bash
# Build tuning variants of libdk_rx.so into build/variants/<name>.so (same sources, different -D knobs).
# usage: tools/variants.sh "name1:-DX=1 -DY=2" "name2:..."      (SRC=<dir> builds from another source tree)
# tcp_kernels.hip (rocPRIM sort, slow to compile) is compiled once into build/obj/ and linked in, or per variant when
# its flags name a DK_TCP_* knob.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
S=${SRC:-$R}
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC"
mkdir -p $R/build/variants $R/build/obj
TCPO=$R/build/obj/tcp_kernels.o
if [ ! -f $TCPO ] || [ $S/demikernel_amd/csrc/tcp_kernels.hip -nt $TCPO ] || [ $S/include/dk_tcp.h -nt $TCPO ]; then
  $HIPCC -c -o $TCPO $S/demikernel_amd/csrc/tcp_kernels.hip
fi
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  srcs=""
  for f in rx_kernels.hip rx_host.cpp diag.hip ring_host.cpp demi_host.cpp comm_host.cpp; do
    [ -f $S/demikernel_amd/csrc/$f ] && srcs="$srcs $S/demikernel_amd/csrc/$f"
  done
  tcpo=$TCPO
  if [[ "$flags" == *-DDK_TCP_* ]]; then  # TCP knobs: this variant's own tcp_kernels object
    tcpo=$R/build/obj/tcp_kernels_$name.o
    $HIPCC -c $flags -o $tcpo $S/demikernel_amd/csrc/tcp_kernels.hip
  fi
  $HIPCC -shared $flags -o $R/build/variants/$name.so $srcs -x none $tcpo -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done
wait
ls $R/build/variants
