#!/bin/bash
# Interleaved A/B of build/variants/*.so (GPU box). usage: tools/gpu_ab.sh "<grids>" "<scheds>" [--knob NAME=v1,v2] wl1 wl2 ...
set -o pipefail
mkdir -p gpurun_out
G=$1; S=$2; shift 2
KNOB=""
if [ "$1" = "--knob" ]; then KNOB="--knob $2"; shift 2; fi
for wl in "$@"; do
  timeout -k 10 240 python3 tools/abtest.py --workload $wl --grids $G ${S:+--scheds $S} $KNOB build/variants/*.so > gpurun_out/ab_$wl.log 2>&1 || exit 12
done
echo done
