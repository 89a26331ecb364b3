set -o pipefail
mkdir -p gpurun_out
A="python3 tools/abtest.py --grids 0"
for wl in c3_udp64 c2_tcp1500 c4_imix; do R=1; [ $wl = c3_udp64 ] && R=8
  timeout -k 10 200 $A --workload $wl --rotate $R --iters 12 --reps 7 --knob DK_RX_COMBINE=0 build/variants/*.so > gpurun_out/abr_$wl.log 2>&1 || exit 3; grep '^{' gpurun_out/abr_$wl.log; done
for spec in c2_tcp1500:4096 c2_tcp1500:32768 c3_udp64:16384 c3_udp64:131072 c4_imix:16384; do wl=${spec%%:*}; fr=${spec#*:}
  timeout -k 10 200 $A --workload $wl --frames $fr --iters 20 --reps 9 --knob DK_RX_COMBINE=0,1,2 build/variants/a_base.so > gpurun_out/abs_$wl$fr.log 2>&1 || exit 4; grep '^{' gpurun_out/abs_$wl$fr.log | sed "s/}/, \"frames\": $fr}/"; done
