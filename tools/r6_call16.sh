#!/bin/bash
# round-6: unclamped column passes (idle waves skip the partial rounds) against the default, alternating
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
B="python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3"
tools/gpu_run.sh \
  "r6/ncl_k1b:500:$K && PHD_LIB=$L/libreport_data_noclamp.so $K && $K && PHD_LIB=$L/libreport_data_noclamp.so $K && $K && PHD_LIB=$L/libreport_data_noclamp.so $K" \
  "r6/ncl_hl:400:$B && PHD_LIB=$L/libreport_data_noclamp.so $B && $B && PHD_LIB=$L/libreport_data_noclamp.so $B"
