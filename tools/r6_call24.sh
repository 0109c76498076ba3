#!/bin/bash
# round-6: K1's run-merge threshold (default: > 1/5 of 4-pixel groups in one cell) on noise and on hblur:
# m0 never merge, m2 > 1/2, m20 > 1/20, mall always
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
H="K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py"
tools/gpu_run.sh \
  "r6/merge_hb:600:$H && PHD_LIB=$L/libreport_data_m0.so $H && PHD_LIB=$L/libreport_data_m2.so $H && PHD_LIB=$L/libreport_data_m20.so $H && PHD_LIB=$L/libreport_data_mall.so $H && $H" \
  "r6/merge_uni:600:$K && PHD_LIB=$L/libreport_data_m0.so $K && PHD_LIB=$L/libreport_data_m20.so $K && PHD_LIB=$L/libreport_data_mall.so $K"
