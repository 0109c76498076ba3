#!/bin/bash
# round-6: 3000-row column plan orders (cf1 20 10 15, cf2 20 15 10, cf3 10 20 15, cf4 15 20 10) against the
# default 15 10 20; the statistics kernel alone, this build against prev (HEAD~2: no device finish)
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
tools/gpu_run.sh \
  "r6/cplan_k1b:600:$K && PHD_LIB=$L/libreport_data_cf1.so $K && PHD_LIB=$L/libreport_data_cf2.so $K && PHD_LIB=$L/libreport_data_cf3.so $K && PHD_LIB=$L/libreport_data_cf4.so $K && $K && PHD_LIB=$L/libreport_data_cf1.so $K && PHD_LIB=$L/libreport_data_cf2.so $K" \
  "r6/stats_ab:300:PHD_LIB=$L/libreport_data_prev.so python tools/config3_time.py && python tools/config3_time.py && PHD_LIB=$L/libreport_data_prev.so python tools/config3_time.py && python tools/config3_time.py"
