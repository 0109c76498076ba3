#!/bin/bash
# round-6: column plan 15 20 10 (cf4) against the default 15 10 20, alternating; the headline with each;
# config 3's statistics kernel with and without a host gap between calls (clock-state probe)
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
B="python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3"
tools/gpu_run.sh \
  "r6/cf4_k1b:500:$K && PHD_LIB=$L/libreport_data_cf4.so $K && $K && PHD_LIB=$L/libreport_data_cf4.so $K && $K && PHD_LIB=$L/libreport_data_cf4.so $K" \
  "r6/cf4_hl:400:$B && PHD_LIB=$L/libreport_data_cf4.so $B && $B && PHD_LIB=$L/libreport_data_cf4.so $B" \
  "r6/cfg3_gap:300:python tools/config3_time.py && CFG3_GAP_US=300 python tools/config3_time.py && PHD_LIB=$L/libreport_data_prev.so python tools/config3_time.py && python tools/config3_time.py && CFG3_GAP_US=300 python tools/config3_time.py"
