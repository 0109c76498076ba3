#!/bin/bash
# round-6: K1 merge threshold 1/2 (m2) against the default 1/5 on every bench line (no CPU baseline), alternating
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
B="python bench.py --no-cpu-baseline --no-one-lane"
tools/gpu_run.sh \
  "r6/m2_full:1100:$B && PHD_LIB=$L/libreport_data_m2.so $B && $B && PHD_LIB=$L/libreport_data_m2.so $B"
