#!/bin/bash
# round-6: K1's run merge by selects (msel), with the merge threshold at 1/2 (msel2), and the threshold at 1/2
# alone (m2), against the default, on hblur and noise, alternating
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
H="K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py"
tools/gpu_run.sh \
  "r6/msel_hb:700:$H && PHD_LIB=$L/libreport_data_msel.so $H && PHD_LIB=$L/libreport_data_msel2.so $H && PHD_LIB=$L/libreport_data_m2.so $H && $H && PHD_LIB=$L/libreport_data_msel.so $H && PHD_LIB=$L/libreport_data_msel2.so $H && PHD_LIB=$L/libreport_data_m2.so $H" \
  "r6/msel_uni:500:$K && PHD_LIB=$L/libreport_data_msel.so $K && PHD_LIB=$L/libreport_data_msel2.so $K && PHD_LIB=$L/libreport_data_m2.so $K"
