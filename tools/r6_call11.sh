#!/bin/bash
# round-6: row-pass luma swizzle forms (sel4 = default, byte rotation = rotw, none = noswz) and the cheaper
# k1_exact (default vs prev = HEAD~1, identical row code); full GPU suite
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
B="python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3"
tools/gpu_run.sh \
  "r6/swz_tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6/swz_k1b:500:PHD_LIB=$L/libreport_data_prev.so $K && $K && PHD_LIB=$L/libreport_data_rotw.so $K && PHD_LIB=$L/libreport_data_noswz.so $K && PHD_LIB=$L/libreport_data_prev.so $K && $K && PHD_LIB=$L/libreport_data_rotw.so $K && PHD_LIB=$L/libreport_data_noswz.so $K" \
  "r6/swz_hl:500:PHD_LIB=$L/libreport_data_prev.so $B && $B && PHD_LIB=$L/libreport_data_rotw.so $B && PHD_LIB=$L/libreport_data_noswz.so $B"
