#!/bin/bash
# round-6: palette partial sums without scratch memory (this build) against prev (60 B of scratch per thread);
# the palette GPU tests; the headline alternating
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
B="python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3"
tools/gpu_run.sh \
  "r6/scr_tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6/scr_hl:600:PHD_LIB=$L/libreport_data_prev.so $B && $B && PHD_LIB=$L/libreport_data_prev.so $B && $B && PHD_LIB=$L/libreport_data_prev.so $B && $B"
