#!/bin/bash
# round-6: the full-prefetch column form at two lanes (pf: PHD_COLUMN_FORM=1) against the library's choice
# (the half form at two lanes), after this round's kernel changes
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
B="python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3"
tools/gpu_run.sh \
  "r6/pf_hl:600:$B && PHD_LIB=$L/libreport_data_pf.so $B && $B && PHD_LIB=$L/libreport_data_pf.so $B && $B && PHD_LIB=$L/libreport_data_pf.so $B"
