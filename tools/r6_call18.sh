#!/bin/bash
# round-6: row-pass pixel loads plain (rownt0) against non-temporal (default): PMC traffic and time
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
B="python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3"
P="-- --steps 1 --warmup 1 --batch 64 --lanes 2 --no-configs --no-one-lane"
tools/gpu_run.sh \
  "r6/nt_pmc:600:python tools/pmc_collect.py --tag nt1 $P && PHD_LIB=$L/libreport_data_rownt0.so python tools/pmc_collect.py --tag nt0 $P" \
  "r6/nt_k1b:400:$K && PHD_LIB=$L/libreport_data_rownt0.so $K && $K && PHD_LIB=$L/libreport_data_rownt0.so $K" \
  "r6/nt_hl:400:$B && PHD_LIB=$L/libreport_data_rownt0.so $B && $B && PHD_LIB=$L/libreport_data_rownt0.so $B"
