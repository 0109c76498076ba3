#!/bin/bash
# round-6: the column walk's fast form from the LDS run list with the u8 segment table (this build) against the
# u32 segment words (prev); full GPU suite; PMC traffic (64-image two-lane passes)
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
B="python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3"
P="-- --steps 1 --warmup 1 --batch 64 --lanes 2 --no-configs --no-one-lane"
tools/gpu_run.sh \
  "r6/seg8_tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6/seg8_pmc:600:python tools/pmc_collect.py --tag seg8 $P && PHD_LIB=$L/libreport_data_prev.so python tools/pmc_collect.py --tag seg32 $P" \
  "r6/seg8_k1b:400:PHD_LIB=$L/libreport_data_prev.so $K && $K && PHD_LIB=$L/libreport_data_prev.so $K && $K" \
  "r6/seg8_hl:400:PHD_LIB=$L/libreport_data_prev.so $B && $B && PHD_LIB=$L/libreport_data_prev.so $B && $B"
