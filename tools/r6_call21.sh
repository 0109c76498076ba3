#!/bin/bash
# round-6: the 3000-row half-prefetch column form at three waves per SIMD (c3: 168 VGPRs, spills) against the
# default two, headline on two lanes (the half form's user)
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
B="python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3"
tools/gpu_run.sh \
  "r6/c3_hl:500:$B && PHD_LIB=$L/libreport_data_c3.so $B && $B && PHD_LIB=$L/libreport_data_c3.so $B" \
  "r6/c3_k1b:300:$K && PHD_LIB=$L/libreport_data_c3.so $K"
