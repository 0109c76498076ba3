#!/bin/bash
# round-6: row-pass stores with DPP-paired reads (this build) against prev; full GPU suite
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
K="K1ONLY=1 K1N=64 python tools/k1bench.py"
B="python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3"
tools/gpu_run.sh \
  "r6/dpp_tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6/dpp_k1b:400:PHD_LIB=$L/libreport_data_prev.so $K && $K && PHD_LIB=$L/libreport_data_prev.so $K && $K" \
  "r6/dpp_hl:400:PHD_LIB=$L/libreport_data_prev.so $B && $B && PHD_LIB=$L/libreport_data_prev.so $B && $B"
