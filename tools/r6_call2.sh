#!/bin/bash
# K1 bank-conflict pricing: conflict-free h/s atomics (xp1), all three (xp2)
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/t_round6:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_round6.py" \
  "r6/k1x_base:120:K1ONLY=1 K1N=64 python tools/k1bench.py" \
  "r6/k1x_xp1:120:PHD_ABLATE=1 PHD_LIB=$L/libreport_data_xp1.so K1ONLY=1 K1N=64 python tools/k1bench.py" \
  "r6/k1x_xp2:120:PHD_ABLATE=1 PHD_LIB=$L/libreport_data_xp2.so K1ONLY=1 K1N=64 python tools/k1bench.py" \
  "r6/k1x_base2:120:K1ONLY=1 K1N=64 python tools/k1bench.py"
