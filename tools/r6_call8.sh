#!/bin/bash
# round-6: where K1's time outside the pixel loop goes (timing builds: no deferred pass / no chunk fold)
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/k1abl:400:K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_ABLATE=1 PHD_LIB=$L/libreport_data_nodefer.so K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_ABLATE=1 PHD_LIB=$L/libreport_data_nofold.so K1ONLY=1 K1N=64 python tools/k1bench.py && K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_ABLATE=1 PHD_LIB=$L/libreport_data_nodefer.so K1ONLY=1 K1N=64 K1GRID=36,4,5 python tools/k1bench.py && PHD_ABLATE=1 PHD_LIB=$L/libreport_data_nofold.so K1ONLY=1 K1N=64 K1GRID=36,4,5 python tools/k1bench.py && K1ONLY=1 K1N=64 K1GRID=36,4,5 python tools/k1bench.py"
