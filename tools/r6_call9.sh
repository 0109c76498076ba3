#!/bin/bash
# round-6: column walk fast form (this build) against the build before it (prev), same box; full GPU suite
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/walk_tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6/walk_k1b:300:PHD_LIB=$L/libreport_data_prev.so K1ONLY=1 K1N=64 python tools/k1bench.py && K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_LIB=$L/libreport_data_prev.so K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py && K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py" \
  "r6/walk_hl:300:PHD_LIB=$L/libreport_data_prev.so python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3 && python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3"
