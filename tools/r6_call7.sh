#!/bin/bash
# round-6: K1 code table (this build) against the build before it (prev), same box; K1 GPU tests
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/ctab_tests:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_round4.py tests/test_gpu_round6.py" \
  "r6/ctab_k1:300:PHD_LIB=$L/libreport_data_prev.so K1ONLY=1 K1N=64 python tools/k1bench.py && K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_LIB=$L/libreport_data_prev.so K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py && K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py && PHD_LIB=$L/libreport_data_prev.so K1ONLY=1 K1N=64 K1GRID=36,4,5 python tools/k1bench.py && K1ONLY=1 K1N=64 K1GRID=36,4,5 python tools/k1bench.py" \
  "r6/ctab_hl:300:PHD_LIB=$L/libreport_data_prev.so python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3 && python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3"
