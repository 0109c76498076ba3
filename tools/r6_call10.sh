#!/bin/bash
# round-6: row-pass store (one thread per column, both rows) against HEAD (prev), and the no-swizzle luma variant; full GPU suite
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/rowst_tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6/rowst_k1b:400:PHD_LIB=$L/libreport_data_prev.so K1ONLY=1 K1N=64 python tools/k1bench.py && K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_LIB=$L/libreport_data_noswz.so K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_LIB=$L/libreport_data_prev.so K1ONLY=1 K1N=64 python tools/k1bench.py && K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_LIB=$L/libreport_data_noswz.so K1ONLY=1 K1N=64 python tools/k1bench.py" \
  "r6/rowst_hl:400:PHD_LIB=$L/libreport_data_prev.so python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3 && python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3 && PHD_LIB=$L/libreport_data_noswz.so python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3"
