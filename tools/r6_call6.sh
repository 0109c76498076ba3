#!/bin/bash
# round-6: the column pass's two-chain run walk (A/B against one chain, same box), its parity tests,
# config 5 per size and alone
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/walk_tests:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_round5.py tests/test_gpu_parity.py" \
  "r6/walk_ab:200:PHD_LIB=$L/libreport_data_walk1.so python tools/kbench.py 2 0 0 0 && python tools/kbench.py 2 0 0 0 && PHD_LIB=$L/libreport_data_walk1.so python tools/kbench.py 2 0 0 0 && python tools/kbench.py 2 0 0 0" \
  "r6/walk_hl:300:PHD_LIB=$L/libreport_data_walk1.so python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3 && python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3" \
  "r6/c5_probe:300:python tools/mixed_probe.py 64" \
  "r6/c5_run:300:python tools/config5_run.py 4 && PHD_LIB=$L/libreport_data_walk1.so python tools/config5_run.py 4"
