#!/bin/bash
# round-6: same-box A/B (round-5 library vs this build), K1 SQ counters, the full default bench line
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/ab2_k1_r5:150:PHD_LIB=$L/libreport_data_r5.so K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_LIB=$L/libreport_data_r5.so K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py" \
  "r6/ab2_k1_r6:150:K1ONLY=1 K1N=64 python tools/k1bench.py && K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py" \
  "r6/ab2_hl_r5:200:PHD_LIB=$L/libreport_data_r5.so python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3" \
  "r6/ab2_hl_r6:200:python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3" \
  "r6/sq_k1:400:python tools/pmc_sq.py 0 --probe 3000x4000:64" \
  "r6/bench_default:600:python bench.py"
