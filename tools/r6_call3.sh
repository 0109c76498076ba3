#!/bin/bash
# round-6 evidence: same-box A/B of the round-5 library (r5) against this build (K1),
# one-lane headline kernel stats (csv), PMC traffic of the headline config (512 images, 2 lanes)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=photohive_dsp_amd/PhotoHive_DSP_lib
tools/gpu_run.sh \
  "r6/ab_k1_r5:120:PHD_LIB=$L/libreport_data_r5.so K1ONLY=1 K1N=64 python tools/k1bench.py && PHD_LIB=$L/libreport_data_r5.so K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py" \
  "r6/ab_k1_r6:120:K1ONLY=1 K1N=64 python tools/k1bench.py && K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py" \
  "r6/ab_hl_r5:200:PHD_LIB=$L/libreport_data_r5.so python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3" \
  "r6/ab_hl_r6:200:python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3" \
  "r6/prof_config2:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6/prof_config2 -o prof -- python3 $R/bench.py --no-configs --no-cpu-baseline --lanes 1 --steps 10 --warmup 2 --no-one-lane --no-kernel-events" \
  "r6/pmc:600:python tools/pmc_collect.py --tag r06 -- --steps 1 --warmup 1 --batch 512 --lanes 2 --no-configs --no-one-lane"
