#!/bin/bash
# K1 beside the FFT chain (round-2 experiment): K1 built
# for 512-thread blocks so one FFT block fits beside it on a CU, the FFTs on
# their own stream (PHD_FFT_OVERLAP=1), K1's LDS budget lowered.  Build the
# variant first (here, not on the GPU box):
#   make -C photohive_dsp_amd/csrc OUT=$PWD/photohive_dsp_amd/PhotoHive_DSP_lib/libreport_data_k512.so \
#        OBJDIR=$PWD/build/obj_k512 EXTRA_HIPFLAGS=-DPHD_K1_T=512
# Measured: 5.60k images/s against 6.09k for the production library.
B="python bench.py --no-cpu-baseline --no-configs --steps 20 --batch 8"
run() { echo "== $1"; shift; env "$@" timeout -k 5 120 $B 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['stages_ms_per_step_rank0'], d['warmup_kernels_us_per_launch'])"; }
L=photohive_dsp_amd/PhotoHive_DSP_lib
run base PHD_LIB=$L/libreport_data.so
run base_overlap PHD_LIB=$L/libreport_data.so PHD_FFT_OVERLAP=1
run k512 PHD_LIB=$L/libreport_data_k512.so
run k512_overlap PHD_LIB=$L/libreport_data_k512.so PHD_FFT_OVERLAP=1
run k512_overlap_lds84 PHD_LIB=$L/libreport_data_k512.so PHD_FFT_OVERLAP=1 PHD_K1_LDS_KB=84
run k512_overlap_lds72 PHD_LIB=$L/libreport_data_k512.so PHD_FFT_OVERLAP=1 PHD_K1_LDS_KB=72
