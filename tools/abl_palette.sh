#!/bin/bash
# K1 / K3 ablation timings (GPU box): production library, then the ablation build
# with PHD_ABLATE masks (K1: 8 classify, 16 hist atomic, 32 sat, 64 fold; K3: 8
# classify, 16 LDS sums, 32 hue).
PHD_QUIET=1 timeout -k 10 120 python tools/k1bench.py 2>&1 | grep -E "hsv_stats 64|K1\+hist|palette_sums|fft"
for a in ${ABL:-0 8 16 32 56 64}; do
  echo "== ablate $a"
  PHD_LIB=photohive_dsp_amd/PhotoHive_DSP_lib/libreport_data_ablate.so PHD_ABLATE=$a PHD_QUIET=1 \
    timeout -k 10 120 python tools/k1bench.py 2>&1 | grep -E "K1\+hist|palette_sums"
done
