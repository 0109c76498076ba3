#!/bin/bash
# round-6: K1's SQ counters at the default grid (18/2/3) on noise and on the structured hblur images
export TMPDIR=/tmp
tools/gpu_run.sh \
  "r6/sqk1_uni:300:PROBE_HSV=18,2,3 python tools/pmc_sq.py 0 --probe 3000x4000:64 && mv gpurun_out/pmc_sq_0.json gpurun_out/pmc_sq_k1_uniform_default_grid.json" \
  "r6/sqk1_hb:300:PROBE_KIND=hblur PROBE_HSV=18,2,3 python tools/pmc_sq.py 0 --probe 3000x4000:64 && mv gpurun_out/pmc_sq_0.json gpurun_out/pmc_sq_k1_hblur_default_grid.json" \
  "r6/probe_hb:200:PROBE_SHAPES=3000x4000 PROBE_HSV=18,2,3 python tools/mixed_probe.py 64 && PROBE_KIND=hblur PROBE_SHAPES=3000x4000 PROBE_HSV=18,2,3 python tools/mixed_probe.py 64"
