#!/bin/bash
# round-6: FFT co-residency study (timing build): persistent column / row grids capped at one block per CU so
# that the two lanes' passes can share CUs, against the same build uncapped
export TMPDIR=/tmp
L=photohive_dsp_amd/PhotoHive_DSP_lib
B="python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 20 --warmup 3"
A="PHD_LIB=$L/libreport_data_ablate.so"
tools/gpu_run.sh \
  "r6/bpc:900:$A $B && $A PHD_COL_BPC=1 $B && $A PHD_ROW_BPC=1 $B && $A PHD_COL_BPC=1 PHD_ROW_BPC=1 $B && $A PHD_COL_BPC=1 PHD_ROW_BPC=1 PHD_K1_BPC=1 $B && $A $B"
