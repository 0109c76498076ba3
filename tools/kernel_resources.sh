#!/bin/bash
# VGPRs, occupancy and spills of every kernel of one HIP source (compiler
# remarks; runs anywhere hipcc does):  tools/kernel_resources.sh photohive_dsp_amd/csrc/fft_ct.hip [extra flags]
src="$1"; shift
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics \
  --cuda-device-only -c -o /dev/null "$src" -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  sed -n 's/.*remark: //p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/^Function Name/ {n=$3; sub("_ZN3phd12_GLOBAL__N_1[0-9]*", "", n); sub("EEvP.*", "", n)}
       /VGPRs:/ && !/Spill/ {v=$2} /Occupancy/ {o=$3} /VGPRs Spill/ {printf "%-60s vgpr %3d occ %d spill %d\n", n, v, o, $3}'
