#!/bin/bash
# K1's two forms on the GPU box: two 512-thread blocks per CU with the
# triangular code table (default where the grid fits) against one 1024-thread
# block per CU (PHD_K1_ONE_BLOCK=1).  Single-image kernel time, then the bench.
run() { n=$1; shift; echo "== $n"; env "$@" timeout -k 5 60 python tools/kbench.py 0 0 0 2>&1 | grep kernel; env "$@" timeout -k 5 100 python bench.py --no-cpu-baseline --no-configs --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['warmup_kernels_us_per_launch']['hsv_stats'])"; }
run two_blocks PHD_K1_TWO=1
run one_block PHD_K1_ONE_BLOCK=1
