#!/bin/bash
# round-6 evidence: one-lane headline kernel stats (csv), PMC traffic of the headline config (512 images, 2 lanes)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh \
  "r6/prof_config2:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6/prof_config2 -o prof -- python3 $R/bench.py --no-configs --no-cpu-baseline --lanes 1 --steps 10 --warmup 2 --no-one-lane --no-kernel-events" \
  "r6/pmc:600:python tools/pmc_collect.py --tag r06 -- --steps 1 --warmup 1 --batch 512 --lanes 2 --no-configs --no-one-lane"
