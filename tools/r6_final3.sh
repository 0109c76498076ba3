#!/bin/bash
# round-6 last look on the final tree: the GPU suite, the default bench line, the one-lane kernel stats
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6h
tools/gpu_run.sh \
  "r6h/tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6h/prof_config2:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6h/prof_config2 -o prof -- python3 $R/bench.py --no-configs --no-cpu-baseline --lanes 1 --steps 10 --warmup 2 --no-one-lane --no-kernel-events; echo prof_rc=\$?; rm -f $R/gpurun_out/r6h/prof_config2/prof_kernel_trace.csv" \
  "r6h/bench:600:python bench.py"
