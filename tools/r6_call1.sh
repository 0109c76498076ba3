#!/bin/bash
# round-6 GPU call: full GPU suite, K1 timings, a short headline, the profiled default command
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tools/gpu_run.sh \
  "r6/gpu_tests:420:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/" \
  "r6/k1_uniform:120:K1ONLY=1 K1N=64 python tools/k1bench.py" \
  "r6/k1_hblur:120:K1ONLY=1 K1N=64 K1KIND=hblur python tools/k1bench.py" \
  "r6/k1_fine:120:K1ONLY=1 K1N=64 K1GRID=36,4,5 python tools/k1bench.py" \
  "r6/bench_short:300:python bench.py --no-configs --no-cpu-baseline --steps 20 --warmup 3" \
  "r6/prof_default:300:cd /tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/prof_default -o prof -- python3 $R/bench.py --no-configs --no-cpu-baseline --steps 4 --warmup 2 --no-one-lane --no-kernel-events; echo prof_rc=\$?"
