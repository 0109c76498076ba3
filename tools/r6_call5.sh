#!/bin/bash
# round-6: which HSA runtime HIP dispatches through (maps, no profiler); the default bench command under
# rocprofv3 (kernel stats csv; exit status recorded; the per-dispatch trace csv is dropped: > 64 MiB)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
tools/gpu_run.sh \
  "r6/maps_noprof:200:PHD_BENCH_MAPS=$R/gpurun_out/r6/maps python bench.py --no-configs --no-cpu-baseline --no-one-lane --steps 2 --warmup 1" \
  "r6/prof_full:900:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6/prof_full -o prof -- python3 $R/bench.py; echo prof_rc=\$?; rm -f $R/gpurun_out/r6/prof_full/prof_kernel_trace.csv"
