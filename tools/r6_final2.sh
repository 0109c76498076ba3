#!/bin/bash
# round-6 closing measurements on the final build: the GPU suite, rocprofv3 kernel stats of the headline on one
# lane and of the default command (exit status recorded), PMC traffic of the headline configuration (512
# images, two lanes), SQ counters of the pipeline kernels, the default bench line
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6g
tools/gpu_run.sh \
  "r6g/tests:600:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "r6g/prof_config2:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6g/prof_config2 -o prof -- python3 $R/bench.py --no-configs --no-cpu-baseline --lanes 1 --steps 10 --warmup 2 --no-one-lane --no-kernel-events; echo prof_rc=\$?; rm -f $R/gpurun_out/r6g/prof_config2/prof_kernel_trace.csv" \
  "r6g/prof_full:900:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6g/prof_full -o prof -- python3 $R/bench.py; echo prof_rc=\$?; rm -f $R/gpurun_out/r6g/prof_full/prof_kernel_trace.csv" \
  "r6g/pmc:600:python tools/pmc_collect.py --tag r06 -- --steps 1 --warmup 1 --batch 512 --lanes 2 --no-configs --no-one-lane" \
  "r6g/sq:400:python tools/pmc_sq.py 0 --probe 3000x4000:64" \
  "r6g/bench:600:python bench.py"
find gpurun_out -name "*kernel_trace.csv" -delete 2>/dev/null
find gpurun_out -path "*pmc_*" -name "*counter_collection.csv" -size +4M -delete 2>/dev/null
du -sh gpurun_out
