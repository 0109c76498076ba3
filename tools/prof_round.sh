# One profiling round on the GPU box (run through gpurun from the repo root):
# PMC HBM traffic per kernel (separate FETCH_SIZE / WRITE_SIZE passes), the
# rocprofv3 kernel statistics of config 2 alone and of the default bench
# command, and the full bench line.  Copy the results into profiles/rNN/.
set -e
TAG="${1:-r03}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/pmc_collect.py --tag "${TAG:-r03}" -- --steps 3 --warmup 1 --no-config3 --batch 8 > gpurun_out/pmc_collect.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o prof -- python bench.py --no-config3 --no-cpu-baseline > gpurun_out/bench_prof2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- python bench.py --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_full.log
