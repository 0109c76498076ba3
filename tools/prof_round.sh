# One measurement round on the GPU box (run through gpurun from the repo root):
# the GPU test suite, K1's batch timing, the FETCH_SIZE calibrations and the
# per-kernel PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes), the
# rocprofv3 kernel statistics of config 2 alone and of the default bench
# command, and the default bench line.  Stops at the first crash / timeout
# (tools/gpu_run.sh).  Copy the results into profiles/rNN/.
#   bash tools/prof_round.sh r05 [steps...]   (steps: tests k1 calib pmc prof bench; default all)
TAG="${1:-r05}"; shift
STEPS="${*:-tests k1 calib pmc prof bench}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
args=()
for s in $STEPS; do
  case $s in
    tests) args+=("gputest:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider");;
    k1) args+=("k1bench:200:python -u tools/k1bench.py");;
    calib) args+=("pmc_calib:400:python tools/pmc_calib.py");;
    pmc) args+=("pmc_collect:400:python tools/pmc_collect.py --tag $TAG -- --steps 3 --warmup 1 --no-configs --batch 8");;
    prof) args+=("prof_config2:400:GPU_MAX_HW_QUEUES=8 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o prof -- python bench.py --no-configs --no-cpu-baseline --lanes 1"
                 "prof_default:500:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o prof -- python bench.py --no-cpu-baseline --hw-queues 8");;
    bench) args+=("bench_full:500:python bench.py");;
  esac
done
bash tools/gpu_run.sh "${args[@]}"
rc=$?
# only the summaries travel back (gpurun copies at most 64 MiB of gpurun_out/)
find gpurun_out -name "*kernel_trace.csv" -delete 2>/dev/null
find gpurun_out -path "*pmc_*" -name "*counter_collection.csv" -size +4M -delete 2>/dev/null
du -sh gpurun_out
exit $rc
