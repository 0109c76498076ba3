tools/gpu_run.sh \
 "sweep:300:python tools/ct_sweep.py --cols 0,12" \
 "cmp:200:python tools/cmp_cols_variant.py 0 12" \
 "hl:200:python tools/only.py headline" \
 "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
