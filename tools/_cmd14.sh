tools/gpu_run.sh \
 "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "sweep:200:python tools/ct_sweep.py --cols 0" \
 "sweep4000:200:python tools/ct_sweep.py --H 4000 --W 6000 --cols 0" \
 "hl:200:python tools/only.py headline config5"
