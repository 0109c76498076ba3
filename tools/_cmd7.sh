tools/gpu_run.sh \
 "sweep3000:200:python tools/ct_sweep.py --cols 0" \
 "sweep3000off:200:PHD_COL_WINDOWS=0 python tools/ct_sweep.py --cols 0" \
 "sweep4000:300:python tools/ct_sweep.py --H 4000 --W 6000 --cols 0,1" \
 "sweep4000off:300:PHD_COL_WINDOWS=0 python tools/ct_sweep.py --H 4000 --W 6000 --cols 0,1" \
 "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "hl:200:python tools/only.py headline"
