tools/gpu_run.sh \
 "planar:200:python -u -m pytest tests/test_gpu_planar.py -x -q --timeout 120 --timeout-method thread" \
 "probe:300:python tools/mixed_probe.py 64" \
 "c5:200:python tools/only.py config5"
