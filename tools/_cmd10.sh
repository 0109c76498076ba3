tools/gpu_run.sh \
 "sweep:400:python tools/ct_sweep.py --cols 0,13,14,15" \
 "sweepw:400:PHD_COL_WINDOWS=2 python tools/ct_sweep.py --cols 0,13,14,15" \
 "probe:200:PROBE_SHAPES=512x512,480x640 PHD_VERBOSE=0 python tools/mixed_probe.py 64"
