tools/gpu_run.sh \
 "hl2:200:ONLY_LANES=2 python tools/only.py headline" \
 "hl2f:200:ONLY_LANES=2 PHD_FFT_BPC=1 python tools/only.py headline" \
 "hl1:200:python tools/only.py headline" \
 "c5l2:200:ONLY_LANES=2 python tools/only.py config5"
