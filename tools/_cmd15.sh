tools/gpu_run.sh \
 "hl1:200:python tools/only.py headline" \
 "hl2:200:ONLY_LANES=2 python tools/only.py headline" \
 "hl2b:200:ONLY_LANES=2 PHD_K1_BPC=1 python tools/only.py headline" \
 "hl1b:200:PHD_K1_BPC=1 python tools/only.py headline"
