tools/gpu_run.sh \
 "sweep3000:200:python tools/ct_sweep.py --cols 0,12" \
 "cmp:200:python tools/cmp_cols_variant.py 0 12" \
 "sweep4000:200:python tools/ct_sweep.py --H 4000 --W 6000 --cols 0" \
 "hl12:200:PHD_CT_COLS_VARIANT=12 python tools/only.py headline" \
 "hl:200:python tools/only.py headline"
