tools/gpu_run.sh \
 "sweep:300:python tools/ct_sweep.py --cols 0,12" \
 "t12:400:PHD_CT_COLS_VARIANT=12 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_round2.py -x -q --timeout 120 --timeout-method thread -k '3000x4000 or 4000x3000 or bit_identical or two_lanes or power_spectrum'" \
 "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "hl:200:python tools/only.py headline" \
 "hl12:200:PHD_CT_COLS_VARIANT=12 python tools/only.py headline"
