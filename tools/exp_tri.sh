L=photohive_dsp_amd/PhotoHive_DSP_lib
run() { n=$1; shift; echo "== $n"; env "$@" timeout -k 5 60 python tools/kbench.py 0 0 0 2>&1 | grep kernel; env "$@" timeout -k 5 100 python bench.py --no-cpu-baseline --no-configs --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['warmup_kernels_us_per_launch']['hsv_stats'])"; }
run base PHD_LIB=$L/libreport_data.so
run tri PHD_LIB=$L/libreport_data_tri.so
run tri512_79 PHD_LIB=$L/libreport_data_tri512.so PHD_K1_LDS_KB=79
run tri512_158 PHD_LIB=$L/libreport_data_tri512.so
