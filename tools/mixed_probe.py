"""Per-size cost of the full report (config 5 sizes): for each shape in
shard.MIXED_SHAPES, a batch of n device-resident images through
phd_report_batch_device, wall time and per-kernel HIP-event averages.
Usage: python tools/mixed_probe.py [n] [h s v]   (PROBE_SHAPES=HxW,..., PROBE_KIND=hblur, PROBE_HSV=h,s,v)"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from photohive_dsp_amd import shard  # noqa: E402
from photohive_dsp_amd.core import make_config  # noqa: E402
from photohive_dsp_amd.lib import lib, last_error  # noqa: E402
from photohive_dsp_amd.structures import Full_Report_Data  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
hsv = ([int(x) for x in sys.argv[2:5]] if len(sys.argv) > 4 else
       [int(x) for x in os.environ["PROBE_HSV"].split(",")] if os.environ.get("PROBE_HSV") else [36, 4, 5])
cfg = make_config(h_partitions=hsv[0], s_partitions=hsv[1], v_partitions=hsv[2])
names = ["k1", "fft_rows", "fft_cols", "cutoffs", "pal_sums", "sharp"]
shapes = sorted(set(shard.MIXED_SHAPES), key=lambda s: s[0] * s[1])
if os.environ.get("PROBE_SHAPES"):
    shapes = [tuple(int(v) for v in x.split("x")) for x in os.environ["PROBE_SHAPES"].split(",")]
for h, w in shapes:
    nb = 3 * h * w
    t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
    for i in range(n):
        if os.environ.get("PROBE_KIND") == "hblur":       # bench.py's structured images
            assert lib.phd_fill_structured_device(t[i * nb:].data_ptr(), h, w, 2 + i, 15, 1, None) == 0
        else:
            assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, 77 + i, None) == 0
    outs = (ctypes.POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()

    def run():
        if lib.phd_report_batch_device(t.data_ptr(), n, h, w, 0, ctypes.byref(cfg), outs, st, None) != 0:
            raise RuntimeError(last_error())
        for i in range(n):
            r = outs[i]
            lib.free_full_report(ctypes.byref(r))
    run()
    lib.phd_profile_kernels(0)
    lib.phd_profile_kernels(63)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stage = [0.0] * 8
    for _ in range(3):
        run()
        tm = (ctypes.c_double * 8)()
        lib.phd_last_timings(tm, 8)
        stage = [a + b / 3 for a, b in zip(stage, tm)]
    wall = (time.perf_counter() - t0) / 3
    us = {}
    for k, nm in enumerate(names):
        tot, cnt = ctypes.c_double(), ctypes.c_long()
        lib.phd_profile_read(k, ctypes.byref(tot), ctypes.byref(cnt))
        if cnt.value:
            us[nm] = round(1000 * tot.value / cnt.value, 1)
    lib.phd_profile_kernels(0)
    print(json.dumps({"shape": [h, w], "us_per_image_wall": round(1e6 * wall / n, 1),
                      "mpx_per_s": round(h * w * n / wall / 1e6), "kernel_us_per_launch": us,
                      "stages_ms": dict(zip(["k1", "fft", "tail", "gpu_total", "host_total", "host_enqueue",
                                             "host_decisions", "host_assembly"], [round(x, 3) for x in stage]))}), flush=True)
    del t
    torch.cuda.empty_cache()
