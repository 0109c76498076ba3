"""Config 5's size groups one at a time: for each shape of shard.MIXED_SHAPES,
as many device-resident uniform images as config 5 holds of it (4096 images,
seed 5), full reports at h/s/v 36/4/5 through phd_report_batch_device (the
call config 5's mixed entry makes per size group), timed over `passes`
passes after one warm call.  Prints one JSON line per shape and a total whose
sum of ms per pass is config 5's pass time without overlap between groups:
python tools/size_sweep.py [passes] [HxW ...] (only those shapes)"""
import collections
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photohive_dsp_amd import shard  # noqa: E402
from photohive_dsp_amd.core import make_config  # noqa: E402
from photohive_dsp_amd.lib import lib, last_error  # noqa: E402
from photohive_dsp_amd.structures import Full_Report_Data  # noqa: E402
import torch  # noqa: E402

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 3
only = set(sys.argv[2:])
counts = collections.Counter(shard.mixed_sizes(4096, 5))
cfg = make_config(h_partitions=36, s_partitions=4, v_partitions=5)
tot_ms = 0.0
tot_px = 0
for (h, w) in shard.MIXED_SHAPES:
    if only and f"{h}x{w}" not in only:
        continue
    n = counts[(h, w)]
    nb = h * w * 3
    t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
    for i in range(n):
        assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, 5000 + i, None) == 0
    outs = (ctypes.POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()

    def run():
        if lib.phd_report_batch_device(t.data_ptr(), n, h, w, 0, ctypes.byref(cfg), outs, st, None) != 0:
            raise RuntimeError(last_error())
        lib.phd_free_reports(outs, n)
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(passes):
        run()
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / passes
    tot_ms += ms
    tot_px += n * h * w
    print(json.dumps({"shape": f"{h}x{w}", "images": n, "ms_per_pass": round(ms, 2),
                      "images_per_s": round(n / ms * 1000, 1), "gpx_per_s": round(n * h * w / ms / 1e6, 2)}),
          flush=True)
    del t
    torch.cuda.empty_cache()
print(json.dumps({"total_ms_per_pass": round(tot_ms, 2), "images_per_s": round(4096 / tot_ms * 1000, 1),
                  "gpx_per_s": round(tot_px / tot_ms / 1e6, 2)}), flush=True)
