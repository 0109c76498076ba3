"""BASELINE config 4 alone (bench.py's config4 workload: 2048 device-resident
4000x3000 images, FFT + blur profile only, one phd_blur_batch_device call per
pass) on one and on two library lanes, for A/B runs of library variants
(PHD_LIB=...): python tools/config4_run.py [images] [passes]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photohive_dsp_amd.core import make_config  # noqa: E402
from photohive_dsp_amd.lib import lib, last_error  # noqa: E402
from photohive_dsp_amd.structures import Blur_Vector  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 3
h, w = 3000, 4000
nb = h * w * 3
t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
for i in range(n):
    assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, 1000 + i, None) == 0
cfg = make_config()
bins = np.zeros((n, cfg.angle_partitions, cfg.radius_partitions))
vecs = (Blur_Vector * (10 * n))()
P = ctypes.POINTER(ctypes.c_double)


def run():
    if lib.phd_blur_batch_device(t.data_ptr(), n, h, w, 0, ctypes.byref(cfg), bins.ctypes.data_as(P), vecs,
                                 None) != 0:
        raise RuntimeError(last_error())


res = {"lib": os.environ.get("PHD_LIB", "default"), "images": n}
prev = lib.phd_set_lanes(0)
for lanes in (1, 2, 1, 2):
    lib.phd_set_lanes(lanes)
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(passes):
        run()
    torch.cuda.synchronize()
    res.setdefault(f"lanes{lanes}_images_per_s", []).append(round(n * passes / (time.perf_counter() - t0), 1))
lib.phd_set_lanes(prev)
print(json.dumps(res), flush=True)
