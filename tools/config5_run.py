"""BASELINE config 5 alone (bench.py's config5 workload: 4096 mixed-size
device-resident images, h/s/v 36/4/5, one phd_report_batch_device_mixed call
per pass), for profiling: python tools/config5_run.py [passes]"""
import ctypes
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
sizes = shard.mixed_sizes(4096, 5)
ts = []
for i, (h, w) in enumerate(sizes):
    t = torch.empty((h, w, 3), dtype=torch.uint8, device="cuda")
    assert lib.phd_fill_uniform_device(t.data_ptr(), h * w * 3, 5000 + i, None) == 0
    ts.append(t)
n = len(ts)
cfg = make_config(h_partitions=36, s_partitions=4, v_partitions=5)
ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
hs = (ctypes.c_int * n)(*[h for h, _ in sizes])
ws = (ctypes.c_int * n)(*[w for _, w in sizes])
outs = (ctypes.POINTER(Full_Report_Data) * n)()
st = (ctypes.c_int * n)()
for p in range(passes + 1):
    if p == 1:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    if lib.phd_report_batch_device_mixed(ptrs, hs, ws, n, ctypes.byref(cfg), outs, st, None) != 0:
        raise SystemExit(last_error())
    lib.phd_free_reports(outs, n)
torch.cuda.synchronize()
print(f"config5: {n * passes / (time.perf_counter() - t0):.0f} images/s over {passes} passes")
