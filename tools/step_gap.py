"""Host time around the headline's calls (bench.py's step: one
phd_report_batch_device call of 512 device-resident 4000x3000 images on two
lanes, then phd_free_reports): per step, the call's wall time, lane 0's
run_reports host total (phd_last_timings) and the free; prints the means:
python tools/step_gap.py [steps]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from photohive_dsp_amd.core import make_config  # noqa: E402
from photohive_dsp_amd.lib import lib, last_error  # noqa: E402
from photohive_dsp_amd.structures import Full_Report_Data  # noqa: E402
import torch  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
if os.environ.get("COLUMN_FORM"):                 # 0 half / 1 full prefetch form (phd_debug_column_form)
    lib.phd_debug_column_form(int(os.environ["COLUMN_FORM"]))
B, H, W = 512, 3000, 4000
nb = H * W * 3
t = torch.empty(B * nb, dtype=torch.uint8, device="cuda")
for i in range(B):
    assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, i, None) == 0
cfg = make_config()
outs = (ctypes.POINTER(Full_Report_Data) * B)()
st = (ctypes.c_int * B)()
acc = {"call_ms": 0.0, "lane0_host_total_ms": 0.0, "free_ms": 0.0}
tm = (ctypes.c_double * 8)()
for k in range(steps + 2):
    t0 = time.perf_counter()
    if lib.phd_report_batch_device(t.data_ptr(), B, H, W, 0, ctypes.byref(cfg), outs, st, None) != 0:
        raise RuntimeError(last_error())
    t1 = time.perf_counter()
    lib.phd_last_timings(tm, 8)
    lib.phd_free_reports(outs, B)
    t2 = time.perf_counter()
    if k >= 2:
        acc["call_ms"] += 1e3 * (t1 - t0)
        acc["lane0_host_total_ms"] += tm[4]
        acc["free_ms"] += 1e3 * (t2 - t1)
print(json.dumps({k: round(v / steps, 3) for k, v in acc.items()}), flush=True)
