"""One 3000x4000 image per call (BASELINE config 2 as stated), for a kernel trace:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st -o st -- python tools/single_trace.py
    python tools/step_gaps.py gpurun_out/st
"""
import ctypes
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error  # noqa: E402
from photohive_dsp_amd.core import make_config  # noqa: E402
from photohive_dsp_amd.structures import Full_Report_Data  # noqa: E402

H, W = 3000, 4000
nb = H * W * 3
t = torch.empty(nb, dtype=torch.uint8, device="cuda")
assert lib.phd_fill_uniform_device(t.data_ptr(), nb, 7, None) == 0
torch.cuda.synchronize()
cfg = make_config()
out = (ctypes.POINTER(Full_Report_Data) * 1)()
st = (ctypes.c_int * 1)()
ts = []
for i in range(40):
    t0 = time.perf_counter()
    if lib.phd_report_batch_device(t.data_ptr(), 1, H, W, nb, ctypes.byref(cfg), out, st, None) != 0:
        raise RuntimeError(last_error())
    ts.append(time.perf_counter() - t0)
    lib.free_full_report(ctypes.byref(out[0]))
ts = sorted(ts[10:])
print(f"median {1000 * ts[len(ts) // 2]:.3f} ms per single-image call")
tm = (ctypes.c_double * 8)()
lib.phd_last_timings(tm, 8)
print("stages (k1, fft, tail, gpu_total, host_total, enqueue, decisions, assembly) ms:", [round(x, 3) for x in tm])
