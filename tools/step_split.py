"""Time a 256-image headline call, its host stages and the report frees around it (GPU box)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.core import make_config
from photohive_dsp_amd.structures import Full_Report_Data
H, W, B = 3000, 4000, 256
nb = 3 * H * W
t = torch.empty(B * nb, dtype=torch.uint8, device="cuda")
for i in range(B):
    assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, i, None) == 0
cfg = make_config()
outs = (ctypes.POINTER(Full_Report_Data) * B)()
st = (ctypes.c_int * B)()
tm = (ctypes.c_double * 8)()
for it in range(8):
    t0 = time.perf_counter()
    assert lib.phd_report_batch_device(t.data_ptr(), B, H, W, nb, ctypes.byref(cfg), outs, st, None) == 0, last_error()
    t1 = time.perf_counter()
    lib.phd_last_timings(tm, 8)
    lib.phd_free_reports(outs, B)
    t2 = time.perf_counter()
    print(f"call {1000*(t1-t0):.3f} ms (host_total {tm[4]:.3f}, gpu_total {tm[3]:.3f}) free {1000*(t2-t1):.3f} ms", flush=True)
