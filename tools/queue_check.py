"""Does the package's GPU_MAX_HW_QUEUES default take effect for an import
order?  (run ON the GPU box, GPU_MAX_HW_QUEUES unset)
    python tools/queue_check.py pkg_first | torch_first | cuda_first
Times 6 two-lane calls of 128 device-resident 4000x3000 images."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

order = sys.argv[1]
if order == "pkg_first":
    import photohive_dsp_amd  # noqa: F401
    import torch
elif order == "torch_first":
    import torch
    import photohive_dsp_amd  # noqa: F401
else:                                   # cuda_first: HIP initialised before the package
    import torch
    torch.cuda.init()
    import photohive_dsp_amd  # noqa: F401
import ctypes
from photohive_dsp_amd.lib import lib
from photohive_dsp_amd.core import make_config
from photohive_dsp_amd.structures import Full_Report_Data
torch.cuda.set_device(0)
n, h, w = 128, 3000, 4000
t = torch.empty(n * h * w * 3, dtype=torch.uint8, device="cuda")
assert lib.phd_fill_uniform_device(t.data_ptr(), t.numel(), 7, None) == 0
cfg = make_config()
outs = (ctypes.POINTER(Full_Report_Data) * n)()
st = (ctypes.c_int * n)()
for k in range(8):
    if k == 2:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
    assert lib.phd_report_batch_device(t.data_ptr(), n, h, w, 0, ctypes.byref(cfg), outs, st, None) == 0
    lib.phd_free_reports(outs, n)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"{order}: GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')} {6 * n / dt:.0f} images/s")
