"""Row / column FFT kernel time vs image height (fixed per-launch overhead):
    python tools/kbench_h.py KERNEL H1 H2 ...   (KERNEL: 1 fft_rows, 2 fft_cols; W = 4000)"""
import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.core import make_config
W = 4000
k = int(sys.argv[1])
cfg = make_config()
for h in [int(x) for x in sys.argv[2:]]:
    n = h * W * 3
    img = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert lib.phd_fill_uniform_device(img.data_ptr(), n, 1, None) == 0
    ms = ctypes.c_double()
    rc = lib.phd_debug_time_kernel(k, img.data_ptr(), h, W, ctypes.byref(cfg), 0, 20, ctypes.byref(ms))
    assert rc == 0, last_error()
    print(f"kernel {k} H={h}: {1000 * ms.value:.1f} us  ({1000 * ms.value * 3000 / h:.1f} us per 3000 rows)")
    del img
