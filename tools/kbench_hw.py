"""Row / column FFT kernel time at any size, per million pixels:
    python tools/kbench_hw.py KERNEL HxW [HxW ...]   (KERNEL: 1 fft_rows, 2 fft_cols)"""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.core import make_config
k = int(sys.argv[1])
cfg = make_config()
for s in sys.argv[2:]:
    h, w = (int(x) for x in s.split("x"))
    n = h * w * 3
    img = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert lib.phd_fill_uniform_device(img.data_ptr(), n, 1, None) == 0
    ms = ctypes.c_double()
    rc = lib.phd_debug_time_kernel(k, img.data_ptr(), h, w, ctypes.byref(cfg), 0, 20, ctypes.byref(ms))
    assert rc == 0, last_error()
    print(f"kernel {k} {h}x{w}: {1000 * ms.value:.1f} us  ({1000 * ms.value / (h * w / 1e6):.2f} us per Mpx)")
    del img
