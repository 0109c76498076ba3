"""Kernel micro-benchmark / ablation on the GPU box:
    python tools/kbench.py KERNEL MASK [MASK ...]   (KERNEL: 0 hsv_stats, 1 fft_rows, 2 fft_cols)"""
import ctypes, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.core import make_config
H, W = (int(x) for x in os.environ.get("KB_SIZE", "3000x4000").split("x"))   # KB_SIZE=HxW
n = H * W * 3
img = torch.empty(n, dtype=torch.uint8, device="cuda")
assert lib.phd_fill_uniform_device(img.data_ptr(), n, 1, None) == 0
cfg = make_config()
k = int(sys.argv[1])
for m in sys.argv[2:]:
    ms = ctypes.c_double()
    rc = lib.phd_debug_time_kernel(k, img.data_ptr(), H, W, ctypes.byref(cfg), int(m), 20, ctypes.byref(ms))
    assert rc == 0, last_error()
    print(f"kernel {k} ablate {m}: {1000 * ms.value:.1f} us  ({n / (ms.value * 1e-3) / 1e9:.0f} GB/s on the RGB8 bytes)")
