"""The statistics-only pass (k_rgb_stats, stats.hip) over 4000x3000 device
images, for tools/pmc_calib.py: its non-temporal dwordx3 loads read each RGB8
byte exactly once (36 MB per image), the same per-lane pattern as K1's."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.structures import RGB_Statistics
H, W, n = 3000, 4000, 8
nb = H * W * 3
t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
assert lib.phd_fill_uniform_device(t.data_ptr(), n * nb, 1, None) == 0
st = (RGB_Statistics * n)()
sat = (ctypes.c_double * n)()
for _ in range(6):
    assert lib.phd_hsv_stats_batch_device(t.data_ptr(), n, H, W, 0, st, sat, None) == 0, last_error()
torch.cuda.synchronize()
print("ok", n, "images per launch")
