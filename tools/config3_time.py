"""BASELINE config 3 timed alone (as bench.py's config3): 512 x 1080p device
images through phd_hsv_stats_batch_device; prints the wall time per call and
the statistics kernel's average launch time (the library's HIP events)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.structures import RGB_Statistics
n, h, w, iters = 512, 1080, 1920, 20
gap = float(os.environ.get("CFG3_GAP_US", "0")) * 1e-6     # host idle between calls (clock-state probe)
nb = h * w * 3
t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
for i in range(n):
    assert lib.phd_fill_uniform_device(t[i * nb:].data_ptr(), nb, i, None) == 0
st = (RGB_Statistics * n)()
sat = (ctypes.c_double * n)()
run = lambda: lib.phd_hsv_stats_batch_device(t.data_ptr(), n, h, w, 0, st, sat, None)
for _ in range(3):
    assert run() == 0, last_error()
lib.phd_profile_kernels(0)
lib.phd_profile_kernels(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    run()
    if gap:
        time.sleep(gap)
wall = (time.perf_counter() - t0) / iters
tot, cnt = ctypes.c_double(), ctypes.c_long()
lib.phd_profile_read(0, ctypes.byref(tot), ctypes.byref(cnt))
lib.phd_profile_kernels(0)
us = 1000 * tot.value / max(cnt.value, 1)
lib_name = os.path.basename(os.environ.get("PHD_LIB", "libreport_data.so"))
print(f"[{lib_name} gap {gap * 1e6:.0f} us] config3 wall {1000 * wall:.3f} ms/call, stats kernel {us:.1f} us/launch, "
      f"{n / wall:.0f} images/s, kernel frac {n * nb / (us * 1e-6) / 8e12:.3f}")
