"""K1 batch timing on the GPU box (HIP events around each K1 launch):
    python tools/k1bench.py [--lib PATH]...
hsv_stats pass (config 3 shape, 64 x 1080p) and full-report K1 (8 x 4000x3000)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.core import make_config
from photohive_dsp_amd.structures import Full_Report_Data, RGB_Statistics

lib.phd_set_lanes(1)              # each K1 launch alone on the GPU (the library's default is 2)


KIND = os.environ.get("K1KIND", "uniform")          # or hblur: SURVEY 8(d) row 2(b)'s structured images


def fill(n, h, w):
    t = torch.empty(n * h * w * 3, dtype=torch.uint8, device="cuda")
    for i in range(n):
        if KIND == "hblur":
            assert lib.phd_fill_structured_device(t[i * h * w * 3:].data_ptr(), h, w, 2 + i, 15, 1, None) == 0
        else:
            assert lib.phd_fill_uniform_device(t[i * h * w * 3:].data_ptr(), h * w * 3, i, None) == 0
    return t


def k1_avg():
    tot, cnt = ctypes.c_double(), ctypes.c_long()
    lib.phd_profile_read(0, ctypes.byref(tot), ctypes.byref(cnt))
    return 1000 * tot.value / max(cnt.value, 1)


tag = os.environ.get("PHD_LIB", "default").split("/")[-1] + f" {KIND}" + (f" grid {os.environ['K1GRID']}" if os.environ.get("K1GRID") else "")
for n, h, w in ([] if os.environ.get("K1ONLY") else [(64, 1080, 1920), (512, 1080, 1920)]):
    t = fill(n, h, w)
    st = (RGB_Statistics * n)()
    sat = (ctypes.c_double * n)()
    lib.phd_profile_kernels(1)
    for _ in range(2):
        assert lib.phd_hsv_stats_batch_device(t.data_ptr(), n, h, w, 0, st, sat, None) == 0, last_error()
    lib.phd_profile_kernels(0)
    lib.phd_profile_kernels(1)
    for _ in range(5):
        lib.phd_hsv_stats_batch_device(t.data_ptr(), n, h, w, 0, st, sat, None)
    us = k1_avg()
    print(f"[{tag}] hsv_stats {n}x{h}x{w}: {us:.1f} us/launch  {n * h * w * 3 / us / 1e3:.0f} GB/s")
    del t
n, h, w = int(os.environ.get("K1N", "64")), 3000, 4000
t = fill(n, h, w)
# K1GRID="36,4,5": config 5's finer palette grid (h/s/v partitions)
grid = [int(x) for x in os.environ.get("K1GRID", "").split(",") if x]
cfg = make_config(h_partitions=grid[0], s_partitions=grid[1], v_partitions=grid[2]) if grid else make_config()
outs = (ctypes.POINTER(Full_Report_Data) * n)()
stt = (ctypes.c_int * n)()
lib.phd_profile_kernels(0)
lib.phd_profile_kernels(63)
for _ in range(4):
    rc = lib.phd_report_batch_device(t.data_ptr(), n, h, w, 0, ctypes.byref(cfg), outs, stt, None)
    assert rc >= 0 and (rc == 0 or os.environ.get("PHD_ABLATE")), last_error()   # ablated builds fail later stages
    for i in range(n):
        if stt[i] == 0:
            lib.free_full_report(ctypes.byref(outs[i]))
us = k1_avg()
print(f"[{tag}] K1+hist {n}x{h}x{w}: {us:.1f} us/launch  {n * h * w * 3 / us / 1e3:.0f} GB/s")
from photohive_dsp_amd.lib import KERNELS
for k, name in enumerate(KERNELS):
    tot, cnt = ctypes.c_double(), ctypes.c_long()
    lib.phd_profile_read(k, ctypes.byref(tot), ctypes.byref(cnt))
    if cnt.value:
        print(f"[{tag}]   {name}: {1000 * tot.value / cnt.value:.1f} us/launch x {cnt.value // 4} per batch"
              f" = {1000 * tot.value / 4 / n:.1f} us/image")
