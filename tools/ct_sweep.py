"""Sweep the compile-time FFT plan variants (PHD_CT_ROWS_VARIANT /
PHD_CT_COLS_VARIANT, phd_internal.h) on the GPU box: per variant, one child
process checks the power spectrum against numpy and times the row and column
kernels (phd_debug_time_kernel).

    python tools/ct_sweep.py [--rows 0,1,2] [--cols 0,1,2] [--H 3000 --W 4000]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes, os, sys
sys.path.insert(0, %(root)r)
import numpy as np, torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from photohive_dsp_amd.core import make_config
from photohive_dsp_amd import synth
H, W = %(H)d, %(W)d
img = synth.make("structured", H, W, 6)
t = torch.from_numpy(np.ascontiguousarray(img)).cuda()
wf = W // 2 + 1
out = torch.empty(wf * H, dtype=torch.float64, device="cuda")
rc = lib.phd_debug_power_spectrum(t.data_ptr(), H, W, out.data_ptr())
assert rc == 0, (rc, last_error())
got = out.cpu().numpy().reshape(wf, H).T
k255 = np.arange(256, dtype=np.float64) / 255.0
f = img.astype(np.int64)
pgm = 0.299 * k255[f[..., 0]] + 0.587 * k255[f[..., 1]] + 0.114 * k255[f[..., 2]]
n = float(H * W)
avg = (f[..., 0].sum() / 255.0 / n + f[..., 1].sum() / 255.0 / n + f[..., 2].sum() / 255.0 / n) / 3.0
X = np.fft.rfft2(pgm - avg)
want = X.real ** 2 + X.imag ** 2
err = np.abs(got - want).max() / want.max()
cfg = make_config()
u = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
assert lib.phd_fill_uniform_device(u.data_ptr(), H * W * 3, 1, None) == 0
res = []
for k in (1, 2):
    ms = ctypes.c_double()
    assert lib.phd_debug_time_kernel(k, u.data_ptr(), H, W, ctypes.byref(cfg), 0, 20, ctypes.byref(ms)) == 0, last_error()
    res.append(1000 * ms.value)
print(f"RESULT err={err:.2e} rows_us={res[0]:.1f} cols_us={res[1]:.1f}")
"""


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", default="0")
    p.add_argument("--cols", default="0")
    p.add_argument("--H", type=int, default=3000)
    p.add_argument("--W", type=int, default=4000)
    a = p.parse_args()
    rows = [int(x) for x in a.rows.split(",")]
    cols = [int(x) for x in a.cols.split(",")]
    pairs = [(r, cols[0]) for r in rows] + [(rows[0], c) for c in cols[1:]]
    code = CHILD % {"root": ROOT, "H": a.H, "W": a.W}
    for r, c in pairs:
        # the variants are experiment switches: only the ablate build reads them
        abl = os.path.join(ROOT, "photohive_dsp_amd", "PhotoHive_DSP_lib", "libreport_data_ablate.so")
        env = dict(os.environ, PHD_CT_ROWS_VARIANT=str(r), PHD_CT_COLS_VARIANT=str(c), PHD_QUIET="1",
                   PHD_LIB=os.environ.get("PHD_LIB", abl))
        pr = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in pr.stdout.splitlines() if l.startswith("RESULT")]
        print(f"rows v{r} cols v{c}: {line[0] if line else 'FAILED rc=%d %s' % (pr.returncode, pr.stderr[-300:])}",
              flush=True)
        if pr.returncode not in (0, 1):
            break


if __name__ == "__main__":
    main()
