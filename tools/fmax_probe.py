"""Spectrum max (fft_max) of two 3000x4000 fixtures: ours (phd_debug_power_spectrum),
a numpy restatement with exact channel sums, and the fixture (GPU box)."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
torch.cuda.set_device(0)
from photohive_dsp_amd.lib import lib, last_error
from tests.conftest import golden_case, golden_image, golden_manifest
for name in ["dominant_3000x4000_intmin", "structured_3000x4000_hsv36"]:
    case = [c for c in golden_manifest()["cases"] if c["name"] == name][0]
    g = golden_case(name); img = golden_image(case)
    H, W = img.shape[:2]; wf = W // 2 + 1
    t = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    out = torch.empty(wf * H, dtype=torch.float64, device="cuda")
    assert lib.phd_debug_power_spectrum(t.data_ptr(), H, W, out.data_ptr()) == 0, last_error()
    p = out.cpu().numpy().reshape(wf, H).T
    # numpy restatement: rgb2pgm, remove_dc_bias, rfft2
    f = img.astype(np.float64) / 255.0
    pgm = 0.299 * f[..., 0] + 0.587 * f[..., 1] + 0.114 * f[..., 2]
    n = H * W
    avg = (f[..., 0].sum() / n + f[..., 1].sum() / n + f[..., 2].sum() / n) / 3.0
    X = np.fft.rfft2(pgm - avg)
    q = X.real ** 2 + X.imag ** 2
    i = np.unravel_index(np.argmax(q), q.shape); j = np.unravel_index(np.argmax(p), p.shape)
    print(name, "fixture fft_max", float(g["fft_max"]), "ours", p.max(), "at", j, "numpy", q.max(), "at", i,
          "rel ours-fixture", (p.max() - float(g["fft_max"])) / float(g["fft_max"]),
          "rel numpy-fixture", (q.max() - float(g["fft_max"])) / float(g["fft_max"]), flush=True)
    print("  DC ours", p[0, 0], "numpy", q[0, 0])
