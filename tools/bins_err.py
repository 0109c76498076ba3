"""Largest relative bin error per golden fixture (GPU box): the device report's
Blur_Profile bins against the reference-generated fixture, with the bin and
its magnitude, to see what bounds BINS_TIGHT_RTOL.
    python tools/bins_err.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import photohive_dsp_amd as phd  # noqa: E402
from tests.conftest import golden_case, golden_image, golden_manifest  # noqa: E402
from tests.test_gpu_parity import _crops  # noqa: E402

worst = []
for case in golden_manifest()["cases"]:
    g = golden_case(case["name"])
    rep = phd.get_report(golden_image(case), salient_characters=_crops(case), **case["config"])
    b = np.array(rep.blur_profile.bins)
    want = g["bins"]
    rel = np.abs(b - want) / np.maximum(np.abs(want), 1e-300)
    i = int(np.argmax(np.where(np.abs(want) > 0, rel, 0)))
    norm = np.max(np.abs(b - want)) / max(np.max(np.abs(want)), 1e-300)
    worst.append((rel.flat[i], case["name"]))
    print(f"{case['name']:40s} max rel {rel.flat[i]:.2e} at bin {i} (value {want.flat[i]:.3e}, max bin {np.max(np.abs(want)):.3e}) "
          f"normwise {norm:.2e}", flush=True)
print("worst", max(worst))
