"""Pin the C restatement against the reference's own C -- TEST INFRASTRUCTURE ONLY.

Runs oracle.report() and ref_pipeline.report() on the same synthetic images
and checks: stats / S-bar / palette / bins bit-exact (same evaluation order),
histogram, parents, kept counts and blur counts exact, vectors identical.
Needs /root/reference (this container only).  Usage:
    python -m oracle.pin_oracle [--quick]
"""
from __future__ import annotations

import sys
import time

import numpy as np

from oracle import oracle as orc
from oracle import ref_pipeline as rp
from photohive_dsp_amd import synth

CASES = [
    # (kind, H, W, seed, config overrides)
    ("uniform", 384, 512, 1, {}),
    ("structured", 384, 512, 2, {}),
    ("hblur", 480, 640, 3, {}),
    ("vblur", 480, 640, 4, {}),
    ("motion", 401, 577, 5, {}),
    ("uniform", 401, 577, 6, {"linked_list_size": 64}),
    ("structured", 577, 401, 7, {"linked_list_size": 64}),
    ("grayish", 512, 512, 8, {}),
    ("black", 400, 400, 0, {}),
    ("dominant", 512, 768, 9, {}),
    ("uniform", 512, 512, 10, {"h_partitions": 36, "s_partitions": 4, "v_partitions": 5}),
    ("structured", 600, 800, 11, {"h_partitions": 36, "s_partitions": 4, "v_partitions": 5,
                                  "linked_list_size": 200}),
    ("structured", 720, 1280, 12, {"downsample_rate": 2}),
    ("uniform", 700, 900, 13, {"downsample_rate": 3, "linked_list_size": 50}),
    ("hblur", 512, 512, 14, {"coverage_thresh": 0.5, "radius_partitions": 20, "angle_partitions": 36}),
    ("structured", 1024, 1024, 20241125, {}),
]
BIG = [
    ("dominant", 3000, 4000, 1, {}),   # saliency INT_MIN path
    ("structured", 1080, 1920, 2, {"linked_list_size": 5000}),
]


def compare(a, b, label):
    bad = []
    for f in ("stats", "palette_hsv", "palette_pct", "bins"):
        x, y = getattr(a, f), getattr(b, f)
        if x.shape != y.shape or not np.array_equal(x, y):
            rel = np.max(np.abs(x - y) / np.maximum(np.abs(y), 1e-300)) if x.shape == y.shape else np.inf
            bad.append(f"{f}: max rel {rel:.3g}")
    if a.average_saturation != b.average_saturation:
        bad.append(f"S-bar {a.average_saturation!r} vs {b.average_saturation!r}")
    for f in ("hist", "valid_parents", "kept", "bin_counts", "blur_angles", "blur_mags"):
        x, y = getattr(a, f), getattr(b, f)
        if x.shape != y.shape or not np.array_equal(x, y):
            bad.append(f"{f} differs")
    for f in ("angle_bin_size", "radius_bin_size", "fft_max"):
        if getattr(a, f) != getattr(b, f):
            bad.append(f"{f} {getattr(a, f)} vs {getattr(b, f)}")
    print(("OK  " if not bad else "FAIL"), label, "; ".join(bad), flush=True)
    return not bad


def main(argv):
    cases = CASES if "--quick" in argv else CASES + BIG
    ok = True
    for kind, h, w, seed, kw in cases:
        img = synth.make(kind, h, w, seed)
        cfg = rp.Config(**kw)
        t0 = time.time()
        r = rp.report(img, cfg)
        t1 = time.time()
        o = orc.report(img, **kw)
        t2 = time.time()
        ok &= compare(o, r, f"{kind} {h}x{w} s={seed} {kw} (ref {t1 - t0:.2f}s, oracle {t2 - t1:.2f}s)")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
