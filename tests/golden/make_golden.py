"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own C.

Run in the build container only (needs /root/reference and `make -C oracle ref`):
    python -m tests.golden.make_golden

Each case stores its input as a generator spec (photohive_dsp_amd.synth) and
the reference outputs of oracle/ref_pipeline.py (the reference's own functions
compiled from /root/reference/src at -O0; DFT = numpy.fft.rfft2 since FFTW is
absent from the image).  No reference source text is stored -- only data.
"""
from __future__ import annotations

import json
import os

import numpy as np

from oracle import ref_pipeline as rp
from photohive_dsp_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    # name, kind, H, W, seed, config overrides, crops
    ("uniform_1024", "uniform", 1024, 1024, 20241125, {}, None),                 # BASELINE config 1
    ("uniform_384x512", "uniform", 384, 512, 1, {}, None),
    ("structured_384x512", "structured", 384, 512, 2, {}, None),
    ("hblur_480x640", "hblur", 480, 640, 3, {}, None),
    ("vblur_480x640", "vblur", 480, 640, 4, {}, None),
    ("motion_401x577_odd", "motion", 401, 577, 5, {}, None),
    ("uniform_401x577_L64", "uniform", 401, 577, 6, {"linked_list_size": 64}, None),
    ("structured_577x401_L64", "structured", 577, 401, 7, {"linked_list_size": 64}, None),
    ("grayish_512", "grayish", 512, 512, 8, {}, None),
    ("black_400", "black", 400, 400, 0, {}, None),
    ("dominant_512x768", "dominant", 512, 768, 9, {}, None),
    ("uniform_512_hsv36_4_5", "uniform", 512, 512, 10,
     {"h_partitions": 36, "s_partitions": 4, "v_partitions": 5}, None),
    ("structured_600x800_hsv36_L200", "structured", 600, 800, 11,
     {"h_partitions": 36, "s_partitions": 4, "v_partitions": 5, "linked_list_size": 200}, None),
    ("structured_720x1280_ds2", "structured", 720, 1280, 12, {"downsample_rate": 2}, None),
    ("uniform_700x900_ds3_L50", "uniform", 700, 900, 13, {"downsample_rate": 3, "linked_list_size": 50}, None),
    ("hblur_512_cov05_r20_a36", "hblur", 512, 512, 14,
     {"coverage_thresh": 0.5, "radius_partitions": 20, "angle_partitions": 36}, None),
    ("structured_1080x1920_L5000", "structured", 1080, 1920, 2, {"linked_list_size": 5000}, None),
    ("structured_crops_600x800", "structured", 600, 800, 15, {},
     [dict(top=10, bottom=210, left=20, right=320), dict(top=300, bottom=599, left=400, right=799),
      dict(top=0, bottom=600, left=0, right=800)]),
]

ERROR_SHAPES = [(349, 350), (350, 349), (2001, 400), (400, 2001), (120000, 10000), (350, 350),
                (400, 2000), (2000, 400), (10000, 12000)]


def main():
    manifest = {"cases": [], "errors": []}
    for name, kind, h, w, seed, kw, crops in CASES:
        img = synth.make(kind, h, w, seed)
        r = rp.report(img, rp.Config(**kw), crops=crops)
        arrays = dict(stats=r.stats, average_saturation=np.array(r.average_saturation), hist=r.hist,
                      valid_parents=r.valid_parents, kept=r.kept, palette_hsv=r.palette_hsv,
                      palette_pct=r.palette_pct, bins=r.bins, bin_counts=r.bin_counts,
                      blur_angles=r.blur_angles, blur_mags=r.blur_mags, fft_max=np.array(r.fft_max),
                      angle_bin_size=np.array(r.angle_bin_size),
                      radius_bin_size=np.array(r.radius_bin_size),
                      image_sha=np.frombuffer(__import__("hashlib").sha256(img.tobytes()).digest(),
                                              dtype=np.uint8))
        if r.sharpness is not None:
            arrays["sharpness"] = r.sharpness
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        manifest["cases"].append(dict(name=name, kind=kind, height=h, width=w, seed=seed, config=kw,
                                      crops=crops))
        print("wrote", name, flush=True)
    for h, w in ERROR_SHAPES:
        manifest["errors"].append(dict(height=h, width=w, rejected=rp.error_check(h, w)))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("manifest written")


if __name__ == "__main__":
    main()
