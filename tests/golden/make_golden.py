"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own C.

Run in the build container only (needs /root/reference and `make -C oracle ref`):
    python -m tests.golden.make_golden [--only name,name,...]

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

HSV36 = {"h_partitions": 36, "s_partitions": 4, "v_partitions": 5}

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
    # round 2: the 12 MP saliency INT_MIN ordering (compare_quantities' cvttss2si,
    # src/color_quantization.c:601-611: the 51 % colour is sorted 2nd) ...
    ("dominant_3000x4000_intmin", "dominant", 3000, 4000, 1, {}, None),
    # ... and BASELINE config 5's shapes at h/s/v 36/4/5 not covered above
    ("uniform_1536x2048_hsv36", "uniform", 1536, 2048, 21, HSV36, None),
    ("structured_640x480_hsv36", "structured", 640, 480, 22, HSV36, None),
    ("dominant_1280x720_hsv36", "dominant", 1280, 720, 23, HSV36, None),
    ("structured_3000x4000_hsv36", "structured", 3000, 4000, 24, HSV36, None),
    # sides above the 8192-point LDS transforms and lengths with large prime
    # factors: the reference takes up to 120 MP in 1:5..5:1 (src/utilities.c:12,
    # 73-80) and FFTW any length (src/fft_processing.c:18-63)
    ("uniform_10000x12000", "uniform", 10000, 12000, 31, {}, None),          # four-step rows and columns
    ("structured_12000x10000", "structured", 12000, 10000, 32, {}, None),
    ("hblur_1700x8209_prime", "hblur", 1700, 8209, 33, {}, None),            # Bluestein rows (8209 prime)
    ("motion_9000x2000", "motion", 9000, 2000, 34, {}, None),                # four-step columns only
    ("structured_1201x1009_primes", "structured", 1201, 1009, 35, HSV36, None),  # Bluestein both ways, odd H
]

# get_full_report_data on planar doubles that are not k/255 (a C caller's
# 16-bit image / 65535, synth.deep): name, kind, H, W, seed, config, crops
PLANAR_CASES = [
    ("deep_structured_600x800_crops", "structured", 600, 800, 41, {},
     [dict(top=10, bottom=210, left=20, right=320), dict(top=300, bottom=599, left=400, right=799)]),
    ("deep_uniform_700x900_ds2_L50", "uniform", 700, 900, 42, {"downsample_rate": 2, "linked_list_size": 50}, None),
    ("deep_motion_1201x1009_hsv36", "motion", 1201, 1009, 43, HSV36, None),
    ("deep_dominant_1024x1536", "dominant", 1024, 1536, 44, {}, None),
    ("deep_hblur_3000x4000", "hblur", 3000, 4000, 45, {}, None),
    # round 5: finite doubles outside [0, 1] that the reference reports on --
    # negative channels (luma down to -2) and spikes on pixels downsample_rgb
    # does not sample (luma 12): the polar bins' fixed point follows the range
    ("deep_structured_neg_600x800", "structured+neg", 600, 800, 46, {}, None),
    ("deep_uniform_spike_700x900_ds2", "uniform+spike", 700, 900, 47, {"downsample_rate": 2}, None),
    ("deep_hblur_neg_3000x4000", "hblur+neg", 3000, 4000, 48, HSV36, None),
]

# get_blur_profile_visual (src/blur_profile.c:140-180) on a Blur_Profile whose
# bins hold their own index a * nr + r: the output is the (phi_bin, r_bin)
# lookup of every pixel, stored as uint16 (H, W, na, nr, radius_bin_size)
VISUAL = [(480, 640, 72, 40, 10), (401, 577, 72, 40, 8), (512, 512, 36, 20, 18), (600, 800, 72, 40, 12),
          (577, 401, 7, 3, 111)]

ERROR_SHAPES = [(349, 350), (350, 349), (2001, 400), (400, 2001), (120000, 10000), (350, 350),
                (400, 2000), (2000, 400), (10000, 12000)]


def visual_fixture():
    import ctypes as C
    L = rp.lib()
    out = {}
    for h, w, na, nr, rbs in VISUAL:
        rows = [(C.c_double * nr)(*[float(a * nr + r) for r in range(nr)]) for a in range(na)]
        ptrs = (C.POINTER(C.c_double) * na)(*[C.cast(r, C.POINTER(C.c_double)) for r in rows])
        bp = rp.Blur_Profile(na, nr, 180 // na, rbs, ptrs)
        img = L.get_blur_profile_visual(C.byref(bp), h, w)
        data = np.ctypeslib.as_array(img.contents.data, shape=(h * w,)).copy()
        L.free_image_pgm(img)
        assert np.all(data == np.rint(data)) and data.max() < 65536
        out[f"{h}x{w}_{na}_{nr}_{rbs}"] = data.reshape(h, w).astype(np.uint16)
    np.savez_compressed(os.path.join(HERE, "blur_visual.npz"), **out)
    print("wrote blur_visual", flush=True)


def main(argv=None):
    import sys
    argv = sys.argv[1:] if argv is None else argv
    only = None
    if "--only" in argv:
        only = set(argv[argv.index("--only") + 1].split(","))
    path = os.path.join(HERE, "manifest.json")
    old = {}
    if only is not None and os.path.exists(path):
        with open(path) as f:
            m0 = json.load(f)
            old = {c["name"]: c for c in m0["cases"] + m0.get("planar_cases", [])}
    manifest = {"cases": [], "errors": []}
    for name, kind, h, w, seed, kw, crops in CASES:
        entry = dict(name=name, kind=kind, height=h, width=w, seed=seed, config=kw, crops=crops)
        manifest["cases"].append(entry)
        if only is not None and name not in only:
            assert name in old, f"{name} has no fixture yet"
            continue
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
        print("wrote", name, flush=True)
    for name, kind, h, w, seed, kw, crops in PLANAR_CASES:
        entry = dict(name=name, kind=kind, height=h, width=w, seed=seed, config=kw, crops=crops)
        manifest.setdefault("planar_cases", []).append(entry)
        if only is not None and name not in only:
            assert name in old or os.path.exists(os.path.join(HERE, f"{name}.npz")), f"{name} has no fixture yet"
            continue
        img = synth.deep(kind, h, w, seed)
        r = rp.report(img, rp.Config(**kw), crops=crops)
        arrays = dict(stats=r.stats, average_saturation=np.array(r.average_saturation), hist=r.hist,
                      valid_parents=r.valid_parents, kept=r.kept, palette_hsv=r.palette_hsv,
                      palette_pct=r.palette_pct, bins=r.bins, blur_angles=r.blur_angles, blur_mags=r.blur_mags,
                      angle_bin_size=np.array(r.angle_bin_size), radius_bin_size=np.array(r.radius_bin_size),
                      image_sha=np.frombuffer(__import__("hashlib").sha256(img.tobytes()).digest(),
                                              dtype=np.uint8))
        if r.sharpness is not None:
            arrays["sharpness"] = r.sharpness
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        print("wrote", name, flush=True)
    for h, w in ERROR_SHAPES:
        manifest["errors"].append(dict(height=h, width=w, rejected=rp.error_check(h, w)))
    with open(path, "w") as f:
        json.dump(manifest, f, indent=1)
    if only is None or "blur_visual" in only:
        visual_fixture()
    print("manifest written")


if __name__ == "__main__":
    main()
