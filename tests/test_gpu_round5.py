"""Round-5 GPU tests: two library lanes on eight HIP hardware queues in a fresh
process (the bench's default configuration), the compile-time size whose
polar-bin table has too many runs per column for the column pass's run lists
(the runtime-plan fallback) against the oracle, and the column pass's two
forms (half- and full-prefetch by LDS-DMA) against each other."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.test_gpu_parity import _phd, assert_report_matches

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_lanes_eight_hw_queues_fresh_process():
    """GPU_MAX_HW_QUEUES=8 must be in the environment before HIP initialises,
    so the batch runs in a child process: 32 device-resident 4000x3000 images
    (uniform and structured), three two-lane calls and one one-lane call;
    every report field is identical between them (S-bar and the palette's
    h / s / v, fp64 sums whose atomics land in any order, within 1e-12)."""
    env = dict(os.environ, GPU_MAX_HW_QUEUES="8")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "lanes_hwq_child.py"), "32"],
                       env=env, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["hw_queues"] == "8" and d["images"] == 32
    assert d["n_diffs"] == 0, d["diffs"]


def test_column_runs_fallback_4000x3000_against_oracle():
    """radius_partitions = 160 at 4000x3000 gives spectrum columns of up to 265
    polar-bin runs, more than the compile-time column pass holds (256): the
    size takes the runtime-plan FFT.  Two calls (the second hits the cached
    decision) both match the oracle."""
    phd, L, torch = _phd()
    from photohive_dsp_amd import synth
    from oracle import oracle as orc
    H, W = 3000, 4000
    assert L.lib.phd_debug_col_runs_max(H, W, 160, 72) > 256
    img = synth.make("structured", H, W, 31)
    o = orc.report(img, fft_workers=8, radius_partitions=160)
    g = dict(stats=o.stats, average_saturation=np.array(o.average_saturation),
             valid_parents=o.valid_parents, palette_pct=o.palette_pct, palette_hsv=o.palette_hsv,
             bins=o.bins, blur_angles=o.blur_angles, blur_mags=o.blur_mags,
             angle_bin_size=np.array(o.angle_bin_size), radius_bin_size=np.array(o.radius_bin_size))
    for _ in range(2):
        rep = phd.get_report(img, radius_partitions=160)
        assert_report_matches(rep, g)


# (height, width): every compile-time column plan with a full-prefetch form, each
# with a compile-time row plan for its width
PF_SIZES = [(3000, 4000), (2000, 3000), (6000, 4000), (1536, 2048), (1080, 1920), (1280, 720),
            (720, 1280), (640, 480), (480, 640), (512, 512)]


@pytest.mark.parametrize("h,w", PF_SIZES)
def test_column_forms_bit_identical(h, w):
    """The compile-time column pass's half- and full-prefetch forms
    (phd_debug_column_form) give the same bins, max and blur vectors for a
    batch (the polar bins are fixed-point sums: bit-identical whatever the
    order), on one lane and, at the default lanes, for a split batch."""
    phd, L, torch = _phd()
    n = 4 if h * w >= 6_000_000 else 6
    # generated on the device (synth.hip): uniform and blurred structured images
    t = torch.empty((n, h, w, 3), dtype=torch.uint8, device="cuda")
    for i in range(n):
        p = t[i].data_ptr()
        rc = (L.lib.phd_fill_uniform_device(p, h * w * 3, 900 + i, None) if i % 2 == 0 else
              L.lib.phd_fill_structured_device(p, h, w, 900 + i, 15, 1, None))
        assert rc == 0
    prev = L.lib.phd_debug_column_form(0)
    try:
        half = phd.report_device(t)
        assert L.lib.phd_debug_column_form(1) == 0
        pf = phd.report_device(t)
    finally:
        L.lib.phd_debug_column_form(prev)
    for a, b in zip(half, pf):
        assert np.array_equal(np.array(a.blur_profile.bins), np.array(b.blur_profile.bins))
        assert [(v.angle, v.magnitude) for v in a.blur_vectors] == [(v.angle, v.magnitude) for v in b.blur_vectors]
        assert a.color_palette.group_ids == b.color_palette.group_ids


@pytest.mark.parametrize("kind,h,w,n", [("structured", 600, 800, 20), ("motion", 401, 577, 17)])
def test_blur_batch_two_lanes_match_one_lane(kind, h, w, n):
    """phd_blur_batch_device (config 4) splits a batch of >= 16 images over the
    two library lanes like the full report's batches: 20 and 17 images (a
    compile-time size and a runtime-plan size; halves of 10 / 10 and 8 / 9)
    give the one-lane call's bins (fp64 atomics in any order: 1e-12) and
    vectors, on two calls in a row."""
    phd, L, torch = _phd()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.core import blur_profiles_device
    imgs = np.stack([synth.make(kind, h, w, 900 + i) for i in range(n)])
    t = torch.from_numpy(imgs).cuda()
    prev = L.lib.phd_set_lanes(1)
    try:
        b1, v1 = blur_profiles_device(t)
        L.lib.phd_set_lanes(2)
        runs = [blur_profiles_device(t) for _ in range(2)]
    finally:
        L.lib.phd_set_lanes(prev)
    for b2, v2 in runs:
        np.testing.assert_allclose(b2, b1, rtol=1e-12, atol=1e-15)
        assert v2 == v1
