"""get_full_report_data on planar doubles that are not k/255.0.

The reference computes HSV, the statistics, the luma and the FFT on whatever
doubles a C caller passes (/root/reference/src/interface.c:20-94,
src/image_processing.c:372-417,505-512,543-553).  The fixtures
(tests/golden/deep_*.npz, manifest "planar_cases") hold the reference's own
outputs on 16-bit images / 65535 (synth.deep), made by tests/golden/make_golden.py
from the reference's C.  Every call goes through the C-ABI entry point.
"""
import ctypes

import numpy as np
import pytest

from tests.conftest import golden_case, golden_manifest

pytestmark = pytest.mark.gpu

PLANAR = golden_manifest().get("planar_cases", [])


def _phd():
    import torch
    import photohive_dsp_amd as phd
    from photohive_dsp_amd import lib as L
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return phd, L


def _call(img, cfg=None, crops=None):
    """get_full_report_data on the float64 HxWx3 image's planes (Report or None)."""
    phd, L = _phd()
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Image_RGB
    c = make_config(**(cfg or {}))
    planes = [np.ascontiguousarray(img[..., k]).ravel() for k in range(3)]
    P = ctypes.POINTER(ctypes.c_double)
    im = Image_RGB(height=img.shape[0], width=img.shape[1], r=planes[0].ctypes.data_as(P),
                   g=planes[1].ctypes.data_as(P), b=planes[2].ctypes.data_as(P))
    cb = phd.set_bounding_boxes(crops) if crops else None
    ptr = L.lib.get_full_report_data(ctypes.byref(im), ctypes.byref(cb) if cb is not None else None, c.h_partitions, c.s_partitions, c.v_partitions,
                                     c.black_thresh, c.gray_thresh, c.coverage_thresh, c.linked_list_size,
                                     c.downsample_rate, c.radius_partitions, c.angle_partitions, c.quantity_weight,
                                     c.saturation_value_weight, c.fft_streak_thresh, c.magnitude_thresh,
                                     c.blur_cutoff_ratio_denom)
    if not ptr:
        return None
    return phd.Report(ptr, img.shape[0], img.shape[1])


@pytest.mark.parametrize("case", PLANAR, ids=[c["name"] for c in PLANAR])
def test_planar_doubles_match_reference_fixture(case):
    from photohive_dsp_amd import synth
    from tests.test_gpu_parity import assert_report_matches
    g = golden_case(case["name"])
    img = synth.deep(case["kind"], case["height"], case["width"], case["seed"])
    import hashlib
    assert hashlib.sha256(img.tobytes()).digest() == g["image_sha"].tobytes(), "generator drifted"
    rep = _call(img, case["config"], case["crops"])
    assert rep is not None
    assert_report_matches(rep, g)
    # what fp64 delivers: sums in another order; the reference's sequential sums of
    # 12 M doubles carry ~1e-10 relative rounding of their own
    st = rep.rgb_stats
    np.testing.assert_allclose([st.Br, st.Bg, st.Bb, st.Cr, st.Cg, st.Cb], g["stats"], rtol=1e-9)
    np.testing.assert_allclose(rep.average_saturation, float(g["average_saturation"]), rtol=1e-9)
    np.testing.assert_allclose(np.array(rep.color_palette.hsv).reshape(-1, 3), g["palette_hsv"], rtol=1e-9)


def test_planar_repeat_bit_identical():
    """The statistics, bins and vectors of the planar path do not move between runs
    (fixed-order partial sums, fixed-point bins)."""
    from photohive_dsp_amd import synth
    img = synth.deep("structured", 700, 900, 3)
    a = _call(img)
    for _ in range(3):
        b = _call(img)
        assert [a.rgb_stats.Br, a.rgb_stats.Cr, a.average_saturation] == [b.rgb_stats.Br, b.rgb_stats.Cr,
                                                                           b.average_saturation]
        assert np.array_equal(np.array(a.blur_profile.bins), np.array(b.blur_profile.bins))
        assert [(v.angle, v.magnitude) for v in a.blur_vectors] == [(v.angle, v.magnitude) for v in b.blur_vectors]


def test_planar_k255_takes_the_rgb8_pipeline():
    """Doubles that are exactly k/255.0 give the RGB8 pipeline's report bit for bit."""
    phd, L = _phd()
    from photohive_dsp_amd import synth
    u8 = synth.make("structured", 600, 800, 12)
    rep = _call(u8.astype(np.float64) / 255.0)
    ref = phd.get_report(u8)
    assert np.array_equal(np.array(rep.blur_profile.bins), np.array(ref.blur_profile.bins))
    assert rep.color_palette.quantities == ref.color_palette.quantities
    assert rep.rgb_stats.Cr == ref.rgb_stats.Cr


def test_planar_rejects_non_finite():
    """NaN in a channel: the reference's (int) casts are undefined there; NULL + message."""
    phd, L = _phd()
    from photohive_dsp_amd import synth
    img = synth.deep("uniform", 400, 400, 1)
    img[10, 10, 1] = np.nan
    assert _call(img) is None
    assert "finite" in L.last_error()


def test_planar_unsampled_spike_and_overflowing_values():
    """downsample_rate 2: a value on a pixel downsample_rgb never samples (odd
    column) reaches only the statistics and the FFT.  A finite spike (40.0)
    gets a report -- the polar bins' fixed-point scale follows the luma range
    (the deep_*_spike fixture pins its values); a value whose power spectrum
    overflows fp64 (1e300) is rejected with a message instead of infinite
    bins."""
    phd, L = _phd()
    from photohive_dsp_amd import synth
    img = synth.deep("uniform", 400, 400, 2)
    ok = _call(img, {"downsample_rate": 2})
    assert ok is not None
    img[11, 11, 0] = 40.0                             # column 11: not sampled at ds = 2 (x * 2)
    spiked = _call(img, {"downsample_rate": 2})
    assert spiked is not None
    assert spiked.color_palette.quantities == ok.color_palette.quantities   # the palette never sees it
    assert np.isfinite(np.array(spiked.blur_profile.bins)).all()
    img[11, 11, 0] = 1e300
    assert _call(img, {"downsample_rate": 2}) is None
    assert "too large" in L.last_error()
