"""Round-3 device pieces: the polar bins' table-driven fp64 log (log_mant) and
the column pass's per-block bin windows (ColBins).  Every call goes through the
C-ABI (photohive_dsp_amd.lib)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _lib():
    import torch
    from photohive_dsp_amd import lib as L
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return L, torch


def test_log_mant_matches_host_log():
    """log_mant (phd_device.h) against numpy's log over the values the column
    passes take it of: mantissa products of up to 16 factors in [1/2, 1) and
    single powers p in [1, N^2] (the runtime-plan pass), plus the edges of the
    table's 32 intervals.  Within 4e-16 * max(1, |log x|) absolute (a few ulp;
    the bins are fixed point at 2^-30 .. 2^-41 per run)."""
    L, torch = _lib()
    rng = np.random.default_rng(3)
    prods = np.prod(rng.uniform(0.5, 1.0, (200_000, 16)), axis=1)
    powers = 10.0 ** rng.uniform(0.0, 15.0, 200_000)
    edges = np.concatenate([1.0 + np.arange(33) / 32.0, np.nextafter(1.0 + np.arange(1, 33) / 32.0, 0.0)]) / 2.0
    x = np.concatenate([prods, powers, edges, [1.0, 0.5, 2.0 ** -40, 1.4e14]])
    dx = torch.from_numpy(x).cuda()
    dy = torch.empty_like(dx)
    assert L.lib.phd_debug_log_mant(dx.data_ptr(), dy.data_ptr(), x.size) == 0, L.last_error()
    y = dy.cpu().numpy()
    want = np.log(x)
    err = np.abs(y - want) / np.maximum(1.0, np.abs(want))
    assert err.max() <= 4e-16, (err.max(), x[np.argmax(err)])


def test_mixed_batch_groups_past_64_images():
    """phd_report_batch_device_mixed runs small sizes in groups larger than 64
    (pixel budget, phd_report.cpp size_groups): 70 images of 352x352 between
    three of 400x400, every report equal to its single-image device report."""
    L, torch = _lib()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.core import report_device, reports_device_mixed
    shapes = [(352, 352)] * 35 + [(400, 400)] * 3 + [(352, 352)] * 35
    imgs = [torch.from_numpy(synth.make(("structured", "uniform", "dominant")[i % 3], h, w, 300 + i)).cuda()
            for i, (h, w) in enumerate(shapes)]
    kw = dict(h_partitions=36, s_partitions=4, v_partitions=5)
    reps = reports_device_mixed(imgs, **kw)
    for i in list(range(0, len(imgs), 7)) + [35, 36, 37, len(imgs) - 1]:
        one = report_device(imgs[i][None].contiguous(), **kw)[0]
        r = reps[i]
        assert r.color_palette.group_ids == one.color_palette.group_ids
        assert r.color_palette.quantities == one.color_palette.quantities
        np.testing.assert_allclose(np.array(r.color_palette.hsv), np.array(one.color_palette.hsv), rtol=1e-12)
        assert np.array_equal(np.array(r.blur_profile.bins), np.array(one.blur_profile.bins))
        assert r.blur_vectors == one.blur_vectors


@pytest.mark.parametrize("shape,n", [((1080, 1920), 5), ((1536, 2048), 3), ((720, 1280), 5), ((1280, 720), 5),
                                     ((640, 480), 5), ((480, 640), 5), ((512, 512), 70)])
def test_compile_time_fft_batches_match_single_reports(shape, n):
    """Config 5's sub-3-MP sizes take compile-time plans, one row and one column
    launch per group of images (launch_fft_*_ct_batch; 70 images of 512x512 make
    two groups).  Every image's bins (fixed point) and blur vectors are
    bit-identical to its single-image report's, which runs the per-image
    kernels, and its palette is the same."""
    L, torch = _lib()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.core import report_device
    h, w = shape
    kinds = ("structured", "uniform", "dominant", "hblur", "motion")
    imgs = np.stack([synth.make(kinds[i % 5], h, w, 300 + i) for i in range(n)])
    t = torch.from_numpy(imgs).cuda()
    reps = report_device(t)
    for i in sorted({0, 1, n // 2, n - 2, n - 1}):
        one = report_device(t[i:i + 1].contiguous())[0]
        r = reps[i]
        assert np.array_equal(np.array(r.blur_profile.bins), np.array(one.blur_profile.bins)), i
        assert r.blur_vectors == one.blur_vectors, i
        assert r.color_palette.group_ids == one.color_palette.group_ids, i
        assert r.color_palette.quantities == one.color_palette.quantities, i


_BATCHED_FIXTURES = ("structured_640x480_hsv36", "hblur_480x640", "vblur_480x640", "dominant_1280x720_hsv36",
                     "structured_1080x1920_L5000", "uniform_1536x2048_hsv36", "uniform_512_hsv36_4_5")


@pytest.mark.parametrize("name", _BATCHED_FIXTURES)
def test_compile_time_fft_batches_match_reference_fixtures(name):
    """The batched compile-time FFT launches (three copies of a golden image in
    one device batch, so one row and one column launch cover all three) against
    the reference's own outputs for that image, at the same bars as the
    single-image fixture test."""
    from tests.conftest import golden_case, golden_image, golden_manifest
    from tests.test_gpu_parity import BINS_NORMWISE, assert_report_matches
    from photohive_dsp_amd.core import report_device
    L, torch = _lib()
    case = next(c for c in golden_manifest()["cases"] if c["name"] == name)
    assert not case["crops"] and not case["config"].get("downsample_rate")
    g = golden_case(name)
    img = np.ascontiguousarray(golden_image(case))
    t = torch.from_numpy(np.stack([img] * 3)).cuda()
    for rep in report_device(t, **case["config"]):
        assert_report_matches(rep, g)
        bins = np.array(rep.blur_profile.bins)
        assert np.max(np.abs(bins - g["bins"])) <= BINS_NORMWISE * max(np.max(np.abs(g["bins"])), 1e-300)
