"""GPU tests of the global-memory FFTs (fft_global.hip) and the generic 2-D path
they carry: image sides above the 8192-point LDS transforms (the reference
takes up to 120 MP within 1:5..5:1, /root/reference/src/utilities.c:12,73-80)
and lengths with a prime factor above 61 (Bluestein), which FFTW handles like
any other length (src/fft_processing.c:18-63).

The full reports of such sizes are checked against the reference's own outputs
by the golden fixtures (test_gpu_parity.py: uniform_10000x12000,
structured_12000x10000, hblur_1700x8209_prime, motion_9000x2000,
structured_1201x1009_primes).  Here: the 1-D transforms against numpy's
pocketfft, determinism and the batched entry points on those sizes.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# relative to the largest output magnitude: fp64 FFTs (four-step and Bluestein
# included) land ~1e-15; the contract downstream is 1e-4 on the blur bins
FFT_RTOL = 1e-12


def _phd():
    import torch
    import photohive_dsp_amd as phd
    from photohive_dsp_amd import lib as L
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return phd, L, torch


@pytest.mark.parametrize("n,count,kind", [
    (350, 7, 0), (4096, 3, 0), (8192, 2, 0), (2000, 5, 0),
    (9000, 3, 1), (12000, 3, 1), (24000, 2, 1), (8200, 2, 1),
    (1009, 5, 2), (1201, 4, 2), (7919, 2, 2), (8209, 2, 2), (10007, 2, 2), (24494, 2, 2),
])
def test_global_fft_matches_numpy(n, count, kind):
    """Direct (one LDS pass), four-step and Bluestein plans against numpy.fft.fft."""
    phd, L, torch = _phd()
    rng = np.random.default_rng(n)
    x = rng.standard_normal((count, n)) + 1j * rng.standard_normal((count, n))
    d = torch.from_numpy(np.ascontiguousarray(x).view(np.float64).copy()).cuda()
    out = torch.empty_like(d)
    k = L.lib.phd_debug_gfft(d.data_ptr(), out.data_ptr(), n, count)
    assert k == kind, (k, L.last_error())
    got = out.cpu().numpy().view(np.complex128).reshape(count, n)
    ref = np.fft.fft(x, axis=1)
    err = np.abs(got - ref).max() / np.abs(ref).max()
    assert err < FFT_RTOL, err
    # in place gives the same bits
    assert L.lib.phd_debug_gfft(d.data_ptr(), d.data_ptr(), n, count) == kind
    np.testing.assert_array_equal(d.cpu().numpy(), out.cpu().numpy())


@pytest.mark.parametrize("shape,kind", [((1201, 1009), "structured"), ((1700, 8209), "hblur"),
                                        ((9000, 2000), "motion")])
def test_generic_path_bins_bit_identical_over_repeats(shape, kind):
    """The generic path's bins are fixed-point integer sums too: repeats agree bit for bit."""
    phd, L, torch = _phd()
    from photohive_dsp_amd import synth
    img = synth.make(kind, shape[0], shape[1], 5)
    t = torch.from_numpy(img).cuda()[None].contiguous()
    b0 = np.array(phd.report_device(t)[0].blur_profile.bins)
    for _ in range(3):
        np.testing.assert_array_equal(np.array(phd.report_device(t)[0].blur_profile.bins), b0)


def test_generic_path_against_oracle_odd_sizes():
    """Odd height with Bluestein rows (W = 1021, prime) and a four-step-free direct
    column plan with a 7 factor: the whole report against the CPU oracle."""
    phd, L, torch = _phd()
    from photohive_dsp_amd import synth
    from oracle import oracle as orc
    from tests.test_gpu_parity import assert_report_matches
    img = synth.make("motion", 1001, 1021, 8)
    rep = phd.get_report(img)
    o = orc.report(img, fft_workers=8)
    g = dict(stats=o.stats, average_saturation=np.array(o.average_saturation), valid_parents=o.valid_parents,
             palette_pct=o.palette_pct, palette_hsv=o.palette_hsv, bins=o.bins, blur_angles=o.blur_angles,
             blur_mags=o.blur_mags, angle_bin_size=np.array(o.angle_bin_size),
             radius_bin_size=np.array(o.radius_bin_size))
    assert_report_matches(rep, g)


def test_blur_batch_device_generic_sizes():
    """phd_blur_batch_device (the FFT + blur-profile path alone) on a Bluestein size
    and a four-step size gives the full report's bins."""
    phd, L, torch = _phd()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.structures import Blur_Vector
    for (h, w) in [(1201, 1009), (9000, 2000)]:
        imgs = [synth.make("structured", h, w, s) for s in (1, 2)]
        t = torch.from_numpy(np.stack(imgs)).cuda().contiguous()
        cfg = make_config()
        bins = np.zeros((2, cfg.angle_partitions, cfg.radius_partitions))
        vecs = (Blur_Vector * 20)()
        rc = L.lib.phd_blur_batch_device(t.data_ptr(), 2, h, w, 0, ctypes.byref(cfg),
                                         bins.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), vecs, None)
        assert rc == 0, L.last_error()
        for i in range(2):
            ref = np.array(phd.get_report(imgs[i]).blur_profile.bins)
            np.testing.assert_allclose(bins[i], ref, rtol=1e-12, atol=1e-14)
