"""Round-4 GPU tests: the device generator of the bench's structured images
 and the batch reports of those images against the
CPU oracle."""
import ctypes

import numpy as np
import pytest

from tests.test_gpu_parity import _phd, assert_report_matches

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,blur,axis", [("structured", 0, 1), ("hblur", 15, 1), ("vblur", 15, 0)])
@pytest.mark.parametrize("h,w", [(97, 131), (3000, 4000)])
def test_structured_fill_matches_synth(kind, blur, axis, h, w):
    """phd_fill_structured_device writes synth.py's bytes exactly."""
    phd, L, torch = _phd()
    from photohive_dsp_amd import synth
    if h == 3000 and kind != "hblur":
        pytest.skip("full size: the bench's kind only")
    t = torch.empty(h * w * 3, dtype=torch.uint8, device="cuda")
    assert L.lib.phd_fill_structured_device(t.data_ptr(), h, w, 2, blur, axis, None) == 0, L.last_error()
    got = t.cpu().numpy().reshape(h, w, 3)
    want = synth.make(kind, h, w, 2)
    bad = np.argwhere(got != want)
    assert bad.shape[0] == 0, f"{bad.shape[0]} bytes differ, first at {bad[:3].tolist()}"


def test_batch_reports_of_device_structured_images_against_oracle():
    """The bench's structured workload: two 4000x3000 hblur images generated on
    the device, one phd_report_batch_device call, each report against the
    oracle."""
    phd, L, torch = _phd()
    from photohive_dsp_amd import synth
    from photohive_dsp_amd.core import Report, make_config
    from photohive_dsp_amd.structures import Full_Report_Data
    from oracle import oracle as orc
    H, W, n = 3000, 4000, 2
    nb = H * W * 3
    t = torch.empty(n * nb, dtype=torch.uint8, device="cuda")
    for i in range(n):
        assert L.lib.phd_fill_structured_device(t[i * nb:].data_ptr(), H, W, 2 + i, 15, 1, None) == 0
    cfg = make_config()
    outs = (ctypes.POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()
    assert L.lib.phd_report_batch_device(t.data_ptr(), n, H, W, nb, ctypes.byref(cfg), outs, st, None) == 0, \
        L.last_error()
    reps = [Report(outs[i], H, W) for i in range(n)]      # each frees its report
    for i in range(n):
        o = orc.report(synth.make("hblur", H, W, 2 + i), fft_workers=8)
        g = dict(stats=o.stats, average_saturation=np.array(o.average_saturation),
                 valid_parents=o.valid_parents, palette_pct=o.palette_pct, palette_hsv=o.palette_hsv,
                 bins=o.bins, blur_angles=o.blur_angles, blur_mags=o.blur_mags,
                 angle_bin_size=np.array(o.angle_bin_size), radius_bin_size=np.array(o.radius_bin_size))
        assert_report_matches(reps[i], g)
