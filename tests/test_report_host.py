"""Host-side parts of the drop-in that need no GPU: get_blur_profile_visual
(src/blur_profile.c:140-180, host code in the reference as here) against the
reference's own output, and Report / to_json (core.py:23-119, 388-436) on a
Full_Report_Data built in memory.

The reference's core.py cannot be imported in this image (it needs tkinter,
matplotlib and a libreport_data.so linked against the absent libfftw3, SURVEY.md
8c), so the to_json expectation is restated from core.py:388-436 line by line:
key order, the hsv_to_rgb integers under the "H/S/V" keys, the zero padding to
100 colours / 10 sharpnesses, and the NaN correction (core.py:109-117) with its
printed line.
"""
import ctypes
import json
import math
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VIS = os.path.join(ROOT, "tests", "golden", "blur_visual.npz")


def _profile(na, nr, rbs, values):
    from photohive_dsp_amd.structures import Blur_Profile
    rows = [(ctypes.c_double * nr)(*values[a]) for a in range(na)]
    ptrs = (ctypes.POINTER(ctypes.c_double) * na)(*[ctypes.cast(r, ctypes.POINTER(ctypes.c_double)) for r in rows])
    bp = Blur_Profile(na, nr, 180 // na, rbs, ptrs)
    bp._keep = (rows, ptrs)
    return bp


@pytest.mark.parametrize("key", list(np.load(VIS).files))
def test_blur_profile_visual_matches_reference(key):
    """The reference's get_blur_profile_visual (compiled from /root/reference/src)
    rendered a profile whose bin (a, r) holds a * nr + r; ours must give the same
    (phi_bin, r_bin) for every pixel (tests/golden/make_golden.py VISUAL)."""
    from photohive_dsp_amd.lib import lib
    want = np.load(VIS)[key]
    hw, na, nr, rbs = key.split("_")
    h, w = map(int, hw.split("x"))
    na, nr, rbs = int(na), int(nr), int(rbs)
    bp = _profile(na, nr, rbs, [[float(a * nr + r) for r in range(nr)] for a in range(na)])
    img = lib.get_blur_profile_visual(ctypes.byref(bp), h, w)
    assert img
    got = np.ctypeslib.as_array(img.contents.data, shape=(h * w,)).copy().reshape(h, w)
    lib.phd_free_pgm(img)
    np.testing.assert_array_equal(got, want.astype(np.float64))


def _report_struct(n_colors, n_sharp, nan_bins=()):
    """A Full_Report_Data in Python memory (never passed to free_full_report)."""
    from photohive_dsp_amd import structures as S
    rng = np.random.default_rng(3)
    keep = []
    st = S.RGB_Statistics(*rng.random(6))
    avg = (S.Pixel_HSV * max(n_colors, 1))()
    for i in range(n_colors):
        avg[i] = S.Pixel_HSV(i, rng.random() * 360, rng.random(), rng.random())
    pct = (ctypes.c_double * max(n_colors, 1))(*rng.random(n_colors))
    cp = S.Color_Palette(n_colors, ctypes.cast(avg, ctypes.POINTER(S.Pixel_HSV)), pct)
    na, nr = 8, 5
    vals = rng.random((na, nr)).tolist()
    for a, r in nan_bins:
        vals[a][r] = math.nan
    bp = _profile(na, nr, 7, vals)
    vec = (S.Blur_Vector * 10)(*[S.Blur_Vector(int(rng.integers(-90, 90)), float(rng.random())) for _ in range(10)])
    bv = S.Blur_Vector_Group(10, vec)
    sh = (ctypes.c_double * max(n_sharp, 1))(*rng.random(n_sharp))
    shs = S.Sharpnesses(n_sharp, sh)
    fr = S.Full_Report_Data(ctypes.pointer(st), ctypes.pointer(cp), ctypes.pointer(bp), ctypes.pointer(bv),
                            0.4321, ctypes.pointer(shs) if n_sharp else None)
    keep += [st, avg, pct, cp, bp, vec, bv, sh, shs]
    return fr, keep, vals


def _expected_json(fr, h, w):
    """core.py:388-436 restated."""
    from photohive_dsp_amd.utils import hsv_to_rgb
    st = fr.rgb_stats.contents
    d = {"Height": h, "Width": w, "Average Saturation": fr.average_saturation, "Red Brightness": st.Br,
         "Green Brightness": st.Bg, "Blue Brightness": st.Bb, "Red Contrast": st.Cr, "Green Contrast": st.Cg,
         "Blue Contrast": st.Cb}
    g = fr.blur_vectors.contents
    for i in range(10):
        d[f"Blur Vector {i+1} Angle"] = g.blur_vectors[i].angle
        d[f"Blur Vector {i+1} Magnitude"] = g.blur_vectors[i].magnitude
    cp = fr.color_palette.contents
    for i in range(100):
        if i < cp.N:
            p = cp.averages[i]
            hh, ss, vv = hsv_to_rgb(p.h, p.s, p.v)
            q = cp.percentages[i]
        else:
            hh, ss, vv, q = 0, 0, 0, 0
        d[f"Color {i+1} H"], d[f"Color {i+1} S"], d[f"Color {i+1} V"] = hh, ss, vv
        d[f"Color {i+1} Percentage"] = q
    n = fr.sharpness.contents.N if fr.sharpness else 0
    for i in range(10):
        d[f"Sharpness {i+1}:"] = fr.sharpness.contents.sharpness[i] if i < n else 0.0
    return json.dumps(d, indent=4)


@pytest.mark.parametrize("n_colors,n_sharp", [(0, 0), (7, 3), (100, 10), (120, 12)])
def test_to_json_matches_reference_layout(n_colors, n_sharp):
    from photohive_dsp_amd.core import Report
    from photohive_dsp_amd.structures import Full_Report_Data
    fr, keep, _ = _report_struct(min(n_colors, 120), n_sharp)
    rep = Report(ctypes.pointer(fr), 3000, 4000)
    try:
        got = rep.to_json()
        assert got == _expected_json(fr, 3000, 4000)
        d = json.loads(got)
        assert list(d)[:9] == ["Height", "Width", "Average Saturation", "Red Brightness", "Green Brightness",
                               "Blue Brightness", "Red Contrast", "Green Contrast", "Blue Contrast"]
        assert len(d) == 9 + 20 + 400 + 10
    finally:
        rep.data_ptr = ctypes.POINTER(Full_Report_Data)()      # Python-owned memory: do not free


def test_nan_bins_corrected_with_reference_message(capsys):
    """core.py:109-117: each NaN bin is printed and replaced by 0."""
    from photohive_dsp_amd.core import Report
    from photohive_dsp_amd.structures import Full_Report_Data
    fr, keep, vals = _report_struct(3, 0, nan_bins=[(1, 2), (6, 0)])
    rep = Report(ctypes.pointer(fr), 400, 500)
    try:
        out = capsys.readouterr().out
        assert "NaN found at angle 1, radius 2. Correcting to 0." in out
        assert "NaN found at angle 6, radius 0. Correcting to 0." in out
        assert rep.blur_profile.bins[1][2] == 0.0 and rep.blur_profile.bins[6][0] == 0.0
        assert rep.blur_profile.bins[0][0] == vals[0][0]
    finally:
        rep.data_ptr = ctypes.POINTER(Full_Report_Data)()
