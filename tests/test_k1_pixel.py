"""K1's per-pixel classification (photohive_dsp_amd/csrc/k1_pixel.h), run on
the host through phd_debug_k1_pixels -- the same source the kernel compiles --
over every RGB8 triple, against the C oracle's rgb2hsv + arm_octree
(/root/reference/src/image_processing.c:384-415,
src/color_quantization.c:127-159).  No GPU: the GPU tests check the same
cells end to end through the palette sums (test_gpu_parity.py)."""
import ctypes

import numpy as np
import pytest

CFGS = [{}, {"h_partitions": 36, "s_partitions": 4, "v_partitions": 5},
        {"black_thresh": 0.25, "gray_thresh": 0.2, "h_partitions": 12},
        {"h_partitions": 5, "s_partitions": 3, "v_partitions": 2},
        {"h_partitions": 360, "s_partitions": 2, "v_partitions": 2}]


@pytest.fixture(scope="module")
def cube():
    k = np.arange(1 << 24, dtype=np.uint32)
    return np.ascontiguousarray(np.stack([(k >> 16) & 255, (k >> 8) & 255, k & 255], axis=1).astype(np.uint8))


@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: "_".join(f"{k[0]}{v}" for k, v in c.items()) or "default")
def test_k1_pixel_classification_rgb_cube(cube, cfg):
    from oracle import oracle as orc
    from photohive_dsp_amd.core import make_config
    from photohive_dsp_amd.lib import last_error, lib
    n = cube.shape[0]
    want_gid, want_hsv = orc.group_ids(cube, with_hsv=True, **cfg)
    c = make_config(**cfg)
    cell = np.empty(n, np.int32)
    h = np.empty(n)
    s = np.empty(n)
    dfr = np.empty(n, np.int32)
    assert lib.phd_debug_k1_pixels(cube.ctypes.data, n, ctypes.byref(c), cell.ctypes.data, h.ctypes.data,
                                   s.ctypes.data, dfr.ctypes.data) == 0, last_error()
    hp, sp, vp = c.h_partitions, c.s_partitions, c.v_partitions
    gs = hp * sp * vp                              # first gray / black group (HueCells)
    lh = 360 // hp
    color = cell < 4 * gs
    grp = np.where(color, cell >> 2, gs + (cell - 4 * gs) // (2 * hp))
    bad = np.nonzero(grp != want_gid)[0]
    assert bad.size == 0, f"{bad.size} group mismatches, e.g. rgb={cube[bad[:4]].tolist()}"

    # h and s: deferred pixels take the reference's own double expression
    # (bit-exact); the fast path's exact rational through an fp32 reciprocal +
    # one fp64 Newton step agrees to a few ulp
    d = dfr != 0
    np.testing.assert_array_equal(h[d], want_hsv[d, 0])
    np.testing.assert_allclose(h, want_hsv[:, 0], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(s, want_hsv[:, 1], rtol=1e-13, atol=1e-13)
    assert d.mean() < 0.1, f"{d.mean():.3%} of the cube deferred"

    # the half-bin cell c - below of each pixel (colour groups: 4 cells around
    # their hue bin, gray / black groups: 2 hp cells)
    hi = np.where(color, grp // (sp * vp), 0)
    cg = np.where(color, (cell & 3) + 2 * hi - 1, (cell - 4 * gs) % (2 * hp))
    x = 2.0 * want_hsv[:, 0] / lh
    r = np.rint(x)
    onb = np.abs(x - r) < 1e-9
    off = ~onb
    np.testing.assert_array_equal(cg[off], np.floor(x[off]).astype(np.int32))
    # on a boundary B_r the pixel sits on one side of it, as calculate_avg_hsv's
    # wrap test puts the reference's double hue (color_quantization.c:527-547)
    ok = (cg[onb] == r[onb]) | (cg[onb] == r[onb] - 1)
    assert ok.all(), f"{(~ok).sum()} boundary pixels off both sides"
