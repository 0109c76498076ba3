"""Python driver for the C restatement (oracle/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Importable on the GPU box (no dependency on /root/reference): tests, smoke()
and bench.py's cpu_baseline use it as the checker.  The 2-D DFT (FFTW in the
reference, src/fft_processing.c:34-50) is numpy/scipy rfft2.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liboracle.so")


class OrcConfig(C.Structure):
    _fields_ = [("h_parts", C.c_int), ("s_parts", C.c_int), ("v_parts", C.c_int),
                ("black_thresh", C.c_double), ("gray_thresh", C.c_double), ("coverage", C.c_double),
                ("linked_list_size", C.c_int), ("downsample_rate", C.c_int),
                ("radius_parts", C.c_int), ("angle_parts", C.c_int),
                ("quantity_weight", C.c_float), ("sv_weight", C.c_float),
                ("streak_thresh", C.c_double), ("mag_thresh", C.c_double), ("cutoff_denom", C.c_int)]


class OrcPalette(C.Structure):
    _fields_ = [("total_length", C.c_int), ("n_hsv", C.c_int), ("average_saturation", C.c_double),
                ("n_parents", C.c_int), ("hist", C.POINTER(C.c_int)), ("parents", C.POINTER(C.c_int)),
                ("kept", C.POINTER(C.c_int)), ("hsv", C.POINTER(C.c_double)),
                ("pct", C.POINTER(C.c_double))]


DEFAULTS = dict(h_partitions=18, s_partitions=2, v_partitions=3, black_thresh=0.1, gray_thresh=0.1,
                coverage_thresh=0.95, linked_list_size=1000, downsample_rate=1,
                radius_partitions=40, angle_partitions=72, quantity_weight=0.1,
                saturation_value_weight=0.9, fft_streak_thresh=1.20, magnitude_thresh=0.3,
                blur_cutoff_ratio_denom=2)   # /root/reference/core.py:442-448


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


_lib = None


def use_build(opt: str = "O2") -> None:
    """Select the restatement's build: "O2" (liboracle.so) or "O0"
    (liboracle_O0.so, the optimisation level the reference ships at).
    Only bench.py's cpu_baseline leg switches builds."""
    global SO, _lib
    SO = os.path.join(HERE, "liboracle.so" if opt == "O2" else f"liboracle_{opt}.so")
    _lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        L = C.CDLL(SO)
        P = C.POINTER
        u8p = P(C.c_uint8)
        L.orc_precheck.argtypes = [C.c_int, C.c_int]
        L.orc_rgb_stats.argtypes = [u8p, C.c_int, C.c_int, P(C.c_double)]
        L.orc_palette_run.argtypes = [u8p, C.c_int, C.c_int, P(OrcConfig), P(OrcPalette)]
        L.orc_palette_free.argtypes = [P(OrcPalette)]
        L.orc_pgm_dc.argtypes = [u8p, C.c_int, C.c_int, C.c_double, P(C.c_double)]
        L.orc_blur_profile.argtypes = [P(C.c_double), C.c_int, C.c_int, C.c_int, C.c_int,
                                       P(C.c_double), P(C.c_longlong), P(C.c_double),
                                       P(C.c_int), P(C.c_int)]
        L.orc_blur_bin_of.argtypes = [C.c_int] * 6 + [P(C.c_int), P(C.c_int)]
        L.orc_vectorize.argtypes = [P(C.c_double), C.c_int, C.c_int, C.c_double, C.c_double,
                                    C.c_int, P(C.c_int), P(C.c_float)]
        L.orc_newton_int_sqrt.argtypes = [C.c_double]
        L.orc_group_ids.argtypes = [u8p, C.c_long, P(OrcConfig), P(C.c_int), P(C.c_double)]
        L.orc_sharpness.argtypes = [u8p, C.c_int, C.c_int, C.c_int] + [P(C.c_int)] * 4 + [P(C.c_double)]
        _lib = L
    return _lib


def make_config(**kw) -> OrcConfig:
    c = dict(DEFAULTS)
    c.update(kw)
    return OrcConfig(c["h_partitions"], c["s_partitions"], c["v_partitions"], c["black_thresh"],
                     c["gray_thresh"], c["coverage_thresh"], c["linked_list_size"],
                     c["downsample_rate"], c["radius_partitions"], c["angle_partitions"],
                     c["quantity_weight"], c["saturation_value_weight"], c["fft_streak_thresh"],
                     c["magnitude_thresh"], c["blur_cutoff_ratio_denom"])


def _u8(img: np.ndarray):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    return img, img.ctypes.data_as(C.POINTER(C.c_uint8))


@dataclass
class OracleReport:
    stats: np.ndarray
    average_saturation: float
    hist: np.ndarray
    valid_parents: np.ndarray
    kept: np.ndarray
    palette_hsv: np.ndarray
    palette_pct: np.ndarray
    bins: np.ndarray
    bin_counts: np.ndarray
    blur_angles: np.ndarray
    blur_mags: np.ndarray
    fft_max: float
    angle_bin_size: int
    radius_bin_size: int
    sharpness: np.ndarray | None = None


def stats(img):
    img, p = _u8(img)
    out = np.zeros(6)
    lib().orc_rgb_stats(p, img.shape[0], img.shape[1], out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def palette(img, **kw):
    img, p = _u8(img)
    cfg = make_config(**kw)
    pal = OrcPalette()
    rc = lib().orc_palette_run(p, img.shape[0], img.shape[1], C.byref(cfg), C.byref(pal))
    if rc != 0:
        raise ValueError(f"orc_palette_run rc={rc}")
    n, tl = pal.n_parents, pal.total_length
    res = dict(
        average_saturation=pal.average_saturation,
        hist=np.ctypeslib.as_array(pal.hist, shape=(tl,)).astype(np.int64),
        valid_parents=np.ctypeslib.as_array(pal.parents, shape=(n,)).astype(np.int64),
        kept=np.ctypeslib.as_array(pal.kept, shape=(n,)).astype(np.int64),
        palette_hsv=np.ctypeslib.as_array(pal.hsv, shape=(n * 3,)).reshape(n, 3).copy(),
        palette_pct=np.ctypeslib.as_array(pal.pct, shape=(n,)).copy(),
    )
    lib().orc_palette_free(C.byref(pal))
    return res


def group_ids(rgb: np.ndarray, with_hsv: bool = False, **kw):
    """HSV group id (and h, s, v) of every pixel of an (..., 3) u8 array."""
    flat, p = _u8(rgb.reshape(-1, 3))
    n = flat.shape[0]
    gid = np.empty(n, dtype=np.int32)
    hsv = np.empty((n, 3)) if with_hsv else None
    cfg = make_config(**kw)
    lib().orc_group_ids(p, n, C.byref(cfg), gid.ctypes.data_as(C.POINTER(C.c_int)),
                        hsv.ctypes.data_as(C.POINTER(C.c_double)) if with_hsv else None)
    return (gid, hsv) if with_hsv else gid


def power_spectrum(pgm: np.ndarray, workers: int = 1) -> np.ndarray:
    try:
        import scipy.fft as sfft
        X = sfft.rfft2(pgm, workers=workers)
    except ImportError:  # pragma: no cover
        X = np.fft.rfft2(pgm)
    return X.real * X.real + X.imag * X.imag


def pgm_dc(img, avg: float) -> np.ndarray:
    img, p = _u8(img)
    H, W = img.shape[:2]
    out = np.empty((H, W))
    lib().orc_pgm_dc(p, H, W, avg, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def blur_profile(power: np.ndarray, nr: int, na: int):
    H, wf = power.shape
    power = np.ascontiguousarray(power, dtype=np.float64)
    bins = np.zeros(na * nr)
    counts = np.zeros(na * nr, dtype=np.int64)
    fmax = C.c_double()
    abs_, rbs = C.c_int(), C.c_int()
    rc = lib().orc_blur_profile(power.ctypes.data_as(C.POINTER(C.c_double)), H, wf, nr, na,
                                bins.ctypes.data_as(C.POINTER(C.c_double)),
                                counts.ctypes.data_as(C.POINTER(C.c_longlong)),
                                C.byref(fmax), C.byref(abs_), C.byref(rbs))
    if rc != 0:
        raise ValueError("radius/angle bin outside the table")
    return bins.reshape(na, nr), counts.reshape(na, nr), fmax.value, abs_.value, rbs.value


def vectorize(bins: np.ndarray, streak: float, mag: float, denom: int):
    na, nr = bins.shape
    b = np.ascontiguousarray(bins, dtype=np.float64)
    ang = np.zeros(10, dtype=np.int32)
    mg = np.zeros(10, dtype=np.float32)
    lib().orc_vectorize(b.ctypes.data_as(C.POINTER(C.c_double)), na, nr, streak, mag, denom,
                        ang.ctypes.data_as(C.POINTER(C.c_int)), mg.ctypes.data_as(C.POINTER(C.c_float)))
    return ang, mg


def sharpness(img, crops):
    img, p = _u8(img)
    n = len(crops)
    arrs = [np.array([c[k] for c in crops], dtype=np.int32) for k in ("top", "bottom", "left", "right")]
    out = np.zeros(n)
    rc = lib().orc_sharpness(p, img.shape[0], img.shape[1], n,
                             *[a.ctypes.data_as(C.POINTER(C.c_int)) for a in arrs],
                             out.ctypes.data_as(C.POINTER(C.c_double)))
    if rc != 0:
        raise ValueError("crop outside the image")
    return out


def report(img: np.ndarray, crops=None, fft_workers: int = 1, **kw) -> OracleReport | None:
    """Full report in the stage order of src/interface.c:20-94."""
    c = dict(DEFAULTS)
    c.update(kw)
    H, W = img.shape[:2]
    if lib().orc_precheck(H, W):
        return None
    st = stats(img)
    pal = palette(img, **kw)
    sh = sharpness(img, crops) if crops is not None else None
    avg = (st[0] + st[1] + st[2]) / 3.0
    power = power_spectrum(pgm_dc(img, avg), workers=fft_workers)
    nr, na = c["radius_partitions"], c["angle_partitions"]
    bins, counts, fmax, abs_, rbs = blur_profile(power, nr, na)
    ang, mg = vectorize(bins, c["fft_streak_thresh"], c["magnitude_thresh"], c["blur_cutoff_ratio_denom"])
    return OracleReport(stats=st, average_saturation=pal["average_saturation"], hist=pal["hist"],
                        valid_parents=pal["valid_parents"], kept=pal["kept"],
                        palette_hsv=pal["palette_hsv"], palette_pct=pal["palette_pct"],
                        bins=bins, bin_counts=counts, blur_angles=ang, blur_mags=mg, fft_max=fmax,
                        angle_bin_size=abs_, radius_bin_size=rbs, sharpness=sh)
