"""Reference-driven full report -- TEST INFRASTRUCTURE ONLY.

Runs the REFERENCE's own C functions (oracle/_ref/libphd_ref.so, compiled from
/root/reference/src at -O0 by oracle/Makefile) in the stage order of
``get_full_report_data`` (/root/reference/src/interface.c:20-94), with two
substitutions for code this image cannot build:

* the 2-D DFT of ``pgm_fft`` (src/fft_processing.c:18-63, FFTW3 r2c, unnormalised,
  e^{-i}) is ``numpy.fft.rfft2`` -- same H x (W/2+1) layout, sign and scale;
  the power is formed exactly as src/fft_processing.c:48-50 does (re*re+im*im).
* ``pgm_normalize_fft`` (src/fft_processing.c:173-213) is restated below.

Used to generate the golden fixtures in tests/golden/ and to pin the plain-C
restatement in oracle/phd_oracle.c.  Needs /root/reference (this container
only); never imported by the product or on the GPU box.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(HERE, "_ref", "libphd_ref.so")


# --- ctypes mirrors of the reference structs (src/*.h) ----------------------
class Pixel_HSV(C.Structure):
    _fields_ = [("parent_id", C.c_int), ("h", C.c_double), ("s", C.c_double), ("v", C.c_double)]


class Image_RGB(C.Structure):
    _fields_ = [("height", C.c_int), ("width", C.c_int),
                ("r", C.POINTER(C.c_double)), ("g", C.POINTER(C.c_double)), ("b", C.POINTER(C.c_double))]


class Image_HSV(C.Structure):
    _fields_ = [("height", C.c_int), ("width", C.c_int), ("pixels", C.POINTER(Pixel_HSV))]


class Image_PGM(C.Structure):
    _fields_ = [("height", C.c_int), ("width", C.c_int), ("data", C.POINTER(C.c_double))]


class RGB_Statistics(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("Br", "Bg", "Bb", "Cr", "Cg", "Cb")]


class HSV_Linked_List(C.Structure):
    pass


HSV_Linked_List._fields_ = [("pixels", C.POINTER(Pixel_HSV)), ("num_pixels", C.c_int),
                            ("array_size", C.c_int), ("i", C.c_int),
                            ("next", C.POINTER(HSV_Linked_List))]


class Octree_Group(C.Structure):
    _fields_ = [("id", C.c_int), ("quantity", C.c_int), ("h", C.c_double), ("s", C.c_double),
                ("v", C.c_double), ("head", C.POINTER(HSV_Linked_List)),
                ("cur", C.POINTER(HSV_Linked_List)), ("is_valid_parent", C.c_bool),
                ("crossed_zero", C.c_bool)]


class Octree(C.Structure):
    _fields_ = [("groups", C.POINTER(Octree_Group)), ("valid_parents", C.POINTER(C.c_int)),
                ("len_valid_parents", C.c_int), ("Lh", C.c_double), ("Ls", C.c_double),
                ("Lv", C.c_double), ("num_h", C.c_int), ("num_s", C.c_int), ("num_v", C.c_int),
                ("num_grays", C.c_int), ("total_length", C.c_int),
                ("black_thresh", C.c_double), ("gray_thresh", C.c_double)]


class Color_Palette(C.Structure):
    _fields_ = [("N", C.c_int), ("averages", C.POINTER(Pixel_HSV)),
                ("percentages", C.POINTER(C.c_double))]


class Polar_Coord(C.Structure):
    _fields_ = [("r_sq", C.c_int), ("phi", C.c_double)]


class Cartesian_To_Polar(C.Structure):
    _fields_ = [("height", C.c_uint), ("width", C.c_uint), ("data", C.POINTER(Polar_Coord))]


class Blur_Profile(C.Structure):
    _fields_ = [("num_angle_bins", C.c_int), ("num_radius_bins", C.c_int),
                ("angle_bin_size", C.c_int), ("radius_bin_size", C.c_int),
                ("bins", C.POINTER(C.POINTER(C.c_double)))]


class Blur_Vector(C.Structure):
    _fields_ = [("angle", C.c_int), ("magnitude", C.c_float)]


class Blur_Vector_Group(C.Structure):
    _fields_ = [("len_vectors", C.c_int), ("blur_vectors", C.POINTER(Blur_Vector))]


class Crop_Boundaries(C.Structure):
    _fields_ = [("N", C.c_int), ("top", C.POINTER(C.c_int)), ("bottom", C.POINTER(C.c_int)),
                ("left", C.POINTER(C.c_int)), ("right", C.POINTER(C.c_int))]


class Sharpnesses(C.Structure):
    _fields_ = [("N", C.c_int), ("sharpness", C.POINTER(C.c_double))]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(f"{REF_SO} missing: run `make -C oracle ref` (needs /root/reference)")
        L = C.CDLL(REF_SO)
        P = C.POINTER
        L.pre_compute_error_checks.restype = C.c_bool
        L.pre_compute_error_checks.argtypes = [P(Image_RGB)]
        L.downsample_rgb.restype = P(Image_RGB)
        L.downsample_rgb.argtypes = [P(Image_RGB), C.c_short]
        L.free_image_rgb.argtypes = [P(Image_RGB)]
        L.rgb2hsv.restype = P(Image_HSV)
        L.rgb2hsv.argtypes = [P(Image_RGB)]
        L.free_image_hsv.argtypes = [P(Image_HSV)]
        L.rgb2pgm.restype = P(Image_PGM)
        L.rgb2pgm.argtypes = [P(Image_RGB)]
        L.create_pgm_image.restype = P(Image_PGM)
        L.create_pgm_image.argtypes = [C.c_int, C.c_int]
        L.free_image_pgm.argtypes = [P(Image_PGM)]
        L.get_hsv_average.restype = C.c_double
        L.get_hsv_average.argtypes = [P(Image_HSV)]
        L.get_rgb_statistics.restype = P(RGB_Statistics)
        L.get_rgb_statistics.argtypes = [P(Image_RGB)]
        L.initialize_octree.restype = P(Octree)
        L.initialize_octree.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_double]
        L.arm_octree.argtypes = [P(Image_HSV), P(Octree), C.c_int]
        L.find_valid_octree_parents.argtypes = [P(Octree), C.c_int, C.c_double]
        L.group_irregular_pixels.argtypes = [P(Octree)]
        L.calculate_avg_hsv.restype = P(Color_Palette)
        L.calculate_avg_hsv.argtypes = [P(Octree), P(Image_HSV)]
        L.free_octree.argtypes = [P(Octree)]
        L.free_color_palette.argtypes = [P(Color_Palette)]
        L.remove_dc_bias.argtypes = [P(Image_PGM), C.c_double]
        L.cartesian_to_polar_conversion.restype = P(Cartesian_To_Polar)
        L.cartesian_to_polar_conversion.argtypes = [C.c_uint, C.c_uint]
        L.free_cartesian_to_polar.argtypes = [P(Cartesian_To_Polar)]
        L.calculate_blur_profile.restype = P(Blur_Profile)
        L.calculate_blur_profile.argtypes = [P(Cartesian_To_Polar), P(Image_PGM), C.c_int, C.c_int]
        L.vectorize_blur_profile.restype = P(Blur_Vector_Group)
        L.vectorize_blur_profile.argtypes = [P(Blur_Profile), C.c_double, C.c_double, C.c_int]
        L.free_blur_profile.argtypes = [P(Blur_Profile)]
        L.free_blur_vector_group.argtypes = [P(Blur_Vector_Group)]
        L.get_blur_profile_visual.restype = P(Image_PGM)
        L.get_blur_profile_visual.argtypes = [P(Blur_Profile), C.c_int, C.c_int]
        L.get_variance_sharpness.restype = P(Sharpnesses)
        L.get_variance_sharpness.argtypes = [P(Image_PGM), P(Crop_Boundaries)]
        L.newton_int_sqrt.restype = C.c_int
        L.newton_int_sqrt.argtypes = [C.c_double]
        _lib = L
    return _lib


# --- configuration (defaults of get_report, /root/reference/core.py:442-448) --
@dataclass
class Config:
    h_partitions: int = 18
    s_partitions: int = 2
    v_partitions: int = 3
    black_thresh: float = 0.1
    gray_thresh: float = 0.1
    coverage_thresh: float = 0.95
    linked_list_size: int = 1000
    downsample_rate: int = 1
    radius_partitions: int = 40
    angle_partitions: int = 72
    quantity_weight: float = 0.1
    saturation_value_weight: float = 0.9
    fft_streak_thresh: float = 1.20
    magnitude_thresh: float = 0.3
    blur_cutoff_ratio_denom: int = 2


@dataclass
class RefReport:
    stats: np.ndarray                      # Br Bg Bb Cr Cg Cb
    average_saturation: float
    hist: np.ndarray                       # arm_octree quantities per group (TL)
    valid_parents: np.ndarray              # ordered palette group ids
    kept: np.ndarray                       # pixels left in each parent's list
    palette_hsv: np.ndarray                # (N, 3)
    palette_pct: np.ndarray                # (N,)
    bins: np.ndarray                       # (na, nr)
    bin_counts: np.ndarray                 # (na, nr) image-independent counts
    blur_angles: np.ndarray                # (10,) int
    blur_mags: np.ndarray                  # (10,) float32
    fft_max: float
    angle_bin_size: int
    radius_bin_size: int
    sharpness: np.ndarray | None = None
    extra: dict = field(default_factory=dict)


def _image_rgb(img: np.ndarray):
    """u8 HxWx3 -> reference Image_RGB of planar doubles k/255.0 (utils.py:30-46);
    a float64 HxWx3 image is passed as the doubles themselves (a C caller's)."""
    f = img if img.dtype == np.float64 else img.astype(np.float64) / 255.0
    planes = [np.ascontiguousarray(f[..., c]).ravel() for c in range(3)]
    P = C.POINTER(C.c_double)
    im = Image_RGB(img.shape[0], img.shape[1], *[p.ctypes.data_as(P) for p in planes])
    return im, planes


_libm = C.CDLL("libm.so.6")
_libm.log.restype = C.c_double
_libm.log.argtypes = [C.c_double]


def _libm_log(x: float) -> float:
    return _libm.log(float(x))


_glibc_log = np.frompyfunc(_libm_log, 1, 1)


def normalize_power(power: np.ndarray) -> tuple[np.ndarray, float]:
    """Restatement of pgm_normalize_fft (src/fft_processing.c:173-213)."""
    flat = power.ravel()
    mx = float(flat[flat.size // 2])          # seed, :174-175
    m = float(np.max(flat))
    if m > mx:                                 # strict '<' scan, :181-184
        mx = m
    with np.errstate(divide="ignore"):
        gs = 1.0 / (2.0 * _libm_log(np.sqrt(mx) + 1.0)) if mx > 0 else np.inf   # :192
    out = np.zeros_like(flat)
    big = flat >= 1.0                          # :197-198, glibc log like the reference
    out[big] = _glibc_log(flat[big]).astype(np.float64) * gs
    return out.reshape(power.shape), mx


def _walk_kept(group) -> int:
    n = 0
    node = group.head
    while node:
        n += node.contents.num_pixels
        node = node.contents.next
    return n


def blur_counts(h: int, wf: int, nr: int, na: int) -> np.ndarray:
    """Per-bin element counts of calculate_blur_profile (src/blur_profile.c:87-98),
    evaluated with the reference's own c2p table and newton_int_sqrt."""
    L = lib()
    conv = L.cartesian_to_polar_conversion(wf, h)
    n = h * wf
    buf = np.ctypeslib.as_array(C.cast(conv.contents.data, C.POINTER(C.c_char * (16 * n))).contents)
    rec = np.frombuffer(bytes(buf), dtype=np.dtype([("r_sq", "<i4"), ("pad", "<i4"), ("phi", "<f8")]))
    L.free_cartesian_to_polar(conv)
    rbss = float((wf * wf + (h * h) // 4) // (nr * nr))
    phi_bin = ((rec["phi"] + 3.14159265 * np.float64(np.float32(0.5))) / 3.14159265
               * float(na - 1)).astype(np.int64)
    uniq, inv = np.unique(rec["r_sq"], return_inverse=True)
    rb = np.array([L.newton_int_sqrt(float(v) / rbss) for v in uniq], dtype=np.int64)[inv]
    rb[rb == nr] -= 1
    counts = np.zeros((na, nr), dtype=np.int64)
    np.add.at(counts, (phi_bin, rb), 1)
    return counts


def report(img: np.ndarray, cfg: Config | None = None, crops=None, want_counts: bool = True) -> RefReport | None:
    """The reference pipeline of src/interface.c:20-94 on a u8 image (or float64 planes)."""
    cfg = cfg or Config()
    L = lib()
    im, _keep = _image_rgb(img)
    pim = C.pointer(im)
    if L.pre_compute_error_checks(pim):                        # interface.c:27
        return None
    ds = L.downsample_rgb(pim, cfg.downsample_rate) if cfg.downsample_rate > 1 else pim
    hsv = L.rgb2hsv(ds)                                         # :46
    pgm = L.rgb2pgm(pim)                                        # :50
    st = L.get_rgb_statistics(pim).contents                     # :55
    stats = np.array([st.Br, st.Bg, st.Bb, st.Cr, st.Cg, st.Cb])
    s_bar = L.get_hsv_average(hsv)                              # :60

    # get_color_palette, step by step (src/color_quantization.c:652-684)
    C.c_float.in_dll(L, "QUANTITY_WEIGHT").value = cfg.quantity_weight
    C.c_float.in_dll(L, "SATURATION_VALUE_WEIGHT").value = cfg.saturation_value_weight
    oc = L.initialize_octree(cfg.h_partitions, cfg.s_partitions, cfg.v_partitions,
                             cfg.black_thresh, cfg.gray_thresh)
    L.arm_octree(hsv, oc, cfg.linked_list_size)
    tl = oc.contents.total_length
    hist = np.array([oc.contents.groups[i].quantity for i in range(tl)], dtype=np.int64)
    n_hsv = hsv.contents.height * hsv.contents.width
    L.find_valid_octree_parents(oc, n_hsv, cfg.coverage_thresh)
    nvp = oc.contents.len_valid_parents
    vp = np.array([oc.contents.valid_parents[i] for i in range(nvp)], dtype=np.int64)
    L.group_irregular_pixels(oc)
    kept = np.array([_walk_kept(oc.contents.groups[int(p)]) for p in vp], dtype=np.int64)
    cp = L.calculate_avg_hsv(oc, hsv)
    pal = np.array([[cp.contents.averages[i].h, cp.contents.averages[i].s, cp.contents.averages[i].v]
                    for i in range(cp.contents.N)]).reshape(-1, 3)
    pct = np.array([cp.contents.percentages[i] for i in range(cp.contents.N)])
    L.free_color_palette(cp)
    L.free_octree(oc)

    sharp = None
    if crops is not None:
        n = len(crops)
        arrs = [(C.c_int * n)(*[c[k] for c in crops]) for k in ("top", "bottom", "left", "right")]
        cb = Crop_Boundaries(n, *arrs)
        sp = L.get_variance_sharpness(pgm, C.byref(cb))
        sharp = np.array([sp.contents.sharpness[i] for i in range(n)])

    # get_blur_profile (src/blur_profile.c:250-293) with the DFT from numpy
    avg = (stats[0] + stats[1] + stats[2]) / 3.0                 # interface.c:78
    L.remove_dc_bias(pgm, avg)
    H, W = img.shape[0], img.shape[1]
    data = np.ctypeslib.as_array(pgm.contents.data, shape=(H * W,)).reshape(H, W)
    X = np.fft.rfft2(data)
    power = X.real * X.real + X.imag * X.imag
    norm, fmax = normalize_power(power)
    wf = W // 2 + 1
    fft_img = L.create_pgm_image(wf, H)
    np.ctypeslib.as_array(fft_img.contents.data, shape=(H * wf,))[:] = norm.ravel()
    conv = L.cartesian_to_polar_conversion(wf, H)
    bp = L.calculate_blur_profile(conv, fft_img, cfg.radius_partitions, cfg.angle_partitions)
    na, nr = cfg.angle_partitions, cfg.radius_partitions
    bins = np.array([[bp.contents.bins[a][r] for r in range(nr)] for a in range(na)])
    bv = L.vectorize_blur_profile(bp, cfg.fft_streak_thresh, cfg.magnitude_thresh,
                                  cfg.blur_cutoff_ratio_denom)
    angles = np.array([bv.contents.blur_vectors[i].angle for i in range(bv.contents.len_vectors)])
    mags = np.array([bv.contents.blur_vectors[i].magnitude for i in range(bv.contents.len_vectors)],
                    dtype=np.float32)
    abs_, rbs = bp.contents.angle_bin_size, bp.contents.radius_bin_size
    L.free_blur_vector_group(bv)
    L.free_blur_profile(bp)
    L.free_cartesian_to_polar(conv)
    L.free_image_pgm(fft_img)
    L.free_image_pgm(pgm)
    L.free_image_hsv(hsv)
    if cfg.downsample_rate > 1:
        L.free_image_rgb(ds)
    counts = blur_counts(H, wf, nr, na) if want_counts else np.zeros((na, nr), dtype=np.int64)
    return RefReport(stats=stats, average_saturation=s_bar, hist=hist, valid_parents=vp, kept=kept,
                     palette_hsv=pal, palette_pct=pct, bins=bins, bin_counts=counts,
                     blur_angles=angles, blur_mags=mags, fft_max=fmax,
                     angle_bin_size=abs_, radius_bin_size=rbs, sharpness=sharp)


def error_check(h: int, w: int) -> bool:
    """pre_compute_error_checks on an h x w image (channels non-NULL)."""
    L = lib()
    z = np.zeros(1)
    P = C.POINTER(C.c_double)
    im = Image_RGB(h, w, z.ctypes.data_as(P), z.ctypes.data_as(P), z.ctypes.data_as(P))
    return bool(L.pre_compute_error_checks(C.byref(im)))
