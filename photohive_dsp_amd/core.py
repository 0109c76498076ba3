"""Python API: get_report / Report / set_bounding_boxes (as /root/reference/core.py).

Same call signature, defaults, fields and error behaviour as the reference
(core.py:23-119, 388-515); the image goes to the MI355X library as raw RGB8
(phd_report_u8) instead of three planar double arrays.  New: get_reports()
for a list of images and report_device() for RGB8 batches already on the GPU.
GUI display methods (tkinter / matplotlib) are out of scope.
"""
from __future__ import annotations

import ctypes
import json
import os
import time
from ctypes import POINTER
from types import SimpleNamespace

import numpy as np

from .lib import last_error, lib
from .structures import Crop_Boundaries, Full_Report_Data, PhdConfig, Pixel_HSV, RGB_Statistics
from .utils import hsv_to_rgb, image_pgm_to_pillow, to_rgb8

DEFAULTS = dict(h_partitions=18, s_partitions=2, v_partitions=3, black_thresh=0.1, gray_thresh=0.1,
                coverage_thresh=0.95, linked_list_size=1000, downsample_rate=1, radius_partitions=40,
                angle_partitions=72, quantity_weight=0.1, saturation_value_weight=0.9,
                fft_streak_thresh=1.20, magnitude_thresh=0.3, blur_cutoff_ratio_denom=2)


def _stream_handle(stream):
    """The hipStream_t a device call runs on: the given torch stream, else
    torch's current stream (its handle 0, the null stream, makes the library
    order its own stream after the null stream's prior work)."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream or None


def make_config(**kw) -> PhdConfig:
    c = dict(DEFAULTS)
    unknown = set(kw) - set(c)
    if unknown:
        raise TypeError(f"unknown parameters {sorted(unknown)}")
    c.update(kw)
    return PhdConfig(**c)


class Report:
    """Report of one image; fields as the reference's Report (core.py:24-119)."""

    def __init__(self, report_ptr, height, width):
        report_data = report_ptr.contents          # NULL -> ValueError, as in the reference
        self.data_ptr = report_ptr
        self.rgb_stats = report_data.rgb_stats.contents
        self.rgb_stats.height = height
        self.rgb_stats.width = width
        self.color_palette = self._convert_color_palette(report_data.color_palette)
        self.blur_profile = self._convert_blur_profile(report_data.blur_profile)
        self.blur_vectors = self._convert_blur_vectors(report_data.blur_vectors)
        self.average_saturation = report_data.average_saturation
        self.sharpnesses = self._convert_sharpnesses(report_data.sharpness)

    @staticmethod
    def _convert_sharpnesses(ptr):
        if not ptr:
            return []
        s = ptr.contents
        return [s.sharpness[i] for i in range(s.N)]

    @staticmethod
    def _convert_blur_vectors(ptr):
        g = ptr.contents
        out = []
        for i in range(g.len_vectors):
            v = SimpleNamespace()
            v.angle = g.blur_vectors[i].angle
            v.magnitude = g.blur_vectors[i].magnitude
            out.append(v)
        return out

    @staticmethod
    def _convert_color_palette(ptr):
        cp = ptr.contents
        averages = ctypes.cast(cp.averages, POINTER(Pixel_HSV * cp.N)).contents if cp.N else []
        cp.colors = [hsv_to_rgb(p.h, p.s, p.v) for p in averages]
        cp.quantities = [cp.percentages[i] for i in range(cp.N)]
        cp.hsv = [(p.h, p.s, p.v) for p in averages]          # new: raw palette HSV
        cp.group_ids = [p.parent_id for p in averages]        # new: octree group of each colour
        return cp

    def _convert_blur_profile(self, ptr):
        c = ptr.contents
        self.bp_ptr = c
        bp = SimpleNamespace()
        bins = [list(ctypes.cast(c.bins[i], POINTER(ctypes.c_double * c.num_radius_bins)).contents)
                for i in range(c.num_angle_bins)]
        for a, row in enumerate(bins):            # core.py:109-117, same message
            for r, val in enumerate(row):
                if np.isnan(val):
                    print(f"NaN found at angle {a}, radius {r}. Correcting to 0.")
                    bins[a][r] = 0.0
        bp.bins = bins
        return bp

    def generate_blur_profile_image(self):
        """core.py:219-228 via get_blur_profile_visual (freed here, unlike the reference)."""
        h, w = self.rgb_stats.height, self.rgb_stats.width
        ptr = lib.get_blur_profile_visual(ctypes.byref(self.bp_ptr), h, w)
        img = image_pgm_to_pillow(ptr, w, h)
        lib.phd_free_pgm(ptr)
        self.blur_profile_image = img.crop((0, 0, w // 2, h))

    def generate_color_palette_image(self):
        """core.py:182-216 (falls back to PIL's default font when DejaVuSans is absent)."""
        from PIL import Image, ImageDraw, ImageFont
        n = len(self.color_palette.colors)
        block = 50
        per_row = int(np.ceil(np.sqrt(n))) if n else 1
        img = Image.new("RGB", (per_row * block, max(1, (n + per_row - 1) // per_row) * block), "black")
        draw = ImageDraw.Draw(img)
        try:
            font = ImageFont.truetype("DejaVuSans.ttf", 12)
        except OSError:
            font = ImageFont.load_default()
        for i, (color, q) in enumerate(zip(self.color_palette.colors, self.color_palette.quantities)):
            x1, y1 = (i % per_row) * block, (i // per_row) * block
            draw.rectangle([x1, y1, x1 + block, y1 + block], fill=tuple(int(c) for c in color))
            text = f"{q:.1%}"
            tw, th = draw.textbbox((0, 0), text, font=font)[2:]
            draw.text((x1 + (block - tw) / 2, y1 + (block - th) / 2), text, fill="black", font=font)
        self.color_palette_image = img

    def to_json(self):
        """core.py:388-436, same keys and padding."""
        d = {
            "Height": self.rgb_stats.height, "Width": self.rgb_stats.width,
            "Average Saturation": self.average_saturation,
            "Red Brightness": self.rgb_stats.Br, "Green Brightness": self.rgb_stats.Bg,
            "Blue Brightness": self.rgb_stats.Bb, "Red Contrast": self.rgb_stats.Cr,
            "Green Contrast": self.rgb_stats.Cg, "Blue Contrast": self.rgb_stats.Cb,
        }
        for i in range(10):
            d[f"Blur Vector {i+1} Angle"] = self.blur_vectors[i].angle
            d[f"Blur Vector {i+1} Magnitude"] = self.blur_vectors[i].magnitude
        for i in range(100):
            if i < len(self.color_palette.colors):
                h, s, v = self.color_palette.colors[i]
                pct = self.color_palette.quantities[i]
            else:
                h, s, v, pct = 0, 0, 0, 0
            d[f"Color {i+1} H"], d[f"Color {i+1} S"], d[f"Color {i+1} V"] = h, s, v
            d[f"Color {i+1} Percentage"] = pct
        for i in range(10):
            d[f"Sharpness {i+1}:"] = self.sharpnesses[i] if i < len(self.sharpnesses) else 0.0
        return json.dumps(d, indent=4)

    def __del__(self):
        ptr = getattr(self, "data_ptr", None)
        if ptr:
            lib.free_full_report(ctypes.byref(ptr))


def _finish(ptr, height, width, kw):
    report = Report(ptr, height, width)
    report.magnitude_threshold = kw.get("magnitude_thresh", DEFAULTS["magnitude_thresh"])
    report.fft_streak_threshold = kw.get("fft_streak_thresh", DEFAULTS["fft_streak_thresh"])
    report.blur_cutoff_ratio_denom = kw.get("blur_cutoff_ratio_denom", DEFAULTS["blur_cutoff_ratio_denom"])
    return report


def get_report(pil_image, salient_characters=None, h_partitions=18, s_partitions=2, v_partitions=3,
               black_thresh=0.1, gray_thresh=0.1, coverage_thresh=0.95, linked_list_size=1000,
               downsample_rate=1, radius_partitions=40, angle_partitions=72, quantity_weight=0.1,
               saturation_value_weight=0.9, fft_streak_thresh=1.20, magnitude_thresh=0.3,
               blur_cutoff_ratio_denom=2):
    """core.py:442-486.  `pil_image` may be a PIL image or an H x W x 3 uint8 array.
    An image the reference rejects (src/utilities.c:64-87) raises ValueError
    ("NULL pointer access"), exactly like the reference binding does."""
    kw = dict(h_partitions=h_partitions, s_partitions=s_partitions, v_partitions=v_partitions,
              black_thresh=black_thresh, gray_thresh=gray_thresh, coverage_thresh=coverage_thresh,
              linked_list_size=linked_list_size, downsample_rate=downsample_rate,
              radius_partitions=radius_partitions, angle_partitions=angle_partitions,
              quantity_weight=quantity_weight, saturation_value_weight=saturation_value_weight,
              fft_streak_thresh=fft_streak_thresh, magnitude_thresh=magnitude_thresh,
              blur_cutoff_ratio_denom=blur_cutoff_ratio_denom)
    rgb = to_rgb8(pil_image)
    height, width = rgb.shape[:2]
    cfg = make_config(**kw)
    crops = ctypes.byref(salient_characters) if isinstance(salient_characters, Crop_Boundaries) \
        else salient_characters
    start = time.time()
    ptr = lib.phd_report_u8(rgb.ctypes.data, height, width, 0, ctypes.byref(cfg), crops)
    if os.environ.get("PHD_VERBOSE"):
        print(f"Elapsed time: {time.time() - start} seconds")
    return _finish(ptr, height, width, kw)


def get_reports(images, **kw):
    """Reports for a list of images (any sizes).  Failed images give None."""
    cfg = make_config(**kw)
    arrs = [to_rgb8(im) for im in images]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
    hs = (ctypes.c_int * n)(*[a.shape[0] for a in arrs])
    ws = (ctypes.c_int * n)(*[a.shape[1] for a in arrs])
    outs = (POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()
    lib.phd_report_batch_u8(ptrs, hs, ws, n, ctypes.byref(cfg), outs, st)
    return [(_finish(outs[i], hs[i], ws[i], kw) if st[i] == 0 else None) for i in range(n)]


def report_device(images, stream=None, **kw):
    """Reports for a uint8 torch tensor [N, H, W, 3] resident on the current GPU."""
    if images.dtype.itemsize != 1 or images.dim() != 4 or images.shape[3] != 3 or not images.is_contiguous():
        raise ValueError("expected a contiguous uint8 [N, H, W, 3] device tensor")
    n, h, w = int(images.shape[0]), int(images.shape[1]), int(images.shape[2])
    cfg = make_config(**kw)
    outs = (POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()
    s = _stream_handle(stream)
    lib.phd_report_batch_device(images.data_ptr(), n, h, w, 0, ctypes.byref(cfg), outs, st, s)
    res = [(_finish(outs[i], h, w, kw) if st[i] == 0 else None) for i in range(n)]
    if any(r is None for r in res):
        raise RuntimeError(f"report_device failed: {last_error()}")
    return res


def reports_device_mixed(images, stream=None, **kw):
    """Reports for a list of uint8 torch tensors [H, W, 3] of any sizes resident
    on the current GPU (BASELINE config 5): one batched run per group of
    same-size images (phd_report_batch_device_mixed)."""
    for im in images:
        if im.dtype.itemsize != 1 or im.dim() != 3 or im.shape[2] != 3 or not im.is_contiguous():
            raise ValueError("expected contiguous uint8 [H, W, 3] device tensors")
    n = len(images)
    cfg = make_config(**kw)
    ptrs = (ctypes.c_void_p * n)(*[im.data_ptr() for im in images])
    hs = (ctypes.c_int * n)(*[int(im.shape[0]) for im in images])
    ws = (ctypes.c_int * n)(*[int(im.shape[1]) for im in images])
    outs = (POINTER(Full_Report_Data) * n)()
    st = (ctypes.c_int * n)()
    s = _stream_handle(stream)
    lib.phd_report_batch_device_mixed(ptrs, hs, ws, n, ctypes.byref(cfg), outs, st, s)
    res = [(_finish(outs[i], hs[i], ws[i], kw) if st[i] == 0 else None) for i in range(n)]
    if any(r is None for r in res):
        raise RuntimeError(f"reports_device_mixed failed: {last_error()}")
    return res


def hsv_stats_device(images, stream=None):
    """rgb2hsv + get_hsv_average + get_rgb_statistics (src/image_processing.c:372-417, 533-553)
    for a uint8 torch tensor [N, H, W, 3] on the current GPU: returns
    ([RGB_Statistics] * N, [average saturation] * N)."""
    if images.dtype.itemsize != 1 or images.dim() != 4 or images.shape[3] != 3 or not images.is_contiguous():
        raise ValueError("expected a contiguous uint8 [N, H, W, 3] device tensor")
    n, h, w = int(images.shape[0]), int(images.shape[1]), int(images.shape[2])
    stats = (RGB_Statistics * n)()
    sat = (ctypes.c_double * n)()
    s = _stream_handle(stream)
    if lib.phd_hsv_stats_batch_device(images.data_ptr(), n, h, w, 0, stats, sat, s) != 0:
        raise RuntimeError(f"hsv_stats_device failed: {last_error()}")
    return list(stats), list(sat)


def blur_profiles_device(images, stream=None, **kw):
    """The FFT + blur-profile path alone (BASELINE config 4; rgb2pgm, pgm_fft,
    calculate_blur_profile, vectorize_blur_profile) for a uint8 torch tensor
    [N, H, W, 3] on the current GPU: returns (bins [N, angle, radius] float64,
    [[(angle, magnitude)] * 10] * N) -- the full report's values."""
    from .structures import Blur_Vector
    if images.dtype.itemsize != 1 or images.dim() != 4 or images.shape[3] != 3 or not images.is_contiguous():
        raise ValueError("expected a contiguous uint8 [N, H, W, 3] device tensor")
    n, h, w = int(images.shape[0]), int(images.shape[1]), int(images.shape[2])
    cfg = make_config(**kw)
    na, nr = cfg.angle_partitions, cfg.radius_partitions
    bins = np.zeros((n, na, nr), dtype=np.float64)
    vecs = (Blur_Vector * (10 * n))()
    s = _stream_handle(stream)
    if lib.phd_blur_batch_device(images.data_ptr(), n, h, w, 0, ctypes.byref(cfg),
                                 bins.ctypes.data_as(POINTER(ctypes.c_double)), vecs, s) != 0:
        raise RuntimeError(f"blur_profiles_device failed: {last_error()}")
    return bins, [[(vecs[10 * i + k].angle, vecs[10 * i + k].magnitude) for k in range(10)] for i in range(n)]


def set_bounding_boxes(bounding_boxes):
    """core.py:489-515."""
    n = len(bounding_boxes)
    arrs = {k: (ctypes.c_int * n)(*[b[k] for b in bounding_boxes]) for k in ("top", "bottom", "left", "right")}
    return Crop_Boundaries(N=n, **arrs)
