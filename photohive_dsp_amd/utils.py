"""Image conversion helpers (API of /root/reference/utils.py:1-86).

The hot-path caller no longer needs pil_image_to_image_rgb (357 ms at 12 MP):
get_report() hands the RGB8 buffer to phd_report_u8 directly.  It is kept for
callers of the legacy get_full_report_data entry point."""
import ctypes

import numpy as np

from .structures import Image_RGB


def hsv_to_rgb(h, s, v):
    """utils.py:7-27 -- palette HSV to integer RGB."""
    c = v * s
    x = c * (1 - abs((h / 60) % 2 - 1))
    m = v - c
    if h < 60:
        r, g, b = c, x, 0
    elif h < 120:
        r, g, b = x, c, 0
    elif h < 180:
        r, g, b = 0, c, x
    elif h < 240:
        r, g, b = 0, x, c
    elif h < 300:
        r, g, b = x, 0, c
    else:
        r, g, b = c, 0, x
    r, g, b = (r + m) * 255, (g + m) * 255, (b + m) * 255
    return int(r), int(g), int(b)


def to_rgb8(image) -> np.ndarray:
    """PIL image / array-like -> C-contiguous uint8 H x W x 3."""
    if hasattr(image, "mode") and getattr(image, "mode", "RGB") != "RGB":
        image = image.convert("RGB")
    arr = np.asarray(image)
    if arr.dtype != np.uint8 or arr.ndim != 3 or arr.shape[2] != 3:
        raise ValueError("expected an RGB8 image (H x W x 3 uint8)")
    return np.ascontiguousarray(arr)


def pil_image_to_image_rgb(pil_image):
    """utils.py:30-46 -- planar doubles k/255.0 for the legacy entry point."""
    width, height = pil_image.size
    img_array = np.array(pil_image) / 255.0
    planes = [np.ascontiguousarray(img_array[:, :, c]).ravel().astype(np.double) for c in range(3)]
    ptrs = [p.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) for p in planes]
    pil_image.r_ctypes, pil_image.g_ctypes, pil_image.b_ctypes = ptrs
    pil_image._phd_planes = planes          # keep the buffers alive with the image
    return Image_RGB(height=height, width=width, r=ptrs[0], g=ptrs[1], b=ptrs[2])


def image_rgb_to_pillow(image_rgb_ptr, width, height):
    from PIL import Image
    image_rgb = image_rgb_ptr.contents
    arr = ctypes.c_double * (width * height)
    chans = [np.ctypeslib.as_array(ctypes.cast(getattr(image_rgb, c), ctypes.POINTER(arr)).contents)
             .reshape(height, width) for c in ("r", "g", "b")]
    img_np = np.clip(np.stack(chans, axis=-1) * 255, 0, 255).astype(np.uint8)
    return Image.fromarray(img_np, "RGB")


def image_pgm_to_pillow(image_pgm_ptr, width, height):
    from PIL import Image
    pgm = image_pgm_ptr.contents
    arr = ctypes.c_double * (width * height)
    data = np.ctypeslib.as_array(ctypes.cast(pgm.data, ctypes.POINTER(arr)).contents).reshape(height, width)
    return Image.fromarray(np.clip(data * 255, 0, 255).astype(np.uint8), "L")
