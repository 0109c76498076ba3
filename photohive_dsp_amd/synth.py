"""Deterministic synthetic RGB8 images (H x W x 3, uint8, C-contiguous).

The reference ships no test images (``data/`` is git-ignored), so
golden fixtures store a generator spec ``(kind, H, W, seed)`` instead of
pixels.  Every generator is built on splitmix64 so the byte stream is fixed by
the algorithm, not by a numpy RNG version.  The same splitmix64 stream is
produced on the device by ``phd_fill_uniform_u8`` (bench inputs), see
``csrc/kernels/synth.hip``.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, offset: int = 0) -> np.ndarray:
    """Return n uint64 words: word i = mix(seed + (offset + i + 1) * golden)."""
    idx = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(h: int, w: int, seed: int) -> np.ndarray:
    """Uniform random bytes; byte j of the image is byte (j % 8) of word j // 8."""
    nbytes = h * w * 3
    words = splitmix64(seed, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].reshape(h, w, 3).copy()


def _unit(seed: int, n: int) -> np.ndarray:
    """n doubles in [0, 1) from the top 53 bits of splitmix64."""
    return (splitmix64(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def box_blur(img: np.ndarray, length: int, axis: int) -> np.ndarray:
    """Causal-free centred box blur of `length` taps along `axis` (edge-clamped), rounded to u8."""
    f = img.astype(np.float64)
    pad = [(0, 0)] * 3
    pad[axis] = (length // 2, length - 1 - length // 2)
    p = np.pad(f, pad, mode="edge")
    c = np.cumsum(p, axis=axis)
    zero_shape = list(c.shape)
    zero_shape[axis] = 1
    c = np.concatenate([np.zeros(zero_shape), c], axis=axis)
    n = img.shape[axis]
    hi = np.take(c, np.arange(length, length + n), axis=axis)
    lo = np.take(c, np.arange(0, n), axis=axis)
    return np.clip(np.rint((hi - lo) / length), 0, 255).astype(np.uint8)


def structured(h: int, w: int, seed: int, blur: int = 0, blur_axis: int = 1) -> np.ndarray:
    """Gradient background + coloured disks + mild noise; optional box (motion) blur."""
    u = _unit(seed, 64)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.empty((h, w, 3), dtype=np.float64)
    img[..., 0] = 255.0 * (0.2 + 0.6 * xx / max(w - 1, 1))
    img[..., 1] = 255.0 * (0.3 + 0.5 * yy / max(h - 1, 1))
    img[..., 2] = 255.0 * (0.5 + 0.4 * u[0])
    for d in range(8):
        cy, cx = u[1 + d] * h, u[9 + d] * w
        rad = (0.05 + 0.2 * u[17 + d]) * min(h, w)
        col = 255.0 * np.array([u[25 + d], u[33 + d], u[41 + d]])
        mask = (yy - cy) ** 2 + (xx - cx) ** 2 < rad * rad
        img[mask] = col
    noise = (_unit(seed + 1, h * w * 3).reshape(h, w, 3) - 0.5) * 24.0
    out = np.clip(np.rint(img + noise), 0, 255).astype(np.uint8)
    if blur > 1:
        out = box_blur(out, blur, axis=0 if blur_axis == 0 else 1)
    return out


def motion_noise(h: int, w: int, seed: int, length: int = 15, axis: int = 1) -> np.ndarray:
    """Uniform noise smeared by a `length`-tap box blur along `axis` (1 = horizontal)."""
    return box_blur(uniform(h, w, seed), length, axis)


def dominant(h: int, w: int, seed: int, frac: float = 0.55) -> np.ndarray:
    """A single sky-blue colour over `frac` of the rows, noise elsewhere.

    Large images of this kind drive the reference's float32 saliency
    comparator into its INT_MIN overflow path.
    """
    img = uniform(h, w, seed)
    rows = int(h * frac)
    img[:rows, :, :] = np.array([70, 130, 220], dtype=np.uint8)
    return img


def grayish(h: int, w: int, seed: int) -> np.ndarray:
    """Low-saturation image: most pixels fall in the gray / black groups."""
    base = uniform(h, w, seed).astype(np.int32)
    g = base[..., :1]
    out = g + (base - g) // 16
    return np.clip(out, 0, 255).astype(np.uint8)


def posterized(h: int, w: int, seed: int, levels: int = 6) -> np.ndarray:
    """Channels drawn from `levels` evenly spaced values (0, 51, ..., 255 for 6):
    most hues are exact ratios, many of them on hue-bin edges and centres."""
    step = 255 // (levels - 1)
    u = splitmix64(seed, h * w * 3) % np.uint64(levels)
    return (u.astype(np.int64) * step).astype(np.uint8).reshape(h, w, 3)


def black(h: int, w: int, seed: int = 0) -> np.ndarray:
    return np.zeros((h, w, 3), dtype=np.uint8)


KINDS = {
    "uniform": uniform,
    "structured": structured,
    "hblur": lambda h, w, s: structured(h, w, s, blur=15, blur_axis=1),
    "vblur": lambda h, w, s: structured(h, w, s, blur=15, blur_axis=0),
    "motion": motion_noise,
    "dominant": dominant,
    "grayish": grayish,
    "black": black,
    "posterized": posterized,
}


def make(kind: str, h: int, w: int, seed: int) -> np.ndarray:
    return KINDS[kind](h, w, seed)


def deep(kind: str, h: int, w: int, seed: int) -> np.ndarray:
    """A 16-bit image as the planar doubles a C caller of get_full_report_data
    may pass (value / 65535, src/interface.c:20-94): the 8-bit `kind` image
    scaled by 257 plus 8 bits of uniform noise.  float64 HxWx3 in [0, 1],
    almost no value equal to any k/255.0.

    Two suffixes give finite doubles outside [0, 1] that the reference still
    reports on (no octree index out of bounds): `kind+neg` -- a rectangle
    (rows H/4..H/2, columns W/3..2W/3) whose channels are -(2 x + 0.01), all
    negative (rgb2hsv's v < 0: the black group), so the luma reaches -2;
    `kind+spike` -- every 97th pixel of the odd columns (which downsample_rgb
    at rate 2 never samples) set to 40.0 in red, so only the statistics, the
    luma and the FFT see it."""
    base_kind, _, mod = kind.partition("+")
    base = make(base_kind, h, w, seed).astype(np.float64) * 257.0
    noise = uniform(h, w, seed + 7919).astype(np.float64)
    img = np.minimum(base + noise, 65535.0) / 65535.0
    if mod == "neg":
        sl = (slice(h // 4, h // 2), slice(w // 3, 2 * w // 3))
        img[sl] = -(2.0 * img[sl] + 0.01)
    elif mod == "spike":
        red = img[:, 1::2, 0].reshape(-1)
        red[::97] = 40.0
        img[:, 1::2, 0] = red.reshape(h, -1)
    elif mod:
        raise ValueError(f"unknown deep modifier {mod!r}")
    return img
