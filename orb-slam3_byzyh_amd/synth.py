"""Deterministic synthetic inputs for the ORB front-end (no image data ships with the reference).

SURVEY.md sec. 8(d): EuRoC-shaped gray frames made of random filled rectangles and triangles with
additive noise (FAST corners at polygon vertices at roughly EuRoC density), a "blurred noise"
texture that stresses NMS and the quad-tree, and a stereo right view made by shifting the left
view by a piecewise-constant disparity field.
"""
from __future__ import annotations

import numpy as np


def polygon_frame(width: int = 640, height: int = 480, seed: int = 1, n_shapes: int = 400,
                  noise_sigma: float = 3.0) -> np.ndarray:
    """`n_shapes` random rectangles/triangles of uniform random intensity, then N(0, sigma) noise."""
    rng = np.random.default_rng(seed)
    img = np.full((height, width), rng.integers(0, 256), dtype=np.float32)
    yy, xx = np.mgrid[0:height, 0:width]
    for _ in range(n_shapes):
        val = float(rng.integers(0, 256))
        cx, cy = rng.integers(0, width), rng.integers(0, height)
        sx, sy = rng.integers(4, max(5, width // 6)), rng.integers(4, max(5, height // 6))
        x0, x1 = max(0, cx - sx // 2), min(width, cx + sx // 2 + 1)
        y0, y1 = max(0, cy - sy // 2), min(height, cy + sy // 2 + 1)
        if rng.integers(0, 2) == 0:
            img[y0:y1, x0:x1] = val
        else:
            p = rng.integers([x0, y0], [x1 + 1, y1 + 1], size=(3, 2)).astype(np.float32)
            X, Y = xx[y0:y1, x0:x1].astype(np.float32), yy[y0:y1, x0:x1].astype(np.float32)

            def edge(a, b):
                return (b[0] - a[0]) * (Y - a[1]) - (b[1] - a[1]) * (X - a[0])

            e0, e1, e2 = edge(p[0], p[1]), edge(p[1], p[2]), edge(p[2], p[0])
            inside = ((e0 >= 0) & (e1 >= 0) & (e2 >= 0)) | ((e0 <= 0) & (e1 <= 0) & (e2 <= 0))
            img[y0:y1, x0:x1][inside] = val
    img += rng.normal(0.0, noise_sigma, size=img.shape).astype(np.float32)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def blurred_noise_frame(width: int = 640, height: int = 480, seed: int = 2, sigma: float = 1.5) -> np.ndarray:
    """White noise smoothed by a separable Gaussian (sigma px), rescaled to 0..255."""
    rng = np.random.default_rng(seed)
    img = rng.random((height, width), dtype=np.float32)
    r = int(np.ceil(3 * sigma))
    k = np.exp(-0.5 * (np.arange(-r, r + 1) / sigma) ** 2).astype(np.float32)
    k /= k.sum()
    img = np.apply_along_axis(lambda v: np.convolve(np.pad(v, r, mode="reflect"), k, "valid"), 1, img)
    img = np.apply_along_axis(lambda v: np.convolve(np.pad(v, r, mode="reflect"), k, "valid"), 0, img)
    img = (img - img.min()) / max(1e-6, float(img.max() - img.min()))
    return np.clip(np.rint(img * 255), 0, 255).astype(np.uint8)


def stereo_pair(width: int = 752, height: int = 480, seed: int = 200, dmin: int = 4, dmax: int = 48):
    """Left = polygon frame; right = left shifted left by a per-(16-row band, 64-col block) disparity."""
    left = polygon_frame(width, height, seed=seed)
    rng = np.random.default_rng(seed + 1)
    disp = rng.integers(dmin, dmax + 1, size=((height + 15) // 16, (width + 63) // 64))
    right = np.empty_like(left)
    for y in range(height):
        for bx in range(disp.shape[1]):
            d = int(disp[y // 16, bx])
            x0, x1 = bx * 64, min(width, bx * 64 + 64)
            src = np.clip(np.arange(x0, x1) + d, 0, width - 1)
            right[y, x0:x1] = left[y, src]
    noise = rng.normal(0.0, 2.0, size=right.shape)
    right = np.clip(np.rint(right.astype(np.float32) + noise), 0, 255).astype(np.uint8)
    return left, right, disp


def frame_batch(n: int, width: int = 640, height: int = 480, seed0: int = 100) -> np.ndarray:
    return np.stack([polygon_frame(width, height, seed=seed0 + i) for i in range(n)])
