"""Output encoding (main.rs:52-63): to_rgb8_gamma2 (color.rs:43-48) + image save by extension."""
from __future__ import annotations

import numpy as np


def to_rgb8_gamma2(pixels: np.ndarray) -> np.ndarray:
    """clamp(0, 255, sqrt(c) * 256) as u8, NaN -> 0 (Rust saturating cast)."""
    p = np.asarray(pixels, np.float32)
    with np.errstate(invalid="ignore"):
        v = np.sqrt(p) * np.float32(256.0)
        v = np.where(v > 255.0, np.float32(255.0), np.where(v < 0.0, np.float32(0.0), v))
        v = np.where(np.isnan(v), np.float32(0.0), v)
    return v.astype(np.uint8)


def save_image(path: str, pixels: np.ndarray, width: int, height: int) -> None:
    """image::save_buffer(path, bytes, W, H, Rgb8): .ppm -> binary P6, otherwise via Pillow."""
    rgb = to_rgb8_gamma2(pixels).reshape(height, width, 3)
    if path.lower().endswith(".ppm"):
        with open(path, "wb") as f:
            f.write(b"P6\n%d %d\n255\n" % (width, height))
            f.write(rgb.tobytes())
        return
    from PIL import Image

    Image.fromarray(rgb, "RGB").save(path)
