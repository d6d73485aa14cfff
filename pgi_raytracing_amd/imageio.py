"""Frame sink writers: the reference shows frames in a D3D11 window (simpleguidx11.cpp:130-202);
headless runs write them instead.  Frames are the framebuffer layout of pgrt_render (row-major,
top-down, RGBA float32)."""
from __future__ import annotations

import numpy as np


def save_pfm(path: str, rgba: np.ndarray) -> None:
    """Portable float map (RGB, little endian).  PFM rows run bottom-up, so the top-down frame
    is flipped on write; values are stored unclamped (NaNs of gamma(c<0) included)."""
    rgb = np.ascontiguousarray(rgba[::-1, :, :3], dtype="<f4")
    h, w = rgb.shape[:2]
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode("ascii"))
        f.write(rgb.tobytes())


def load_pfm(path: str) -> np.ndarray:
    """Inverse of save_pfm: (H, W, 3) float32, top-down."""
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = (int(x) for x in f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4").reshape(h, w, 3)
    return np.ascontiguousarray(data[::-1]).astype(np.float32)


def to_rgb8(rgba: np.ndarray) -> np.ndarray:
    """Display encoding of the window: clamp to [0, 1] (NaN -> 0) and scale to bytes."""
    c = np.nan_to_num(rgba[..., :3].astype(np.float32), nan=0.0, posinf=1.0, neginf=0.0)
    return (np.clip(c, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)


def save_png(path: str, rgba: np.ndarray) -> None:
    from PIL import Image  # present in the image; only the writer needs it

    Image.fromarray(to_rgb8(rgba), "RGB").save(path)
