"""Generate the client's media assets procedurally (no binary is copied from anywhere): the page
background (PNG), the favicon (ICO with 16/32/48 px PNG images), the player icon and the
source-code link icon (SVG).  Reference media it stands in for: /root/reference/media
(background.jpeg, icon.ico, person-circle.png, github-mark/).

    python tools/make_media.py [out_dir]
"""
from __future__ import annotations

import os
import struct
import sys
import zlib

import numpy as np


def png_bytes(rgba: np.ndarray) -> bytes:
    h, w, _ = rgba.shape
    raw = b"".join(b"\x00" + rgba[y].astype(np.uint8).tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b""))


def background(w=960, h=540, seed=7) -> np.ndarray:
    """dusk gradient with soft low-frequency 'mantle' bands (upsampled value noise)"""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    t = y / h
    top, bottom = np.array([18, 20, 32], np.float32), np.array([46, 34, 58], np.float32)
    img = top[None, None] * (1 - t[..., None]) + bottom[None, None] * t[..., None]
    coarse = rng.standard_normal((7, 13)).astype(np.float32)
    gy = np.clip((y / h) * 6, 0, 5.999)
    gx = np.clip((x / w) * 12, 0, 11.999)
    y0, x0 = gy.astype(int), gx.astype(int)
    fy, fx = gy - y0, gx - x0
    fy, fx = fy * fy * (3 - 2 * fy), fx * fx * (3 - 2 * fx)
    n = (coarse[y0, x0] * (1 - fx) * (1 - fy) + coarse[y0, x0 + 1] * fx * (1 - fy)
         + coarse[y0 + 1, x0] * (1 - fx) * fy + coarse[y0 + 1, x0 + 1] * fx * fy)
    band = 0.5 + 0.5 * np.sin(6.0 * t + 1.7 * n)
    img = img + band[..., None] * np.array([10, 8, 16], np.float32)
    rgba = np.concatenate([np.clip(img, 0, 255), np.full((h, w, 1), 255, np.float32)], axis=-1)
    return rgba.astype(np.uint8)


def mantle_icon(size: int) -> np.ndarray:
    """a blurred 'painting' disc with a sharp letter-like stroke: the game in one glyph"""
    y, x = np.mgrid[0:size, 0:size].astype(np.float32) + 0.5
    c = size / 2
    r = np.hypot(x - c, y - c) / c
    disc = np.clip((1.0 - r) * size * 0.5, 0, 1)
    hue = np.stack([200 + 40 * (y / size), 120 + 60 * (x / size), 220 - 80 * (y / size)], -1)
    stroke = (np.abs((x - c) * 0.9 + (y - c) * 0.45) < size * 0.08) & (r < 0.75)
    rgb = np.where(stroke[..., None], 250.0, hue)
    return np.concatenate([rgb, (disc * 255)[..., None]], -1).astype(np.uint8)


def ico_bytes(sizes=(16, 32, 48)) -> bytes:
    images = [png_bytes(mantle_icon(s)) for s in sizes]
    out = struct.pack("<HHH", 0, 1, len(images))
    off = 6 + 16 * len(images)
    for s, data in zip(sizes, images):
        out += struct.pack("<BBBBHHII", s % 256, s % 256, 0, 0, 1, 32, len(data), off)
        off += len(data)
    return out + b"".join(images)


PERSON_SVG = """<svg xmlns="http://www.w3.org/2000/svg" viewBox="0 0 32 32" width="32" height="32">
  <circle cx="16" cy="16" r="15" fill="none" stroke="#c9c3d8" stroke-width="2"/>
  <circle cx="16" cy="12.5" r="5" fill="#c9c3d8"/>
  <path d="M6.5 26.5c1.8-4.6 5.3-7 9.5-7s7.7 2.4 9.5 7" fill="#c9c3d8"/>
</svg>
"""

CODE_SVG = """<svg xmlns="http://www.w3.org/2000/svg" viewBox="0 0 32 32" width="32" height="32">
  <rect x="1.5" y="4.5" width="29" height="23" rx="4" fill="none" stroke="#c9c3d8" stroke-width="2"/>
  <path d="M12 11l-5 5 5 5M20 11l5 5-5 5M17.5 9.5l-3 13" fill="none" stroke="#c9c3d8" stroke-width="2"
        stroke-linecap="round" stroke-linejoin="round"/>
</svg>
"""


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cassmantle_amd", "media")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "background.png"), "wb") as f:
        f.write(png_bytes(background()))
    with open(os.path.join(out, "icon.ico"), "wb") as f:
        f.write(ico_bytes())
    with open(os.path.join(out, "person-circle.svg"), "w") as f:
        f.write(PERSON_SVG)
    with open(os.path.join(out, "code-mark.svg"), "w") as f:
        f.write(CODE_SVG)
    print("wrote", sorted(os.listdir(out)))


if __name__ == "__main__":
    main()
