#!/usr/bin/env python3
"""Synthetic environment maps and a minimal OpenEXR writer (test / bench inputs).

The reference's env maps (exr/*.exr) are Git-LFS pointers in the mounted reference, so the
environment-light paths are exercised on deterministic synthetic skies of the same layout:
HDRImageBuffer data[w*j + i], row j = 0 at theta = 0 (+y, straight up), phi = 2 pi (i + .5) / w
(environment_light.cpp:81-104). write_exr emits single-part scanline files with NONE / RLE /
ZIPS / ZIP compression and HALF / FLOAT channels B, G, R (alphabetical, as OpenEXR stores them).

usage: envmap.py OUT.exr W H [zip|zips|none|rle] [half|float]
"""
import struct
import sys
import zlib

import numpy as np


def synth_envmap(w: int, h: int, sun=(0.55, 0.35), seed: int = 7) -> np.ndarray:
    """(h, w, 3) float32 radiance: a sky gradient above the horizon, a dim ground, a bright sun
    lobe at (theta, phi) = sun * (pi, 2 pi) and mild deterministic texture."""
    j = (np.arange(h) + 0.5) / h * np.pi            # theta per row
    i = (np.arange(w) + 0.5) / w * 2 * np.pi        # phi per column
    th, ph = np.meshgrid(j, i, indexing="ij")
    up = np.cos(th)
    sky = np.stack([0.35 + 0.25 * up, 0.5 + 0.3 * up, 0.8 + 0.4 * up], -1) * (up > 0)[..., None]
    ground = np.stack([0.12, 0.10, 0.08], -1) * np.ones_like(th)[..., None] * (up <= 0)[..., None]
    st, sp = sun[0] * np.pi, sun[1] * 2 * np.pi
    d = np.stack([np.sin(th) * np.cos(ph), np.cos(th), np.sin(th) * np.sin(ph)], -1)
    s = np.array([np.sin(st) * np.cos(sp), np.cos(st), np.sin(st) * np.sin(sp)])
    lobe = np.exp((d @ s - 1.0) * 60.0)[..., None] * np.array([40.0, 36.0, 30.0])
    rng = np.random.default_rng(seed)
    tex = 1.0 + 0.15 * rng.random((h, w, 1))
    return ((sky + ground) * tex + lobe).astype(np.float32)


def _half_bytes(a):
    return a.astype("<f2").tobytes()


def _predict_interleave(raw: bytes) -> bytes:
    """OpenEXR zip/rle pre-pass: split even / odd bytes, then delta-encode (ImfZip.cpp)."""
    b = np.frombuffer(raw, dtype=np.uint8)
    t = np.concatenate([b[0::2], b[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128 + 256) & 0xFF
    return d.astype(np.uint8).tobytes()


def _rle(data: bytes) -> bytes:
    out = bytearray()
    n = len(data)
    i = 0
    while i < n:
        j = i
        while j + 1 < n and data[j + 1] == data[i] and j - i < 127:
            j += 1
        run = j - i + 1
        if run >= 3:
            out += struct.pack("b", run - 1) + bytes([data[i]])
            i = j + 1
            continue
        k = i
        while k < n and k - i < 127:
            if k + 2 < n and data[k] == data[k + 1] == data[k + 2]:
                break
            k += 1
        out += struct.pack("b", -(k - i)) + data[i:k]
        i = k
    return bytes(out)


def write_exr(path: str, rgb: np.ndarray, compression: str = "zip", pixel: str = "half") -> None:
    rgb = np.asarray(rgb, dtype=np.float32)
    h, w, _ = rgb.shape
    comp = {"none": 0, "rle": 1, "zips": 2, "zip": 3}[compression]
    ptype = {"half": 1, "float": 2}[pixel]
    lines = 16 if comp == 3 else 1

    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data

    ch = b""
    for name in ("B", "G", "R"):
        ch += name.encode() + b"\0" + struct.pack("<iB3xii", ptype, 0, 1, 1)
    ch += b"\0"
    hdr = b"".join([
        attr("channels", "chlist", ch),
        attr("compression", "compression", bytes([comp])),
        attr("dataWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)),
        attr("displayWindow", "box2i", struct.pack("<4i", 0, 0, w - 1, h - 1)),
        attr("lineOrder", "lineOrder", bytes([0])),
        attr("pixelAspectRatio", "float", struct.pack("<f", 1.0)),
        attr("screenWindowCenter", "v2f", struct.pack("<2f", 0.0, 0.0)),
        attr("screenWindowWidth", "float", struct.pack("<f", 1.0)),
    ]) + b"\0"
    head = struct.pack("<ii", 20000630, 2) + hdr
    nchunks = (h + lines - 1) // lines
    chunks = []
    for c in range(nchunks):
        y0, y1 = c * lines, min(h, (c + 1) * lines)
        raw = b""
        for y in range(y0, y1):
            for k in (2, 1, 0):   # B, G, R
                row = rgb[y, :, k]
                raw += _half_bytes(row) if ptype == 1 else row.astype("<f4").tobytes()
        if comp in (2, 3):
            data = zlib.compress(_predict_interleave(raw), 9)
        elif comp == 1:
            data = _rle(_predict_interleave(raw))
            if len(data) >= len(raw):
                data = raw
        else:
            data = raw
        chunks.append(struct.pack("<ii", y0, len(data)) + data)
    off = len(head) + 8 * nchunks
    table = b""
    for cdat in chunks:
        table += struct.pack("<Q", off)
        off += len(cdat)
    with open(path, "wb") as f:
        f.write(head + table + b"".join(chunks))


def main():
    out, w, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    comp = sys.argv[4] if len(sys.argv) > 4 else "zip"
    pix = sys.argv[5] if len(sys.argv) > 5 else "half"
    write_exr(out, synth_envmap(w, h), comp, pix)


if __name__ == "__main__":
    main()
