"""Test infrastructure: a small PNG writer with full control over what goes into the file --
bit depth 1/2/4/8/16, every colour type, per-row filters, Adam7 interlace and the colour chunks
(gAMA, sRGB, iCCP, cHRM, tRNS, PLTE) -- so the colour-capture conversions can be checked against
the system libpng on exactly the files a browser or a camera app writes (RGBA canvas PNGs,
16-bit RGB, gamma / ICC tagged files).  PNG 1.2 / ISO 15948 layout."""
from __future__ import annotations

import struct
import zlib

import numpy as np

CHANNELS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}
ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def chunk(kind: bytes, data: bytes) -> bytes:
    return struct.pack(">I", len(data)) + kind + data + struct.pack(">I", zlib.crc32(kind + data) & 0xffffffff)


def _pack_rows(img: np.ndarray, depth: int, ctype: int) -> list[bytes]:
    """Rows of samples [h, w, c] (ints) -> packed scanline bytes (no filter byte)."""
    h, w = img.shape[:2]
    c = CHANNELS[ctype]
    a = img.reshape(h, w * c)
    rows = []
    for y in range(h):
        r = a[y]
        if depth == 16:
            rows.append(r.astype(">u2").tobytes())
        elif depth == 8:
            rows.append(r.astype(np.uint8).tobytes())
        else:
            per = 8 // depth
            n = (len(r) + per - 1) // per
            out = bytearray(n)
            for i, v in enumerate(r):
                out[i // per] |= (int(v) & ((1 << depth) - 1)) << (8 - depth * (i % per + 1))
            rows.append(bytes(out))
    return rows


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def _filter(rows: list[bytes], bpp: int, filters) -> bytes:
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for y, r in enumerate(rows):
        ft = filters[y % len(filters)]
        f = bytearray(len(r))
        for x in range(len(r)):
            a = r[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            pred = (0, a, b, (a + b) >> 1, _paeth(a, b, c))[ft]
            f[x] = (r[x] - pred) & 0xff
        out.append(ft)
        out += f
        prev = r
    return bytes(out)


def encode(img: np.ndarray, depth: int = 8, ctype: int | None = None, filters=(0, 1, 2, 3, 4), interlace: bool = False,
           chunks=(), level: int = 6, palette=None) -> bytes:
    """PNG bytes of ``img`` ([h, w] or [h, w, c] sample values, already at ``depth``).
    ``chunks``: (type, data) pairs written after IHDR (before PLTE / IDAT), e.g. (b"gAMA", ...)."""
    img = np.asarray(img)
    if img.ndim == 2:
        img = img[..., None]
    h, w, c = img.shape
    if ctype is None:
        ctype = {1: 0, 2: 4, 3: 2, 4: 6}[c]
    assert CHANNELS[ctype] == c
    bpp = max(1, c * depth // 8)
    raw = b""
    if interlace:
        for x0, y0, dx, dy in ADAM7:
            sub = img[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                raw += _filter(_pack_rows(sub, depth, ctype), bpp, filters)
    else:
        raw = _filter(_pack_rows(img, depth, ctype), bpp, filters)
    out = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    for kind, data in chunks:
        out += chunk(kind, data)
    if palette is not None:
        out += chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    out += chunk(b"IDAT", zlib.compress(raw, level)) + chunk(b"IEND", b"")
    return out


def gama(g: float) -> tuple[bytes, bytes]:
    return b"gAMA", struct.pack(">I", int(round(g * 100000)))


def srgb(intent: int = 0) -> tuple[bytes, bytes]:
    return b"sRGB", bytes([intent])


def chrm_srgb() -> tuple[bytes, bytes]:
    v = [31270, 32900, 64000, 33000, 30000, 60000, 15000, 6000]
    return b"cHRM", struct.pack(">8I", *v)


def iccp(profile: bytes, name: bytes = b"ICC profile") -> tuple[bytes, bytes]:
    return b"iCCP", name + b"\0\0" + zlib.compress(profile)


def minimal_rgb_profile() -> bytes:
    """A structurally valid ICC v2 RGB display profile (header + rXYZ/gXYZ/bXYZ/wtpt + one
    gamma-2.2 TRC shared by r/g/b): passes libpng's header and tag-table checks and is not one of
    the sRGB profiles libpng recognises, so it leaves the file's gamma unset."""
    def s15(x):
        return struct.pack(">i", int(round(x * 65536)))

    def xyz(x, y, z):
        return b"XYZ \0\0\0\0" + s15(x) + s15(y) + s15(z)
    curv = b"curv\0\0\0\0" + struct.pack(">I", 1) + struct.pack(">H", int(2.2 * 256)) + b"\0\0"
    tags = [(b"rXYZ", xyz(0.4361, 0.2225, 0.0139)), (b"gXYZ", xyz(0.3851, 0.7169, 0.0971)),
            (b"bXYZ", xyz(0.1431, 0.0606, 0.7141)), (b"wtpt", xyz(0.9642, 1.0, 0.8249)),
            (b"rTRC", curv), (b"gTRC", curv), (b"bTRC", curv)]
    n = len(tags)
    off = 128 + 4 + 12 * n
    table, data = b"", b""
    shared = None
    for sig, d in tags:
        if sig in (b"gTRC", b"bTRC"):
            table += sig + struct.pack(">II", shared[0], shared[1])
            continue
        o = off + len(data)
        table += sig + struct.pack(">II", o, len(d))
        if sig == b"rTRC":
            shared = (o, len(d))
        data += d
        while len(data) % 4:
            data += b"\0"
    size = off + len(data)
    hdr = struct.pack(">I", size) + b"none" + bytes([2, 0x10, 0, 0]) + b"mntrRGB XYZ " + bytes(12) + b"acsp" \
        + b"APPL" + bytes(4) + b"none" + b"none" + bytes(8) + struct.pack(">I", 0) \
        + s15(0.9642) + s15(1.0) + s15(0.8249) + b"none" + bytes(16) + bytes(28)
    assert len(hdr) == 128, len(hdr)
    return hdr + struct.pack(">I", n) + table + data
