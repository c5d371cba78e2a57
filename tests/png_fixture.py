"""Minimal PNG encoder for mask fixtures (test data generator, not a reference restatement).

encode() writes the given samples in any colour type / bit depth / interlace the product decoder
must accept, and returns (png_bytes, rgb) where rgb is what libpng hands OpenCV's PngDecoder for
IMREAD_COLOR (imgcodecs/src/grfmt_png.cpp:240-286): 16-bit samples keep their high byte, gray 1/2/4-bit
samples are scaled to 8 bits, palettes are looked up, alpha is dropped."""
import struct
import zlib

import numpy as np

_ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
_CHANS = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}


def _chunk(tag, data):
    return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def _pack_rows(samples, depth):
    """samples: (h, w, c) ints -> list of packed row byte strings."""
    h, w, c = samples.shape
    rows = []
    for y in range(h):
        v = samples[y].reshape(-1)
        if depth == 16:
            rows.append(v.astype(">u2").tobytes())
        elif depth == 8:
            rows.append(v.astype(np.uint8).tobytes())
        else:
            per = 8 // depth
            out = bytearray((len(v) * depth + 7) // 8)
            for i, s in enumerate(v):
                out[i // per] |= int(s) << (8 - depth * (i % per + 1))
            rows.append(bytes(out))
    return rows


def _filter(rows, bpp, seed):
    """Apply a rotating mix of the five filter types so the decoder's unfilter is exercised."""
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for k, r in enumerate(rows):
        f = (k + seed) % 5
        enc = bytearray(len(r))
        for x in range(len(r)):
            a = r[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            if f == 0:
                p = 0
            elif f == 1:
                p = a
            elif f == 2:
                p = b
            elif f == 3:
                p = (a + b) >> 1
            else:
                pp = a + b - c
                pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
                p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
            enc[x] = (r[x] - p) & 0xFF
        out += bytes([f]) + enc
        prev = r
    return bytes(out)


def encode(samples, ctype, depth=8, palette=None, interlace=False, seed=0):
    samples = np.asarray(samples)
    if samples.ndim == 2:
        samples = samples[..., None]
    h, w, c = samples.shape
    assert c == _CHANS[ctype]
    bpp = max(1, c * depth // 8)
    if interlace:
        raw = b""
        for x0, y0, dx, dy in _ADAM7:
            sub = samples[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                raw += _filter(_pack_rows(sub, depth), bpp, seed)
    else:
        raw = _filter(_pack_rows(samples, depth), bpp, seed)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1 if interlace else 0)
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if ctype == 3:
        png += _chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    png += _chunk(b"IDAT", zlib.compress(raw, 6)) + _chunk(b"IEND", b"")
    s = samples.astype(np.int64)
    if depth == 16:
        s = s >> 8
    if ctype == 3:
        rgb = np.asarray(palette, np.uint8)[s[..., 0]]
    elif ctype in (0, 4):
        g = s[..., 0] * 255 // ((1 << depth) - 1) if depth < 8 else s[..., 0]
        rgb = np.repeat(g[..., None], 3, axis=2)
    else:
        rgb = s[..., :3]
    return png, np.ascontiguousarray(rgb.astype(np.uint8))
