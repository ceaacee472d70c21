"""Test-side OpenEXR ENCODER (numpy + zlib), written from the published OpenEXR 2 file
format, used to check the product decoder (raytracer-795_amd/host/exr_read.cpp) on every
codec the reference's LoadEXR reads for a texture (src/Helper.cpp:346-359): NONE, RLE,
ZIPS, ZIP and PIZ, HALF / FLOAT / UINT channels, scanline and one-level tiled layouts.

It is written in the encode direction, in numpy: the PIZ wavelet is the forward lifting
equations applied level by level to index arrays of disjoint lattice cells
(`_wavelet_forward_2d`), the Huffman stage builds code lengths with a heap and assigns
OpenEXR's canonical codes (longest codes smallest).  The decoder (C++, decode direction) reads
lengths into a count-per-length table and decodes by code ranges, and inverts the wavelet
cell by cell.  History: until round 4 this file's wavelet encoder was a transliteration of the
vendored tinyexr's `wav2Encode` (src/tinyexr.h:8065-8160), so the round trip was not
independent of tinyexr's reading of the format; it was rewritten from the equations (DESIGN.md
§10).  It is not the reference's codec (compiling the reference's vendored tinyexr as a
checker was refused here)."""
from __future__ import annotations

import heapq
import struct
import zlib

import numpy as np

NONE, RLE, ZIPS, ZIP, PIZ = 0, 1, 2, 3, 4
UINT, HALF, FLOAT = 0, 1, 2
_LINES = {NONE: 1, RLE: 1, ZIPS: 1, ZIP: 16, PIZ: 32}


def _attr(name, typ, data: bytes) -> bytes:
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def _values(plane: np.ndarray, ptype: int) -> bytes:
    if ptype == HALF:
        return plane.astype(np.float16).astype("<f2").tobytes()
    if ptype == FLOAT:
        return plane.astype("<f4").tobytes()
    return plane.astype("<u4").tobytes()


# ---------------------------------------------------------------- RLE / ZIP
def _predict_split(raw: bytes) -> bytes:
    b = np.frombuffer(raw, np.uint8)
    t = np.concatenate([b[0::2], b[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128) & 0xFF
    return d.astype(np.uint8).tobytes()


def _rle(b: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(b)
    while i < n:
        j = i
        while j + 1 < n and b[j + 1] == b[i] and j - i < 127:
            j += 1
        run = j - i + 1
        if run >= 3:
            out += struct.pack("b", run - 1) + b[i:i + 1]
            i = j + 1
            continue
        k = i
        while k < n and k - i < 127:      # literal stretch until a run of 3 starts
            if k + 2 < n and b[k] == b[k + 1] == b[k + 2]:
                break
            k += 1
        out += struct.pack("b", -(k - i)) + b[i:k]
        i = k
    return bytes(out)


# ---------------------------------------------------------------- PIZ
def _lift_narrow(a: np.ndarray, b: np.ndarray):
    """Forward lifting step for values below 2^14 (format description, "PIZ"): on the signed
    16-bit readings, low = floor((a + b) / 2), high = a - b, both stored mod 2^16."""
    sa = a - ((a >= 0x8000) << 16)
    sb = b - ((b >= 0x8000) << 16)
    return ((sa + sb) >> 1) & 0xFFFF, (sa - sb) & 0xFFFF


def _lift_wide(a: np.ndarray, b: np.ndarray):
    """Forward lifting step for the full 16-bit range (modular form): with a' = a + 2^15 mod 2^16,
    high = a' - b mod 2^16 and low = floor((a' + b) / 2), plus 2^15 when a' < b, mod 2^16."""
    ash = (a + 0x8000) & 0xFFFF
    low = (ash + b) >> 1
    low = np.where(ash < b, low + 0x8000, low) & 0xFFFF
    return low, (ash - b) & 0xFFFF


def _wavelet_forward_2d(plane: np.ndarray, maxval: int) -> None:
    """In-place multi-level 2-D transform of one (ny, nx) plane of 16-bit values (as int64).

    Level k uses pair distance p = 2^k on the lattice of step q = 2p, for as long as q fits in
    min(nx, ny).  Every q-aligned cell {(y, x), (y, x+p), (y+p, x), (y+p, x+p)} lying wholly inside
    the plane is lifted along x (both rows), then the two low and the two high results along y;
    where the plane leaves a strip of width p past the last full cell (nx & p, ny & p), its
    cells are lifted along the one axis that still has a partner.  The cells of one level are
    disjoint, so each level is a handful of gathers and scatters over index arrays."""
    lift = _lift_narrow if maxval < (1 << 14) else _lift_wide
    ny, nx = plane.shape
    p = 1
    while 2 * p <= min(nx, ny):
        q = 2 * p
        xs = np.arange(0, nx - q + 1, q)               # left column of every full cell
        ys = np.arange(0, ny - q + 1, q)               # top row of every full cell
        Y, X = np.meshgrid(ys, xs, indexing="ij")
        tl, tr = plane[Y, X], plane[Y, X + p]
        bl, br = plane[Y + p, X], plane[Y + p, X + p]
        tlo, thi = lift(tl, tr)                        # along x
        blo, bhi = lift(bl, br)
        plane[Y, X], plane[Y + p, X] = lift(tlo, blo)  # along y: the lows ...
        plane[Y, X + p], plane[Y + p, X + p] = lift(thi, bhi)   # ... and the highs
        if nx & p:                                     # strip right of the last full column
            xe = len(xs) * q
            plane[ys, xe], plane[ys + p, xe] = lift(plane[ys, xe], plane[ys + p, xe])
        if ny & p:                                     # strip below the last full row
            ye = len(ys) * q
            plane[ye, xs], plane[ye, xs + p] = lift(plane[ye, xs], plane[ye, xs + p])
        p = q


def _huffman_lengths(freq: dict) -> dict:
    if len(freq) == 1:
        return {next(iter(freq)): 1}
    heap = [(f, i, [s]) for i, (s, f) in enumerate(sorted(freq.items()))]
    heapq.heapify(heap)
    depth = {s: 0 for s in freq}
    cnt = len(heap)
    while len(heap) > 1:
        f1, _, s1 = heapq.heappop(heap)
        f2, _, s2 = heapq.heappop(heap)
        for s in s1 + s2:
            depth[s] += 1
        heapq.heappush(heap, (f1 + f2, cnt, s1 + s2))
        cnt += 1
    assert max(depth.values()) <= 58
    return depth


def _canonical(lengths: dict) -> dict:
    """OpenEXR's canonical assignment: the longest codes take the numerically smallest values."""
    n = [0] * 59
    for l in lengths.values():
        n[l] += 1
    c = 0
    start = [0] * 59
    for l in range(58, 0, -1):
        start[l] = c
        c = (c + n[l]) >> 1
    codes = {}
    for s in sorted(lengths):
        l = lengths[s]
        codes[s] = (start[l], l)
        start[l] += 1
    return codes


class _Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, nbits, value):
        self.v = (self.v << nbits) | (value & ((1 << nbits) - 1))
        self.n += nbits

    def bytes(self):
        pad = (-self.n) % 8
        return (self.v << pad).to_bytes((self.n + pad) // 8, "big") if self.n else b""


def _huf_compress(data: list, use_runs: bool = True) -> bytes:
    if not data:
        return b""
    freq = {}
    for s in data:
        freq[s] = freq.get(s, 0) + 1
    im, iM = min(freq), max(freq) + 1           # iM: the run-length pseudo symbol
    freq[iM] = 1
    codes = _canonical(_huffman_lengths(freq))
    table = _Bits()
    s = im
    while s <= iM:
        l = codes[s][1] if s in codes else 0
        if l == 0:
            z = 1
            while s + z <= iM and s + z not in codes and z < 255 + 6:
                z += 1
            if z >= 2:
                if z >= 6:
                    table.put(6, 63)
                    table.put(8, z - 6)
                else:
                    table.put(6, 59 + z - 2)
                s += z
                continue
        table.put(6, l)
        s += 1
    tab = table.bytes()
    bits = _Bits()
    rc, rl = codes[iM]
    i = 0
    while i < len(data):
        v = data[i]
        run = 0
        while use_runs and i + run + 1 < len(data) and data[i + run + 1] == v and run < 255:
            run += 1
        c, l = codes[v]
        if run and l + rl + 8 < l * run:
            bits.put(l, c)
            bits.put(rl, rc)
            bits.put(8, run)
            i += run + 1
        else:
            bits.put(l, c)
            i += 1
    body = bits.bytes()
    return struct.pack("<iiiii", im, iM, len(tab), bits.n, 0) + tab + body


def _piz(raw: bytes, nx: int, ny: int, types: list) -> bytes:
    words = list(np.frombuffer(raw, "<u2").astype(np.int64))
    # per line, per channel -> planar per channel
    sizes = [1 if t == HALF else 2 for t in types]
    planes = [[] for _ in types]
    o = 0
    for _ in range(ny):
        for c, sz in enumerate(sizes):
            planes[c] += words[o:o + nx * sz]
            o += nx * sz
    tmp = [int(v) for p in planes for v in p]
    present = np.zeros(1 << 16, bool)
    present[np.array(tmp, dtype=np.int64)] = True
    present[0] = False
    bitmap = np.packbits(present, bitorder="little")
    nz = np.nonzero(bitmap)[0]
    mn, mxb = (int(nz[0]), int(nz[-1])) if len(nz) else (8191, 0)
    lut = np.zeros(1 << 16, np.int64)
    keep = present.copy()
    keep[0] = True
    vals = np.nonzero(keep)[0]
    lut[vals] = np.arange(len(vals))
    maxv = len(vals) - 1
    arr = lut[np.array(tmp, dtype=np.int64)]
    base = 0
    for sz in sizes:
        # a channel of sz 16-bit words per pixel is sz interleaved planes, each transformed alone
        block = arr[base:base + nx * ny * sz].reshape(ny, nx, sz)
        for j in range(sz):
            plane = np.ascontiguousarray(block[:, :, j])
            _wavelet_forward_2d(plane, maxv)
            block[:, :, j] = plane
        base += nx * ny * sz
    huf = _huf_compress([int(v) for v in arr])
    out = struct.pack("<HH", mn, mxb)
    if mn <= mxb:
        out += bitmap[mn:mxb + 1].tobytes()
    return out + struct.pack("<i", len(huf)) + huf


def _compress(raw: bytes, comp: int, nx: int, ny: int, types: list, force: bool) -> bytes:
    if comp == NONE:
        return raw
    if comp == RLE:
        data = _rle(_predict_split(raw))
    elif comp in (ZIPS, ZIP):
        data = zlib.compress(_predict_split(raw), 6)
    else:
        data = _piz(raw, nx, ny, types)
    # OpenEXR stores a chunk raw unless compression shrinks it; `force` keeps the compressed
    # form whenever its size differs from the raw size (still a valid file) so tests always
    # exercise the codec
    if len(data) < len(raw) or (force and len(data) != len(raw)):
        return data
    return raw


def write_exr(path: str, channels: dict, comp: int = NONE, ptype=HALF, tile: int = 0,
              data_origin=(0, 0), force: bool = True) -> bytes:
    """channels: name -> (h, w) array, written in sorted name order (the OpenEXR rule).
    ptype: one pixel type for all channels, or a dict name -> type."""
    names = sorted(channels)
    h, w = next(iter(channels.values())).shape
    types = [ptype[n] if isinstance(ptype, dict) else ptype for n in names]
    x0, y0 = data_origin
    chl = b"".join(n.encode() + b"\0" + struct.pack("<iB3xii", t, 0, 1, 1) for n, t in zip(names, types)) + b"\0"
    box = struct.pack("<iiii", x0, y0, x0 + w - 1, y0 + h - 1)
    hdr = (_attr("channels", "chlist", chl) + _attr("compression", "compression", bytes([comp]))
           + _attr("dataWindow", "box2i", box) + _attr("displayWindow", "box2i", box)
           + _attr("lineOrder", "lineOrder", b"\0") + _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
           + _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0))
           + _attr("screenWindowWidth", "float", struct.pack("<f", 1.0)))
    if tile:
        hdr += _attr("tiles", "tiledesc", struct.pack("<IIB", tile, tile, 0))
    hdr += b"\0"
    version = 2 | (0x200 if tile else 0)
    head = struct.pack("<II", 20000630, version) + hdr

    def block(xa, ya, nx, ny):
        raw = b"".join(_values(channels[n][ya + y, xa:xa + nx], t)
                       for y in range(ny) for n, t in zip(names, types))
        return _compress(raw, comp, nx, ny, types, force)

    chunks = []
    if tile:
        for ty in range((h + tile - 1) // tile):
            for tx in range((w + tile - 1) // tile):
                nx, ny = min(tile, w - tx * tile), min(tile, h - ty * tile)
                d = block(tx * tile, ty * tile, nx, ny)
                chunks.append(struct.pack("<iiiii", tx, ty, 0, 0, len(d)) + d)
    else:
        lpb = _LINES[comp]
        for ya in range(0, h, lpb):
            d = block(0, ya, w, min(lpb, h - ya))
            chunks.append(struct.pack("<ii", y0 + ya, len(d)) + d)
    off = len(head) + 8 * len(chunks)
    table = b""
    for c in chunks:
        table += struct.pack("<Q", off)
        off += len(c)
    data = head + table + b"".join(chunks)
    with open(path, "wb") as fh:
        fh.write(data)
    return data


def expected_rgba(channels: dict, ptype=HALF) -> np.ndarray:
    """What LoadEXR returns for such a file: (h, w, 4) float32, values rounded through the
    stored pixel type, A = 1 without an alpha channel, one channel replicated into four."""
    def stored(n):
        t = ptype[n] if isinstance(ptype, dict) else ptype
        a = channels[n]
        if t == HALF:
            return a.astype(np.float16).astype(np.float32)
        if t == FLOAT:
            return a.astype(np.float32)
        return a.astype(np.uint32).view(np.float32)

    names = sorted(channels)
    if len(names) == 1:
        v = stored(names[0])
        return np.stack([v, v, v, v], -1)
    short = {n.rsplit(".", 1)[-1]: n for n in names[:4]}
    h, w = channels[names[0]].shape
    a = stored(short["A"]) if "A" in short else np.ones((h, w), np.float32)
    return np.stack([stored(short["R"]), stored(short["G"]), stored(short["B"]), a], -1)
