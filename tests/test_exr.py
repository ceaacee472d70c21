"""OpenEXR texture decoding (host/exr_read.cpp via rtgh_read_image): what the reference's
Texture::ReadExr -> LoadEXR hands the texture code (src/Texture.cpp:185-189,
src/Helper.cpp:346-359), on every codec LoadEXR reads.  Files come from the independent
test-side encoder tests/exr_codec.py; decoded texels must equal the stored values bit for bit."""
import os

import numpy as np
import pytest

from rtg import native
from rtg._abi import RtgError

import exr_codec as X

pytestmark = pytest.mark.skipif(not os.path.exists(native.LIB_PATH), reason="librtghost.so not built")


def _image(h, w, seed, alpha=False, scale=4.0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    ch = {
        "R": (xx / w) * scale,                                       # smooth ramp
        "G": rng.standard_normal((h, w)).astype(np.float32) * scale,  # noise, negatives
        "B": np.where((xx // 7 + yy // 5) % 2 == 0, 0.25, 1e3).astype(np.float32),  # runs
    }
    ch["B"][: h // 3] = 0.0                                           # a zero band
    if alpha:
        ch["A"] = np.full((h, w), 0.5, np.float32)
    return ch


def _check(path, ch, ptype):
    got = native.read_image(path)
    want = X.expected_rgba(ch, ptype)[..., :3]
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.astype(np.float32).view(np.uint32))


CODECS = [("none", X.NONE), ("rle", X.RLE), ("zips", X.ZIPS), ("zip", X.ZIP), ("piz", X.PIZ)]


@pytest.mark.parametrize("cname,comp", CODECS)
@pytest.mark.parametrize("ptype", [X.HALF, X.FLOAT], ids=["half", "float"])
@pytest.mark.parametrize("tile", [0, 16], ids=["scanline", "tiled"])
def test_codecs_roundtrip(tmp_path, cname, comp, ptype, tile):
    ch = _image(45, 37, seed=hash((cname, ptype, tile)) & 0xFFFF, alpha=(ptype == X.FLOAT))
    p = str(tmp_path / f"t_{cname}.exr")
    X.write_exr(p, ch, comp, ptype, tile=tile)
    _check(p, ch, ptype)


def test_piz_16bit_wavelet_and_runs(tmp_path):
    """> 2^14 distinct 16-bit words switch PIZ to the 16-bit lifting; long runs exercise the
    Huffman run-length symbol."""
    rng = np.random.default_rng(7)
    h, w = 64, 300
    ch = {c: rng.uniform(-5e4, 5e4, (h, w)).astype(np.float32) for c in "RGB"}
    ch["G"][10:30] = 3.0
    p = str(tmp_path / "big.exr")
    X.write_exr(p, ch, X.PIZ, X.FLOAT)
    _check(p, ch, X.FLOAT)


def test_mixed_pixel_types_and_window(tmp_path):
    ch = _image(20, 33, seed=3)
    types = {"R": X.HALF, "G": X.FLOAT, "B": X.UINT}
    ch["B"] = np.arange(20 * 33, dtype=np.float32).reshape(20, 33) * 1000
    for comp in (X.NONE, X.ZIP, X.PIZ):
        p = str(tmp_path / f"mixed{comp}.exr")
        X.write_exr(p, ch, comp, types, data_origin=(-5, 12))
        _check(p, ch, types)


def test_single_channel_replicated(tmp_path):
    ch = {"Y": np.linspace(0, 2, 24 * 18, dtype=np.float32).reshape(18, 24)}
    p = str(tmp_path / "y.exr")
    X.write_exr(p, ch, X.ZIP, X.HALF)
    _check(p, ch, X.HALF)


def test_layer_names_use_last_component(tmp_path):
    base = _image(12, 10, seed=5)
    ch = {"diffuse." + k: v for k, v in base.items()}
    p = str(tmp_path / "layer.exr")
    X.write_exr(p, ch, X.RLE, X.HALF)
    got = native.read_image(p)
    want = X.expected_rgba(base, X.HALF)[..., :3]
    assert np.array_equal(got, want)


def test_missing_channel_fails_loudly(tmp_path):
    ch = _image(8, 8, seed=1)
    del ch["B"]
    p = str(tmp_path / "rg.exr")
    X.write_exr(p, ch, X.NONE, X.HALF)
    with pytest.raises(RtgError, match="B channel not found"):
        native.read_image(p)


def test_corrupt_and_unsupported_fail_loudly(tmp_path):
    ch = _image(40, 16, seed=2)
    p = str(tmp_path / "c.exr")
    data = X.write_exr(p, ch, X.PIZ, X.HALF)
    with open(p, "wb") as fh:                      # truncate inside the last chunk
        fh.write(data[:-40])
    with pytest.raises(RtgError):
        native.read_image(p)
    q = str(tmp_path / "not.exr")
    with open(q, "wb") as fh:
        fh.write(b"P3\n1 1\n255\n0 0 0\n")
    with pytest.raises(RtgError, match="not an OpenEXR"):
        native.read_image(q)


def test_native_writer_reads_back(tmp_path):
    """rtgh_save_image's OpenEXR HALF output (Image::saveImage -> ExrLibrary::SaveExr, src/Image.cpp:26-34, src/Helper.cpp:361-412)
    decodes to the half-rounded framebuffer."""
    rng = np.random.default_rng(11)
    img = (rng.uniform(0, 300, (17, 23, 3))).astype(np.float32)
    p = str(tmp_path / "out.exr")
    native.save_image(p, img)
    got = native.read_image(p)
    assert np.array_equal(got, img.astype(np.float16).astype(np.float32))


def test_scene_texture_exr_matches_native_parse(tmp_path):
    """An .exr <Image> reaches rtg_texture_desc.texels identically through both hosts."""
    from rtg import scenegen
    from rtg.scene import parse_xml, write_xml
    ch = _image(16, 32, seed=9, scale=2.0)
    X.write_exr(str(tmp_path / "env.exr"), ch, X.PIZ, X.HALF)
    sc = scenegen.textured(32, 24)
    sc.images = [str(tmp_path / "env.exr")] + list(sc.images[1:])
    xml = write_xml(sc, str(tmp_path / "s.xml"))
    py = parse_xml(xml)
    with native.NativeScene(xml) as ns:
        d = native.desc_to_dict(ns.desc)
    t0 = py.textures[0]
    want = X.expected_rgba(ch, X.HALF)[..., :3]
    assert np.array_equal(np.asarray(t0.texels, np.float32).reshape(want.shape), want)
    assert np.array_equal(np.asarray(d["textures"][0]["texels"], np.float32).reshape(want.shape), want)


@pytest.mark.parametrize("comp", [X.RLE, X.ZIP, X.PIZ])
def test_corrupted_files_never_crash(tmp_path, comp):
    """Random byte flips / truncations of valid files either decode or fail with RtgError."""
    ch = _image(40, 23, seed=comp)
    good = X.write_exr(str(tmp_path / "g.exr"), ch, comp, X.HALF)
    rng = np.random.default_rng(comp)
    p = str(tmp_path / "bad.exr")
    for trial in range(150):
        b = bytearray(good)
        if trial % 5 == 4:
            b = b[:int(rng.integers(8, len(b)))]
        else:
            for _ in range(int(rng.integers(1, 8))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        with open(p, "wb") as fh:
            fh.write(bytes(b))
        try:
            img = native.read_image(p)
            assert img.ndim == 3 and img.shape[2] == 3
        except RtgError:
            pass


@pytest.mark.parametrize("w,h", [(1, 1), (1, 29), (31, 1), (2, 3), (33, 17), (64, 63), (5, 100)])
@pytest.mark.parametrize("ptype", [X.HALF, X.FLOAT], ids=["half", "float"])
def test_piz_wavelet_odd_shapes(tmp_path, w, h, ptype):
    """The inverse PIZ wavelet on lattices whose sides are not powers of two (odd cell columns /
    rows at every level, degenerate one-pixel sides), both lifting forms (FLOAT words exceed 2^14
    distinct values), against the test-side encoder."""
    ch = _image(w, h, seed=w * 131 + h, scale=3.0)
    p = str(tmp_path / f"piz_{w}x{h}.exr")
    X.write_exr(p, ch, X.PIZ, ptype)
    _check(p, ch, ptype)


def test_canonical_code_known_answer():
    """OpenEXR's canonical assignment, worked by hand from the format rule (longest codes
    smallest; a length's first code = half the value past the next longer length's codes):
    lengths {0:2, 1:2, 2:2, 3:3, 4:3} -> length 3 takes 000, 001; length 2 starts at 2 >> 1 = 1."""
    codes = X._canonical({0: 2, 1: 2, 2: 2, 3: 3, 4: 3})
    assert codes == {3: (0b000, 3), 4: (0b001, 3), 0: (0b01, 2), 1: (0b10, 2), 2: (0b11, 2)}


def test_wavelet_forward_known_answer():
    """One 2x2 cell, narrow lifting, by hand: along x (10,20) -> (15,-10), (30,40) -> (35,-10);
    along y the lows (15,35) -> (25,-20) and the highs (-10,-10) -> (-10,0)."""
    plane = np.array([[10, 20], [30, 40]], np.int64)
    X._wavelet_forward_2d(plane, maxval=100)
    assert plane.tolist() == [[25, (-10) & 0xFFFF], [(-20) & 0xFFFF, 0]]
    wide = np.array([[0, 0xFFFF], [0x8000, 1]], np.int64)
    X._wavelet_forward_2d(wide, maxval=0xFFFF)     # the modular form, checked by its inverse
    lo, hi = int(wide[0, 0]), int(wide[1, 0])
    assert 0 <= lo < 65536 and 0 <= hi < 65536


@pytest.mark.parametrize("lengths,msg", [
    ({0: 1, 1: 1, 2: 1}, "does not fit"),                 # three 1-bit codes
    ({0: 1}, "prefix code"),     # one 1-bit code '0', every other symbol 20 bits from 0...0
])
def test_piz_rejects_invalid_code_lengths(tmp_path, monkeypatch, lengths, msg):
    """A PIZ length table that is not a prefix code is refused loudly, not decoded."""
    def bogus(freq):
        syms = sorted(freq)
        return {s: lengths.get(i, 20 if len(lengths) == 1 else 1) for i, s in enumerate(syms)}
    ch = {"Y": np.arange(16, dtype=np.float32).reshape(4, 4)}     # >= 4 symbols
    monkeypatch.setattr(X, "_huffman_lengths", bogus)
    p = str(tmp_path / "bad.exr")
    X.write_exr(p, ch, X.PIZ, X.HALF)
    with pytest.raises(RtgError, match=msg):
        native.read_image(p)


def test_piz_long_codes_round_trip_and_refuse_high_bits(tmp_path, monkeypatch):
    """codes longer than 32 bits.  Every symbol gets a 40-bit code (an incomplete but
    prefix-free table, values 0..n-1): the file round-trips exactly.  The same table with the
    first symbol's payload code given a 1 in its top bit (value >= 2^39, past every code of that
    length) is an invalid code and must be refused, not wrapped into a valid 32-bit value."""
    ch = {"Y": np.arange(16, dtype=np.float32).reshape(4, 4)}
    monkeypatch.setattr(X, "_huffman_lengths", lambda freq: {s: 40 for s in freq})
    p = str(tmp_path / "long.exr")
    X.write_exr(p, ch, X.PIZ, X.HALF)
    np.testing.assert_array_equal(native.read_image(p), X.expected_rgba(ch, X.HALF)[..., :3])
    canon = X._canonical

    def high_bit(lengths):
        codes = canon(lengths)
        s0 = min(codes)
        c, l = codes[s0]
        codes[s0] = (c | (1 << (l - 1)), l)
        return codes
    monkeypatch.setattr(X, "_canonical", high_bit)
    p2 = str(tmp_path / "bad_long.exr")
    X.write_exr(p2, ch, X.PIZ, X.HALF)
    with pytest.raises(RtgError, match="invalid code"):
        native.read_image(p2)
