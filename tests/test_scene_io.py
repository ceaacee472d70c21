"""Host plumbing around the hot path: the XML/PLY parser mirror of src/Parser.h (quirks
included), the XML writer used for the synthetic scenes, and Image::saveImage's formats."""
import os
import struct

import numpy as np
import pytest

from rtg import _abi as A
from rtg import scenegen
from rtg.render import _is_png, exr_half_bytes, ppm_p3_bytes
from rtg.scene import parse_object_transformations, parse_xml, read_ply, write_ply_binary, write_xml


def desc_equal(a, b):
    da, ka = a.to_desc()
    db, kb = b.to_desc()
    import ctypes as C
    # compare every flattened array bitwise and every record field
    for x, y in zip(ka, kb):
        if isinstance(x, np.ndarray):
            assert x.dtype == y.dtype and x.shape == y.shape
            assert np.array_equal(np.ascontiguousarray(x).view(np.uint8), np.ascontiguousarray(y).view(np.uint8))
        else:
            assert C.sizeof(x) == C.sizeof(y)
            bx, by = bytes(x), bytes(y)
            # texel pointers differ between the two descriptors: compare structs without them
            if isinstance(x, (A.TextureDesc * len(x)).__mro__[0]):
                continue
            assert bx == by
    for f, _ in A.SceneDesc._fields_:
        v1, v2 = getattr(da, f), getattr(db, f)
        if isinstance(v1, (int, float)):
            assert v1 == v2, f


@pytest.mark.parametrize("name,make", [
    ("simple", lambda: scenegen.simple(16, 16)),
    ("bunny", lambda: scenegen.bunny5k(16, 12, level=2)),
    ("dragon", lambda: scenegen.dragon1m(16, 9, spp=4, nu=40, nv=20)),
    ("cornell", lambda: scenegen.cornell(16, 12, spp=4)),
])
def test_xml_round_trip(tmp_path, name, make):
    sc = make()
    xml = write_xml(sc, str(tmp_path / f"{name}.xml"))
    back = parse_xml(xml)
    desc_equal(sc, back)


def test_textured_round_trip(tmp_path):
    from PIL import Image
    sc = scenegen.textured(16, 12)
    Image.fromarray(scenegen.checker_texture().astype(np.uint8)).save(tmp_path / "checker.png")
    sc.images = ["checker.png"]
    xml = write_xml(sc, str(tmp_path / "tex.xml"))
    back = parse_xml(xml)
    assert len(back.textures) == len(sc.textures)
    for t1, t2 in zip(sc.textures, back.textures):
        assert (t1.kind, t1.decal, t1.interp, t1.normalizer) == (t2.kind, t2.decal, t2.interp, t2.normalizer)
        if t1.texels is not None:
            assert np.array_equal(t1.texels, t2.texels)
    desc_equal(sc, back)


def test_object_transformation_parsing_quirks():
    # src/Parser.h:769-796: tokens are found only at s/t/r (a composite only as first token)
    T, S, R, Cc = A.XF_TRANSLATION, A.XF_SCALING, A.XF_ROTATION, A.XF_COMPOSITE
    assert parse_object_transformations("t1 s2 r3") == [(T, 1), (S, 2), (R, 3)]
    assert parse_object_transformations("c1 t2") == [(Cc, 1), (T, 2)]
    assert parse_object_transformations("t1 c1") == [(T, 1)]
    assert parse_object_transformations("r12\ns3") == [(R, 12), (S, 3)]


def test_texture_map_state_carries_over(tmp_path):
    xml = tmp_path / "s.xml"
    xml.write_text("""<Scene>
<Cameras><Camera id="1"><Position>0 0 0</Position><Gaze>0 0 -1</Gaze><Up>0 1 0</Up>
<NearPlane>-1 1 -1 1</NearPlane><NearDistance>1</NearDistance><ImageResolution>4 4</ImageResolution>
<ImageName>a.png</ImageName></Camera></Cameras>
<Materials><Material id="1"><AmbientReflectance>1 1 1</AmbientReflectance>
<DiffuseReflectance>1 1 1</DiffuseReflectance><SpecularReflectance>0 0 0</SpecularReflectance></Material></Materials>
<Textures>
<TextureMap id="1" type="perlin"><DecalMode>replace_kd</DecalMode><NoiseConversion>absval</NoiseConversion><NoiseScale>3</NoiseScale></TextureMap>
<TextureMap id="2" type="perlin"><BumpFactor>0.5</BumpFactor></TextureMap>
</Textures>
<VertexData>0 0 -2</VertexData>
<Objects><Sphere id="1"><Material>1</Material><Textures>1 2</Textures><Center>1</Center><Radius>1</Radius></Sphere></Objects>
<Lights><AmbientLight>1 1 1</AmbientLight></Lights>
</Scene>""")
    sc = parse_xml(str(xml))
    t1, t2 = sc.textures
    # the second map inherits decal mode, noise conversion and scale from the first
    assert t2.decal == A.DECAL_REPLACE_KD and t2.noise_conv == A.NC_ABSVAL and t2.noise_scale == 3.0
    assert t2.bump_factor == 0.5
    assert sc.objects[0].textures == [1, 2]


def test_ply_quad_split_and_offsets(tmp_path):
    verts = np.array([(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0)], np.float32)
    write_ply_binary(str(tmp_path / "q.ply"), verts, np.array([[0, 1, 2, 3]]))
    v, uv, f = read_ply(str(tmp_path / "q.ply"))
    assert f == [[0, 1, 2, 3]] and uv is None
    xml = tmp_path / "s.xml"
    xml.write_text("""<Scene><Cameras><Camera id="1"><Position>0 0 1</Position><Gaze>0 0 -1</Gaze><Up>0 1 0</Up>
<FovY>60</FovY><NearDistance>1</NearDistance><ImageResolution>8 4</ImageResolution><ImageName>a.exr</ImageName>
</Camera></Cameras>
<Materials><Material id="1"><AmbientReflectance>1 1 1</AmbientReflectance><DiffuseReflectance>1 1 1</DiffuseReflectance>
<SpecularReflectance>0 0 0</SpecularReflectance></Material></Materials>
<VertexData>5 5 5
6 6 6</VertexData>
<Objects><Mesh id="1"><Material>1</Material><Faces plyFile="q.ply"/></Mesh></Objects>
<Lights></Lights></Scene>""")
    sc = parse_xml(str(xml))
    # quad (0,1,2,3) -> (0,1,2),(2,3,0), indices offset by the 2 XML vertices (1-based)
    assert sc.objects[0].faces.tolist() == [[3, 4, 5], [5, 6, 3]]
    assert len(sc.vertices) == 6
    cam = sc.cameras[0]
    half = np.float32(np.tan(np.float32(np.float32(60 * 0.5) * (np.pi / np.float32(180.0)))))
    assert cam.near_plane[3] == pytest.approx(float(half), rel=1e-6)
    assert cam.near_plane[1] == pytest.approx(2 * float(half), rel=1e-6)


def test_image_writers():
    assert _is_png("out.png") and _is_png("a.png.exr") and not _is_png("out.exr")
    img = np.array([[[300.0, 12.7, -0.5]]], np.float32)
    assert ppm_p3_bytes(img) == b"P3\n1 1\n255\n255 12 0 \n"
    exr = exr_half_bytes(np.zeros((2, 3, 3), np.float32))
    assert exr[:4] == b"\x76\x2f\x31\x01"
    assert len(exr) > 2 * 3 * 3 * 2


# (unsigned char)_data[i] of src/Image.cpp:96 on x86-64 gcc: cvttss2si to int32, low byte kept
PPM_CASES = [(-1.0, 255), (-255.5, 1), (-300.0, 212), (-0.5, 0), (-0.0, 0), (float("nan"), 0),
             (-float("inf"), 0), (float("inf"), 255), (300.0, 255), (12.7, 12), (-3e9, 0),
             (-2147483648.0, 0), (255.9, 255), (-2147483520.0, 128), (-65535.0, 1)]


def test_ppm_negative_pixels_keep_the_low_byte():
    vals = [v for v, _ in PPM_CASES]
    img = np.array(vals, np.float32).reshape(1, len(vals) // 3, 3)
    body = ppm_p3_bytes(img).decode().split("\n")[3].split()
    assert [int(x) for x in body] == [u for _, u in PPM_CASES]


def test_ppm_cast_matches_compiled_x86_cast(tmp_path):
    """Pin the expected bytes on the host compiler itself: the reference's clamp + cast
    (src/Image.cpp:64-68, 96) compiled by gcc, fed the same floats."""
    import shutil
    import subprocess
    import platform
    if shutil.which("gcc") is None or platform.machine() != "x86_64":
        pytest.skip("needs gcc on x86-64")
    src = tmp_path / "cast.c"
    src.write_text("""#include <stdio.h>
#include <stdlib.h>
int main(int argc, char** argv) {
    for (int i = 1; i < argc; i++) {
        volatile float v = strtof(argv[i], 0);
        if (v > 255) v = 255;
        printf("%d ", (unsigned char)v);
    }
    return 0;
}
""")
    exe = tmp_path / "cast"
    subprocess.run(["gcc", "-O3", "-std=c11", "-o", str(exe), str(src)], check=True)
    args = ["nan" if v != v else repr(float(v)) for v, _ in PPM_CASES]
    out = subprocess.run([str(exe)] + args, check=True, capture_output=True, text=True).stdout.split()
    assert [int(x) for x in out] == [u for _, u in PPM_CASES]
