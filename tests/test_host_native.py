"""The native host side (librtghost.so: C++ Parser / Image / renderScene loop, include/rtg_host.h)
against the Python mirror rtg/scene.py: the same XML file must give the same rtg_scene_desc,
value for value, and Image::saveImage must write the same bytes."""
import ctypes as C
import os

import numpy as np
import pytest

from rtg import _abi as A
from rtg import native, scenegen
from rtg.render import exr_half_bytes, ppm_p3_bytes
from rtg.scene import parse_xml, write_xml


def _eq(a, b, path=""):
    if isinstance(a, dict):
        assert a.keys() == b.keys(), path
        for k in a:
            _eq(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, list):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _eq(x, y, f"{path}[{i}]")
    elif isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape, path
        assert np.array_equal(a.view(np.uint8) if a.dtype.kind == "f" else a,
                              b.view(np.uint8) if b.dtype.kind == "f" else b), path
    elif isinstance(a, float):
        assert np.float32(a).tobytes() == np.float32(b).tobytes(), (path, a, b)
    else:
        assert a == b, (path, a, b)


def _compare(xml):
    py = parse_xml(xml)
    d_py, keep = py.to_desc()
    with native.NativeScene(xml) as ns:
        _eq(native.desc_to_dict(d_py), native.desc_to_dict(ns.desc))
        assert len(ns.cameras) == len(py.cameras)
        for (cd, name), tm, cam in zip(ns.cameras, ns.tonemaps, py.cameras):
            assert name == cam.image_name
            assert bytes(cd) == bytes(cam.desc())
            assert (tm is None) == (cam.tonemap is None)
            if tm is not None:
                assert np.array_equal(np.float32(tm), np.float32(cam.tonemap))
    return py


SCENES = {
    "simple": lambda: scenegen.simple(16, 16),
    "bunny": lambda: scenegen.bunny5k(16, 12, level=2),
    "dragon_ply": lambda: scenegen.dragon1m(16, 9, spp=4, nu=40, nv=20),
    "cornell": lambda: scenegen.cornell(16, 12, spp=4),
    "multilight": lambda: scenegen.multilight(16, 12),
    "cornell_pt": lambda: scenegen.cornell_pt(16, 12, spp=4),
    "cornell_pt_tonemap": lambda: _with_tonemap(scenegen.cornell_pt(16, 12, spp=4)),
}


def _with_tonemap(sc):
    sc.cameras[0].tonemap = (0.18, 1.5, 0.9, 2.2)
    return sc


@pytest.mark.parametrize("name", list(SCENES))
def test_native_parser_matches_python(tmp_path, name):
    xml = write_xml(SCENES[name](), str(tmp_path / f"{name}.xml"))
    _compare(xml)


@pytest.mark.parametrize("fmt", ["png", "ppm"])
def test_native_parser_textures(tmp_path, fmt):
    from PIL import Image
    sc = scenegen.textured(16, 12)
    img = scenegen.checker_texture().astype(np.uint8)
    if fmt == "png":
        Image.fromarray(img).save(tmp_path / "checker.png")
    else:
        h, w, _ = img.shape
        (tmp_path / "checker.ppm").write_bytes(f"P6\n{w} {h}\n255\n".encode() + img.tobytes())
    sc.images = [f"checker.{fmt}"]
    xml = write_xml(sc, str(tmp_path / "tex.xml"))
    py = _compare(xml)
    assert py.textures[0].texels is not None


def test_native_parser_envmap_exr(tmp_path):
    """hw6 SphericalDirectionalLight over an OpenEXR sky: both hosts decode the file (native
    rtgh_read_image) to the same linear texels, normalizer 1, bilinear."""
    from rtg.render import exr_half_bytes
    sc = scenegen.envmap(16, 12)
    sky = sc.textures[0].texels
    (tmp_path / "sky.exr").write_bytes(exr_half_bytes(sky))
    xml = write_xml(sc, str(tmp_path / "env.xml"))
    py = _compare(xml)
    assert py.environment_light == 0
    assert np.array_equal(np.asarray(py.textures[0].texels, np.float32).reshape(sky.shape), sky)


def test_native_parser_quirks(tmp_path):
    """Hand-written XML: FovY / GazePoint cameras, composite-first transformation lists,
    texture-map state carried over, XML faces with offsets, instances, entity escapes."""
    xml = tmp_path / "q.xml"
    xml.write_text("""<?xml version="1.0"?>
<!-- quirk scene -->
<Scene>
  <MaxRecursionDepth>3</MaxRecursionDepth>
  <BackgroundColor>1 2</BackgroundColor>
  <ShadowRayEpsilon>1e-3</ShadowRayEpsilon>
  <Cameras>
    <Camera id="1" handedness="leftish">
      <Position>0 0 5</Position><GazePoint>0.1 0.2 0</GazePoint><Up>0 1 0</Up>
      <FovY>47.5</FovY><NearDistance>0.75</NearDistance><ImageResolution>33 17</ImageResolution>
      <NumSamples>5</NumSamples><FocusDistance>4</FocusDistance><ApertureSize>0.3</ApertureSize>
      <ImageName>  out&amp;1.png </ImageName>
      <Renderer>PathTracing</Renderer><RendererParams>NextEventEstimation</RendererParams>
    </Camera>
  </Cameras>
  <BRDFs><TorranceSparrow id="3" kdfresnel="true"><Exponent>11</Exponent></TorranceSparrow></BRDFs>
  <Materials>
    <Material id="1" degamma="true" BRDF="3"><DiffuseReflectance>0.5 0.25 0.125</DiffuseReflectance>
      <Roughness>0.1</Roughness></Material>
    <Material id="2" type="dielectric_x"><RefractionIndex>1.33</RefractionIndex>
      <AbsorptionCoefficient>0.1 0.2 0.3</AbsorptionCoefficient></Material>
  </Materials>
  <Textures>
    <TextureMap type="perlin"><DecalMode>bump_normal</DecalMode><NoiseScale>2.5</NoiseScale></TextureMap>
    <TextureMap><NoiseConversion>absval</NoiseConversion><BumpFactor>0.25</BumpFactor></TextureMap>
  </Textures>
  <Transformations>
    <Translation id="1">1 2 3</Translation><Scaling id="1">2 2 2</Scaling>
    <Rotation id="1">30 0 1 0</Rotation>
    <Composite id="1">1 0 0 1  0 1 0 2  0 0 1 3  0 0 0 1</Composite>
  </Transformations>
  <VertexData>0 0 0  1 0 0  0 1 0  1 1 0  0.5 0.5 1  2 2 2</VertexData>
  <TexCoordData>0 0 1 0 0 1 1 1</TexCoordData>
  <Objects>
    <Sphere id="1"><Material>2</Material><Center>5</Center><Radius>0.4</Radius>
      <Transformations>c1 t1 s1</Transformations><MotionBlur>0 0.5</MotionBlur></Sphere>
    <Triangle id="1"><Material>1</Material><Indices>1 2 3</Indices><Textures>1 2</Textures>
      <Transformations>r1 c1 t1</Transformations></Triangle>
    <Mesh id="7" shadingMode="smooth"><Material>1</Material><Textures>2</Textures>
      <Faces vertexOffset="1" textureOffset="2">0 1 2 1 2 3</Faces></Mesh>
    <MeshInstance id="8" baseMeshId="7" resetTransform=" True "><Material>2</Material>
      <Transformations>s1</Transformations></MeshInstance>
    <LightSphere id="2"><Material>1</Material><Center>6</Center><Radius>0.3</Radius>
      <Radiance>5 6 7</Radiance></LightSphere>
  </Objects>
  <Lights>
    <AmbientLight>10 10 10</AmbientLight>
    <PointLight id="1"><Position>0 4 0</Position><Intensity>100 100 100</Intensity></PointLight>
    <AreaLight id="1"><Position>0 3 0</Position><Normal>0 -1 0</Normal><Intensity>5 5 5</Intensity><Size>2</Size></AreaLight>
    <SpotLight id="1"><Position>1 3 0</Position><Direction>0 -1 0</Direction><Intensity>9 9 9</Intensity>
      <CoverageAngle>40</CoverageAngle><FalloffAngle>20</FalloffAngle></SpotLight>
  </Lights>
</Scene>
""")
    py = _compare(str(xml))
    assert py.cameras[0].image_name == "out&1.png"
    assert [o.is_light for o in py.objects] == [False, True, False, False]


def test_native_save_image_bytes(tmp_path):
    rng = np.random.default_rng(3)
    img = (rng.standard_normal((7, 9, 3)) * 200 + 100).astype(np.float32)
    img[0, 0] = [np.nan, -0.0, 255.9]
    img[0, 1] = [1e6, 65519.0, 65520.0]                     # half rounding to max / inf
    img[1, 0] = [3e-8, 6e-8, 1e-5]                           # half subnormals / zero
    img[1, 1] = [-np.inf, np.inf, 2.9802322e-08]
    for name, ref in (("a.png", ppm_p3_bytes(img)), ("a.exr", exr_half_bytes(img))):
        p = str(tmp_path / name)
        native.save_image(p, img)
        assert open(p, "rb").read() == ref, name


def test_native_parse_error_is_reported(tmp_path):
    p = tmp_path / "bad.xml"
    p.write_text("<Scene><Objects></Scene>")
    with pytest.raises(A.RtgError, match="XML"):
        native.NativeScene(str(p))
    with pytest.raises(A.RtgError):
        native.NativeScene(str(tmp_path / "missing.xml"))


def test_native_jpeg_texture(tmp_path):
    """JPEG textures decode through libjpeg 9 (dlopen'ed); PIL's decoder may round the IDCT
    differently, so the two hosts agree to a couple of 8-bit steps."""
    from PIL import Image
    sc = scenegen.textured(16, 12)
    Image.fromarray(scenegen.checker_texture().astype(np.uint8)).save(tmp_path / "checker.jpg", quality=95, subsampling=0)
    sc.images = ["checker.jpg"]
    xml = write_xml(sc, str(tmp_path / "tex.xml"))
    py = parse_xml(xml)
    with native.NativeScene(xml) as ns:
        t = ns.desc.textures[0]
        nat = np.ctypeslib.as_array(t.texels, shape=(t.height, t.width, 3))
        assert nat.shape == py.textures[0].texels.shape
        assert np.abs(nat - py.textures[0].texels).max() <= 3


def test_host_library_exports_every_declared_symbol():
    import re
    import subprocess
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "rtg_host.h")
    decl = set(re.findall(r"^\s*(?:int32_t|const char\*|void|const rtg_scene_desc\*)\s+(rtgh_\w+)\s*\(",
                          open(hdr).read(), re.M))
    assert len(decl) == 12
    out = subprocess.run(["nm", "-D", "--defined-only", native.LIB_PATH], capture_output=True, text=True, check=True)
    syms = set(re.findall(r"\sT\s(rtgh_\w+)", out.stdout))
    assert decl <= syms, decl - syms
    assert os.access(native.CLI_PATH, os.X_OK)


def test_native_parser_survives_corrupted_files(tmp_path):
    """Truncated / mutated scene files and PLYs parse or fail with an error, never crash
    (scripts/xml_fuzz.cpp runs the same idea under ASan/UBSan)."""
    rng = np.random.default_rng(7)
    sc = scenegen.dragon1m(8, 6, spp=1, nu=20, nv=10)
    good = open(write_xml(sc, str(tmp_path / "d.xml")), "rb").read()
    ply = [p for p in os.listdir(tmp_path) if p.endswith(".ply")][0]
    ply_good = (tmp_path / ply).read_bytes()
    for t in range(120):
        b = bytearray(good)
        if t % 3 == 0:
            b = b[:int(rng.integers(1, len(b)))]
        else:
            for _ in range(int(rng.integers(1, 6))):
                b[int(rng.integers(0, len(b)))] = int(rng.choice(list(b'<>"-9 e/\0')))
        if t % 4 == 3:                               # and a damaged mesh file
            pb = bytearray(ply_good)
            for _ in range(8):
                pb[int(rng.integers(0, min(len(pb), 400)))] = int(rng.integers(0, 256))
            (tmp_path / ply).write_bytes(bytes(pb[:int(rng.integers(1, len(pb)))]))
        else:
            (tmp_path / ply).write_bytes(ply_good)
        x = tmp_path / "m.xml"
        x.write_bytes(bytes(b))
        try:
            with native.NativeScene(str(x)) as ns:
                assert ns.desc.num_objects >= 0
        except A.RtgError:
            pass
