"""rtg_cli (native parser + librtg + Image::saveImage, the reference's `./raytracer scene.xml`)
writes the same image files as the Python host path for the same XML."""
import os
import subprocess

import numpy as np
import pytest

import rtg
from rtg import native, scenegen
from rtg.scene import parse_xml, write_xml

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,make", [
    ("simple", lambda: scenegen.simple(40, 30)),
    ("cornell", lambda: scenegen.cornell(32, 24, spp=4)),
    ("cornell_pt", lambda: scenegen.cornell_pt(32, 24, spp=4)),
    ("dragon_ply", lambda: scenegen.dragon1m(40, 24, spp=2, nu=60, nv=30)),
])
def test_cli_matches_python_host(gpu, tmp_path, name, make):
    sc = make()
    sc.cameras[0].image_name = f"{name}.png"
    xml = write_xml(sc, str(tmp_path / f"{name}.xml"))
    cli_dir, py_dir = tmp_path / "cli", tmp_path / "py"
    cli_dir.mkdir()
    py_dir.mkdir()
    r = subprocess.run([native.CLI_PATH, xml, "--out-dir", str(cli_dir), "--device", str(gpu)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "BVH construction complete." in r.stdout
    rtg.render_scene(parse_xml(xml), out_dir=str(py_dir), device=gpu)
    a = (cli_dir / f"{name}.png").read_bytes()
    b = (py_dir / f"{name}.png").read_bytes()
    assert a == b


def test_cli_exr_output(gpu, tmp_path):
    """Non-.png names go through the OpenEXR HALF writer (src/Helper.cpp:361-412)."""
    sc = scenegen.cornell_pt(24, 18, spp=2)
    sc.cameras[0].image_name = "pt.exr"
    xml = write_xml(sc, str(tmp_path / "pt.xml"))
    native.render_scene(xml, device=gpu, out_dir=str(tmp_path))
    with rtg.Renderer(parse_xml(xml), device=gpu) as r:
        img = r.render(0)
    from rtg.render import exr_half_bytes
    assert (tmp_path / "pt.exr").read_bytes() == exr_half_bytes(img)


def test_cli_tonemap_outputs(gpu, tmp_path):
    """A camera with a hw5 <Tonemap>: the HDR image under its ImageName and the tone-mapped
    one next to it as .png, identical between the native and the Python host."""
    sc = scenegen.cornell_pt(32, 24, spp=2)
    sc.cameras[0].image_name = "tm.exr"
    sc.cameras[0].tonemap = (0.18, 1.0, 1.0, 2.2)
    xml = write_xml(sc, str(tmp_path / "tm.xml"))
    cli_dir, py_dir = tmp_path / "cli", tmp_path / "py"
    cli_dir.mkdir()
    py_dir.mkdir()
    native.render_scene(xml, device=gpu, out_dir=str(cli_dir))
    rtg.render_scene(parse_xml(xml), out_dir=str(py_dir), device=gpu)
    for f in ("tm.exr", "tm.png"):
        assert (cli_dir / f).read_bytes() == (py_dir / f).read_bytes(), f


def test_cli_envmap_exr_texture(gpu, tmp_path):
    """hw6 image-based lighting from an OpenEXR sky (decoded by host/exr_read.cpp in both
    hosts), HDR output plus the tone-mapped .png: native == Python host, and the frame equals
    the oracle's on the generated (in-memory) scene."""
    import pyoracle
    from rtg.render import exr_half_bytes
    sc = scenegen.envmap(40, 30, spp=2)
    sc.cameras[0].tonemap = (0.18, 0.5, 1.0, 2.2)
    cli_dir, py_dir = tmp_path / "cli", tmp_path / "py"
    cli_dir.mkdir()
    py_dir.mkdir()
    (tmp_path / "sky.exr").write_bytes(exr_half_bytes(sc.textures[0].texels))
    xml = write_xml(sc, str(tmp_path / "env.xml"))
    native.render_scene(xml, device=gpu, out_dir=str(cli_dir))
    rtg.render_scene(parse_xml(xml), out_dir=str(py_dir), device=gpu)
    for f in ("env.exr", "env.png"):
        assert (cli_dir / f).read_bytes() == (py_dir / f).read_bytes(), f
    with rtg.Renderer(parse_xml(xml), device=gpu) as r:
        img = r.render(0)
    ref, _, _, _ = pyoracle.Oracle(sc).render(0)
    assert float(np.nanmax(np.abs(img.astype(np.float64) - ref))) < 1e-3
