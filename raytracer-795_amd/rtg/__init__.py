"""rtg — MI355X-native render loop for the CENG795 XML ray tracer (badiba/raytracer-795).

The hot path (ray generation, BVH closest-hit, recursive shading) runs in the HIP
library librtg.so behind the C ABI of include/rtg.h; this package is the host-side
mirror of the reference's Parser / Scene::renderScene() / Image interface.
"""
from . import _abi
from ._abi import RtgError, load_library
from .render import Comm, Renderer, render_scene, save_image, tonemap
from .scene import Camera, Instance, Light, Material, Object, Scene, Texture, parse_xml, write_xml

__all__ = ["RtgError", "load_library", "Comm", "Renderer", "render_scene", "save_image", "tonemap", "Camera", "Instance", "Light",
           "Material", "Object", "Scene", "Texture", "parse_xml", "write_xml", "_abi"]
