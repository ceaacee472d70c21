"""Host mirror of `Scene::renderScene()` / `Image` over the librtg C ABI.

    sc = rtg.parse_xml("scene.xml")        # new Scene(xml)         (src/Scene.cpp:455)
    rtg.render_scene(sc)                   # pScene->renderScene()  (src/Scene.cpp:294)

`Renderer` keeps the flattened scene resident on one GPU (rtg_scene_create) and renders
cameras into host or device framebuffers; `save_image` writes what Image::saveImage does
(src/Image.cpp:26-107): a P3 text PPM clamped to 255 when the name contains ".png",
otherwise an OpenEXR file (half RGB).
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import zlib

import numpy as np

from . import _abi as A
from .scene import Camera, Scene

DEFAULT_SEED = 0x5EED2026


class Renderer:
    def __init__(self, scene: Scene, device: int = 0, bvh_builder: int = A.RTG_BVH_AUTO, tlas: int = 0,
                 traversal_tree: int = 0, uniform_walk: int = 0):
        self.lib = A.load_library()
        self.scene = scene
        desc, self._keep = scene.to_desc()
        h = C.c_void_p()
        bo = A.BuildOpts(bvh_builder, tlas, traversal_tree, uniform_walk)
        A.check(self.lib.rtg_scene_create_ex(C.byref(desc), int(device), C.byref(bo), C.byref(h)), self.lib)
        self.handle = h
        self.device = device

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rtg_scene_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def opts(seed=DEFAULT_SEED, row_offset=0, row_stride=1, traversal=0, max_batch_rays=0, collect_stats=0,
             collect_timing=0, streams=0, row_block=1, compact_rows=0, num_devices=0, devices=None, schedule=0,
             tile_band=0, segment_pixels=0, segment_nodes=0):
        o = A.RenderOpts()
        o.schedule = schedule
        o.tile_band, o.segment_pixels, o.segment_nodes = tile_band, segment_pixels, segment_nodes
        o.seed = seed
        o.row_offset, o.row_stride, o.row_block = row_offset, row_stride, row_block
        o.traversal = traversal
        o.max_batch_rays = max_batch_rays
        o.collect_stats = collect_stats
        o.collect_timing = collect_timing
        o.streams = streams
        o.compact_rows = compact_rows
        o.num_devices = num_devices
        if devices is not None:
            arr = (C.c_int32 * len(devices))(*devices)
            o.devices = C.cast(arr, C.POINTER(C.c_int32))
            o._devices_keepalive = arr
        return o

    def render(self, camera: Camera | int = 0, **kw) -> np.ndarray:
        cam = self.scene.cameras[camera] if isinstance(camera, int) else camera
        o = self.opts(**kw)
        rows = (self.lib.rtg_shard_rows(cam.ny, o.row_offset, o.row_stride, o.row_block) if o.compact_rows
                else cam.ny)
        out = np.empty((rows, cam.nx, 3), np.float32)
        cd = cam.desc()
        A.check(self.lib.rtg_render(self.handle, C.byref(cd), C.byref(o), out.ctypes.data_as(A.PF)), self.lib)
        return out

    def render_device(self, camera: Camera | int, out_ptr: int, stream: int = 0, **kw):
        """Render into caller-owned device memory (e.g. a torch CUDA tensor's data_ptr)."""
        cam = self.scene.cameras[camera] if isinstance(camera, int) else camera
        cd = cam.desc()
        o = self.opts(**kw)
        A.check(self.lib.rtg_render_device(self.handle, C.byref(cd), C.byref(o), C.c_void_p(out_ptr),
                                           C.c_void_p(stream)), self.lib)

    def render_ranked(self, camera: Camera | int, comm: "Comm", frame_ptr: int, stream: int = 0, **kw):
        """One rank of a one-process-per-GPU render (rtg_render_ranked): this rank's row-block shard,
        gathered over RCCL into `frame_ptr` (device memory, rank 0; other ranks may pass 0)."""
        cam = self.scene.cameras[camera] if isinstance(camera, int) else camera
        cd = cam.desc()
        o = self.opts(**kw)
        A.check(self.lib.rtg_render_ranked(self.handle, C.byref(cd), C.byref(o), comm.handle,
                                           C.c_void_p(frame_ptr or None), C.c_void_p(stream)), self.lib)

    def stats(self) -> dict:
        s = A.RenderStats()
        A.check(self.lib.rtg_last_render_stats(self.handle, C.byref(s)), self.lib)
        return {k: (list(v) if isinstance(v, C.Array) else v)
                for k, v in ((k, getattr(s, k)) for k, _ in A.RenderStats._fields_)}

    def trace(self, origins: np.ndarray, directions: np.ndarray, times=None, traversal=0) -> dict:
        n = len(origins)
        rays = (A.Ray * max(n, 1))()
        o = np.asarray(origins, np.float32).reshape(-1, 3)
        d = np.asarray(directions, np.float32).reshape(-1, 3)
        t = np.zeros(n, np.float32) if times is None else np.asarray(times, np.float32)
        buf = np.frombuffer(rays, dtype=np.float32, count=7 * max(n, 1)).reshape(-1, 7)
        buf[:n, 0:3], buf[:n, 3:6], buf[:n, 6] = o, d, t
        hits = (A.Hit * max(n, 1))()
        A.check(self.lib.rtg_trace_closest(self.handle, rays, n, hits, traversal), self.lib)
        return hits_to_dict(hits, n)

    def build_stats(self) -> dict:
        b = A.BuildStats()
        A.check(self.lib.rtg_scene_build_stats(self.handle, C.byref(b)), self.lib)
        return {k: getattr(b, k) for k, _ in A.BuildStats._fields_}

    def bvh(self, obj: int):
        return _bvh(self.lib.rtg_scene_object_bvh, self.handle, obj)

    def matrices(self, top: int):
        inv = np.zeros(16, np.float32)
        it = np.zeros(16, np.float32)
        A.check(self.lib.rtg_scene_object_matrices(self.handle, top, inv.ctypes.data_as(A.PF),
                                                   it.ctypes.data_as(A.PF)), self.lib)
        return inv, it

    def vertex_normals(self):
        out = np.zeros((len(self.scene.vertices), 3), np.float32)
        A.check(self.lib.rtg_scene_vertex_normals(self.handle, out.ctypes.data_as(A.PF)), self.lib)
        return out


def hits_to_dict(hits, n: int) -> dict:
    raw = np.frombuffer(hits, dtype=np.int32, count=11 * max(n, 1)).reshape(-1, 11)[:n]
    f = raw.view(np.float32)
    return {"full": raw[:, 0].copy(), "object": raw[:, 1].copy(), "prim": raw[:, 2].copy(),
            "material": raw[:, 3].copy(), "t": f[:, 4].copy(), "point": f[:, 5:8].copy(),
            "normal": f[:, 8:11].copy()}


def _bvh(fn, handle, obj):
    npr, nn = C.c_int32(), C.c_int32()
    A.check(fn(handle, obj, C.byref(npr), C.byref(nn), None, None, None))
    perm = np.zeros(max(npr.value, 1), np.int32)
    nodes = np.zeros((max(nn.value, 1), 4), np.int32)
    boxes = np.zeros((max(nn.value, 1), 6), np.float32)
    A.check(fn(handle, obj, None, None, perm.ctypes.data_as(A.PI), nodes.ctypes.data_as(A.PI),
               boxes.ctypes.data_as(A.PF)))
    return perm[:npr.value], nodes[:nn.value], boxes[:nn.value]


# ---------------------------------------------------------------------------- Image
def _is_png(name: str) -> bool:
    """Image::IsPNG (src/Image.cpp:36-60): the substring ".png" anywhere in the name."""
    c = 0
    for ch in name:
        if ch == ".":
            c = 1
        elif ch == "p" and c == 1:
            c = 2
        elif ch == "n" and c == 2:
            c = 3
        elif ch == "g" and c == 3:
            return True
        else:
            c = 0
    return False


def ppm_p3_bytes(rgb: np.ndarray) -> bytes:
    """Image::SavePng (src/Image.cpp:62-103): values > 255 clamped, (unsigned char) cast,
    P3 text with a trailing space after every value and a newline per row."""
    h, w, _ = rgb.shape
    v = np.asarray(rgb, np.float32).copy()
    v[v > 255] = 255
    # (unsigned char)_data[i] (src/Image.cpp:96) as x86-64 gcc compiles it: cvttss2si to a 32-bit
    # int (truncation toward zero), low byte kept: -1 -> 255, -255.5 -> 1, -300 -> 212; NaN and
    # values below -2^31 give 0x80000000 -> 0
    ok = v >= np.float32(-2147483648.0)
    u8 = np.where(ok, np.trunc(np.where(ok, v, 0)), 0).astype(np.int64) & 0xFF
    lines = [f"P3\n{w} {h}\n255\n"]
    for y in range(h):
        lines.append(" ".join(str(int(x)) for x in u8[y].reshape(-1)) + " \n")
    return "".join(lines).encode()


def exr_half_bytes(rgb: np.ndarray) -> bytes:
    """Minimal scanline OpenEXR, ZIP compression off, HALF B/G/R channels (what
    ExrLibrary::SaveExr requests, src/Helper.cpp:361-412)."""
    h, w, _ = rgb.shape
    half = np.asarray(rgb, np.float32).astype(np.float16)

    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data

    chl = b""
    for ch in ("B", "G", "R"):
        chl += ch.encode() + b"\0" + struct.pack("<iB3xii", 1, 0, 1, 1)
    chl += b"\0"
    hdr = b"\x76\x2f\x31\x01" + struct.pack("<i", 2)
    hdr += attr("channels", "chlist", chl)
    hdr += attr("compression", "compression", b"\0")
    hdr += attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += attr("lineOrder", "lineOrder", b"\0")
    hdr += attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    hdr += attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0))
    hdr += attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    hdr += b"\0"
    table_off = len(hdr)
    line_bytes = w * 2 * 3
    first = table_off + 8 * h
    offsets = b"".join(struct.pack("<Q", first + y * (8 + line_bytes)) for y in range(h))
    body = bytearray()
    for y in range(h):
        body += struct.pack("<ii", y, line_bytes)
        for c in (2, 1, 0):
            body += half[y, :, c].astype("<f2").tobytes()
    return hdr + offsets + bytes(body)


def save_image(name: str, rgb: np.ndarray) -> str:
    """Image::saveImage (src/Image.cpp:26-34)."""
    data = ppm_p3_bytes(rgb) if _is_png(name) else exr_half_bytes(rgb)
    with open(name, "wb") as fh:
        fh.write(data)
    return name


def tonemap(img: np.ndarray, key=0.18, burn=1.0, saturation=1.0, gamma=2.2, device: int = 0) -> np.ndarray:
    """hw5 Photographic tone mapping on the GPU (rtg_tonemap): 0..255 floats."""
    lib = A.load_library()
    a = np.ascontiguousarray(img, np.float32)
    out = np.zeros_like(a)
    tm = A.TonemapDesc(A.TMO_PHOTOGRAPHIC, key, burn, saturation, gamma)
    A.check(lib.rtg_tonemap(device, a.ctypes.data_as(A.PF), a.shape[1], a.shape[0], C.byref(tm),
                            out.ctypes.data_as(A.PF)), lib)
    return out


def tonemapped_name(name: str) -> str:
    """Where a camera's tone-mapped image goes: its ImageName with the extension set to .png."""
    stem, _ = os.path.splitext(name)
    return stem + ".png"


class Comm:
    """An RCCL communicator of librtg (rtg_comm_init_rank) for rtg_render_ranked."""

    @staticmethod
    def unique_id() -> bytes:
        lib = A.load_library()
        buf = (C.c_uint8 * A.RTG_COMM_ID_BYTES)()
        A.check(lib.rtg_comm_unique_id(buf), lib)
        return bytes(buf)

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int, timeout_ms: int = 0):
        """timeout_ms bounds every wait of this rank (set-up, failure agreement, gather; the latter two
        count from this rank's shard end, so the bound must cover the peers' remaining render time); 0 = no
        deadline.  With a bound, a rank whose peers do not join returns an error instead of hanging."""
        self.lib = A.load_library()
        if len(uid) != A.RTG_COMM_ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        buf = (C.c_uint8 * A.RTG_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        A.check(self.lib.rtg_comm_init_rank_timeout(buf, int(nranks), int(rank), int(device), int(timeout_ms),
                                                    C.byref(h)), self.lib)
        self.handle = h
        self.rank, self.nranks, self.device = rank, nranks, device

    def close(self):
        if getattr(self, "handle", None):
            self.lib.rtg_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_scene(scene: Scene, out_dir: str | None = None, device: int = 0, seed: int = DEFAULT_SEED) -> list:
    """Scene::renderScene (src/Scene.cpp:294-363): every camera rendered and saved.  A camera
    with a hw5 <Tonemap> also gets its tone-mapped image (tonemapped_name; a .png ImageName is
    written tone-mapped instead of clamped)."""
    written = []
    print("BVH construction complete.")
    with Renderer(scene, device) as r:
        for cam in scene.cameras:
            img = r.render(cam, seed=seed)
            name = cam.image_name if out_dir is None else os.path.join(out_dir, os.path.basename(cam.image_name))
            tm = None if cam.tonemap is None else tonemap(img, *cam.tonemap, device=device)
            if tm is None or not _is_png(name):
                written.append(save_image(name, img))
            if tm is not None:
                written.append(save_image(tonemapped_name(name), tm))
    return written
