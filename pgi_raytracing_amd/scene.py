"""Host-side scene container (setup for the trace path, not part of the hot loop).

``Scene`` owns the de-indexed triangle arrays, materials, decoded textures and lights and
builds the ``pgrt_scene_desc`` handed to libpgrt (and, in tests only, to the oracle).
It mirrors what Raytracer::LoadScene assembles (raytracer.cpp:48-128): surfaces from
LoadOBJ, SphericalMap(background), one white light at (-500,-100,500).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from . import abi


def freeimage_pitch(width: int, bpp: int) -> int:
    """FreeImage_GetPitch: row bytes rounded up to a 32-bit boundary."""
    return ((width * bpp * 8 + 31) // 32) * 4


_JPEG = None


def _jpeg_lib():
    """libpgrt_image.so (csrc/image_jpeg.c): IJG libjpeg 9 with FreeImage's JPEG_DEFAULT load
    settings (IFAST IDCT, no fancy upsampling)."""
    global _JPEG
    if _JPEG is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libpgrt_image.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: build it with `make` (JPEG textures are decoded like "
                               "FreeImage's JPEG_DEFAULT load, texture.cpp:5-54)")
        lib = C.CDLL(path)
        lib.pgrt_jpeg_decode.argtypes = [C.c_char_p, C.c_int] + [C.POINTER(C.c_int)] * 4 + [C.c_void_p, C.c_size_t]
        lib.pgrt_jpeg_decode.restype = C.c_int
        lib.pgrt_jpeg_error.restype = C.c_char_p
        lib.pgrt_png_decode.argtypes = [C.c_char_p] + [C.POINTER(C.c_int)] * 4 + [C.c_void_p, C.c_size_t]
        lib.pgrt_png_decode.restype = C.c_int
        lib.pgrt_png_error.restype = C.c_char_p
        _JPEG = lib
    return _JPEG


def decode_jpeg(path: str, accurate: bool = False):
    """(width, height, bpp, pitch, bytes): BGR, top-down, FreeImage pitch.  accurate=False is
    FreeImage's JPEG_DEFAULT (IFAST); True its JPEG_ACCURATE (ISLOW + fancy upsampling)."""
    lib = _jpeg_lib()
    w, h, b, p = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    args = (path.encode(), 1 if accurate else 0, C.byref(w), C.byref(h), C.byref(b), C.byref(p))
    if lib.pgrt_jpeg_decode(*args, None, 0) != 0:
        raise RuntimeError(lib.pgrt_jpeg_error().decode())
    buf = np.zeros(p.value * h.value, np.uint8)
    if lib.pgrt_jpeg_decode(*args, buf.ctypes.data, buf.size) != 0:
        raise RuntimeError(lib.pgrt_jpeg_error().decode())
    return w.value, h.value, b.value, p.value, buf


def decode_png(path: str):
    """(width, height, bpp, pitch, bytes): BGR(A), top-down, FreeImage pitch (libpgrt_image.so's
    libpng decode, csrc/image_png.c; lossless, so FreeImage's bytes)."""
    lib = _jpeg_lib()
    w, h, b, p = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    args = (path.encode(), C.byref(w), C.byref(h), C.byref(b), C.byref(p))
    if lib.pgrt_png_decode(*args, None, 0) != 0:
        raise RuntimeError(lib.pgrt_png_error().decode())
    buf = np.zeros(p.value * h.value, np.uint8)
    if lib.pgrt_png_decode(*args, buf.ctypes.data, buf.size) != 0:
        raise RuntimeError(lib.pgrt_png_error().decode())
    return w.value, h.value, b.value, p.value, buf


@dataclass
class TextureData:
    """Texture::Texture (texture.cpp:5-54): raw BGR(A), top-down, FreeImage pitch.

    JPEG: FreeImage_Load with flags 0 = JPEG_DEFAULT (FreeImage.h:693-695), i.e. IJG libjpeg's
    fast integer IDCT without fancy upsampling (decode_jpeg, libpgrt_image.so).  PNG: libpng
    (decode_png, the same library; lossless, so the bytes are FreeImage's)."""

    width: int
    height: int
    pitch: int
    bpp: int
    data: np.ndarray  # uint8, pitch*height
    name: str = ""

    @staticmethod
    def from_file(path: str) -> "TextureData":
        with open(path, "rb") as fh:  # FreeImage_GetFileType: the signature decides (texture.cpp:15)
            sig = fh.read(8)
        jpeg = sig[:3] == b"\xff\xd8\xff" or (sig[:8] != b"\x89PNG\r\n\x1a\n"
                                               and path.lower().endswith((".jpg", ".jpeg", ".jpe")))
        w, h, bpp, pitch, buf = decode_jpeg(path) if jpeg else decode_png(path)
        return TextureData(w, h, pitch, bpp, buf, os.path.basename(path))

    @staticmethod
    def from_bgr(bgr: np.ndarray, name: str = "") -> "TextureData":
        h, w, ch = bgr.shape
        pitch = freeimage_pitch(w, ch)
        buf = np.zeros((h, pitch), np.uint8)
        buf[:, : w * ch] = bgr.reshape(h, w * ch)
        return TextureData(w, h, pitch, ch, np.ascontiguousarray(buf.reshape(-1)), name)

    def to_c(self) -> abi.Texture:
        t = abi.Texture()
        t.width, t.height, t.pitch, t.bpp = self.width, self.height, self.pitch, self.bpp
        t.data = self.data.ctypes.data_as(C.POINTER(C.c_ubyte))
        return t


@dataclass
class MaterialData:
    name: str = "default"
    diffuse: tuple = (0.4, 0.4, 0.4)   # material.cpp:11-14 defaults
    specular: tuple = (0.8, 0.8, 0.8)
    shininess: float = 1.0
    ior: float = 1.5
    type: int = 0                      # uninitialised in the reference; 0 -> Phong
    diffuse_tex: int = -1

    def to_c(self) -> abi.Material:
        m = abi.Material()
        for i in range(3):
            m.diffuse[i] = self.diffuse[i]
            m.specular[i] = self.specular[i]
        m.shininess = self.shininess
        m.ior = self.ior
        m.type = self.type
        m.diffuse_tex = self.diffuse_tex
        return m


@dataclass
class LightData:
    position: tuple = (-500.0, -100.0, 500.0)  # raytracer.cpp:66-68
    diffuse: tuple = (1.0, 1.0, 1.0)
    specular: tuple = (1.0, 1.0, 1.0)

    def to_c(self) -> abi.Light:
        l = abi.Light()
        for i in range(3):
            l.position[i] = self.position[i]
            l.diffuse[i] = self.diffuse[i]
            l.specular[i] = self.specular[i]
        return l


@dataclass
class Scene:
    positions: np.ndarray            # float32 9N
    normals: np.ndarray              # float32 9N
    uvs: np.ndarray                  # float32 6N
    material_ids: np.ndarray         # int32 N
    materials: list = field(default_factory=list)
    textures: list = field(default_factory=list)
    env_texture: int = -1
    lights: list = field(default_factory=lambda: [LightData()])
    surfaces: list = field(default_factory=list)  # (name, first_triangle, count)
    _keep: list = field(default_factory=list, repr=False)

    @property
    def num_triangles(self) -> int:
        return int(self.material_ids.shape[0])

    def set_environment(self, path_or_tex) -> None:
        tex = path_or_tex if isinstance(path_or_tex, TextureData) else TextureData.from_file(path_or_tex)
        self.textures.append(tex)
        self.env_texture = len(self.textures) - 1

    def desc(self) -> abi.SceneDesc:
        for name in ("positions", "normals", "uvs"):
            a = getattr(self, name)
            setattr(self, name, np.ascontiguousarray(a, dtype=np.float32))
        self.material_ids = np.ascontiguousarray(self.material_ids, dtype=np.int32)
        n = self.num_triangles
        assert self.positions.size == 9 * n and self.normals.size == 9 * n and self.uvs.size == 6 * n
        mats = (abi.Material * max(1, len(self.materials)))(*[m.to_c() for m in self.materials])
        texs = (abi.Texture * max(1, len(self.textures)))(*[t.to_c() for t in self.textures])
        lights = (abi.Light * max(1, len(self.lights)))(*[l.to_c() for l in self.lights])
        d = abi.SceneDesc()
        d.num_triangles = n
        d.positions = abi.fptr(self.positions)
        d.normals = abi.fptr(self.normals)
        d.uvs = abi.fptr(self.uvs)
        d.material_ids = abi.iptr(self.material_ids)
        d.num_materials = len(self.materials)
        d.materials = C.cast(mats, C.POINTER(abi.Material))
        d.num_textures = len(self.textures)
        d.textures = C.cast(texs, C.POINTER(abi.Texture))
        d.env_texture = self.env_texture
        d.num_lights = len(self.lights)
        d.lights = C.cast(lights, C.POINTER(abi.Light))
        self._keep = [mats, texs, lights]
        return d


def single_triangle_scene() -> Scene:
    """tutorial_1's triangle (tutorials.cpp:29-80): (0,0,0),(2,0,0),(0,3,0), normals +z,
    UVs (0,1),(1,1),(0,0)."""
    pos = np.array([0, 0, 0, 2, 0, 0, 0, 3, 0], np.float32)
    nrm = np.array([0, 0, 1, 0, 0, 1, 0, 0, 1], np.float32)
    uv = np.array([0, 1, 1, 1, 0, 0], np.float32)
    return Scene(pos, nrm, uv, np.zeros(1, np.int32), [MaterialData()], [], -1, [LightData()])


def random_soup_scene(n=1_000_000, seed=42) -> Scene:
    """BASELINE C5 scene (tools/scenes.py random_triangles)."""
    import sys

    sys.path.insert(0, os.path.join(abi.ROOT, "tools"))
    from scenes import random_triangles

    p, nrm, uv, mids, mats = random_triangles(n, seed)
    mds = [MaterialData(f"m{i}", tuple(map(float, m["diffuse"])), tuple(m["specular"]), m["shininess"],
                        m["ior"], m["type"], -1) for i, m in enumerate(mats)]
    return Scene(p, nrm, uv, mids, mds, [], -1, [LightData()])
