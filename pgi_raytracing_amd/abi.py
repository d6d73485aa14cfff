"""ctypes mirror of include/pgrt.h (the C ABI of libpgrt.so).

Only data layouts and the loader live here; the product entry points are wrapped in
``pgi_raytracing_amd.raytracer``.  The oracle (tests only) shares these struct layouts.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
# PGRT_LIB: development override (A/B of two builds of the library in one session)
LIB_PATH = os.environ.get("PGRT_LIB") or os.path.join(PKG_DIR, "lib", "libpgrt.so")

PGRT_OK = 0
PGRT_MATERIAL_DIELECTRIC = 4
PGRT_IOR_AIR = np.float32(1.000293)
PGRT_JITTER_NONE, PGRT_JITTER_HASH, PGRT_JITTER_HASH_CORRELATED = 0, 1, 2
PGRT_MODE_WHITTED, PGRT_MODE_PATH = 0, 1

ERRORS = {
    -1: "PGRT_ERR_INVALID_ARGUMENT",
    -2: "PGRT_ERR_HIP",
    -3: "PGRT_ERR_OUT_OF_MEMORY",
    -4: "PGRT_ERR_NO_SCENE",
    -5: "PGRT_ERR_NO_CAMERA",
    -6: "PGRT_ERR_RCCL",
    -7: "PGRT_ERR_IO",
    -8: "PGRT_ERR_NO_DEVICE",
}
globals().update({name: code for code, name in ERRORS.items()})  # PGRT_ERR_* as module constants


class Material(C.Structure):
    _fields_ = [
        ("diffuse", C.c_float * 3),
        ("specular", C.c_float * 3),
        ("shininess", C.c_float),
        ("ior", C.c_float),
        ("type", C.c_int),
        ("diffuse_tex", C.c_int),
    ]


class Texture(C.Structure):
    _fields_ = [
        ("width", C.c_int),
        ("height", C.c_int),
        ("pitch", C.c_int),
        ("bpp", C.c_int),
        ("data", C.POINTER(C.c_ubyte)),
    ]


class Light(C.Structure):
    _fields_ = [
        ("position", C.c_float * 3),
        ("diffuse", C.c_float * 3),
        ("specular", C.c_float * 3),
    ]


class SceneDesc(C.Structure):
    _fields_ = [
        ("num_triangles", C.c_int),
        ("positions", C.POINTER(C.c_float)),
        ("normals", C.POINTER(C.c_float)),
        ("uvs", C.POINTER(C.c_float)),
        ("material_ids", C.POINTER(C.c_int)),
        ("num_materials", C.c_int),
        ("materials", C.POINTER(Material)),
        ("num_textures", C.c_int),
        ("textures", C.POINTER(Texture)),
        ("env_texture", C.c_int),
        ("num_lights", C.c_int),
        ("lights", C.POINTER(Light)),
    ]


class Camera(C.Structure):
    _fields_ = [
        ("width", C.c_int),
        ("height", C.c_int),
        ("fov_y", C.c_float),
        ("from_", C.c_float * 3),
        ("at", C.c_float * 3),
        ("up", C.c_float * 3),
    ]


class RenderParams(C.Structure):
    _fields_ = [
        ("spp_side", C.c_int),
        ("max_level", C.c_int),
        ("dof", C.c_int),
        ("focal_distance", C.c_float),
        ("aperture", C.c_float),
        ("gamma_level", C.c_float),
        ("jitter", C.c_int),
        ("seed", C.c_uint32),
        ("frame", C.c_uint32),
        ("rect_x", C.c_int),
        ("rect_y", C.c_int),
        ("rect_w", C.c_int),
        ("rect_h", C.c_int),
        ("profile", C.c_int),
        ("mode", C.c_int),
    ]


PGRT_BVH_LBVH, PGRT_BVH_PLOC = 1, 2
PGRT_PACKETS_AUTO, PGRT_PACKETS_OFF = 0, -1


class Config(C.Structure):
    """pgrt_config: speed-only choices (frames are bit-identical for every value)."""
    _fields_ = [
        ("size", C.c_uint),
        ("bvh_builder", C.c_int),
        ("bvh_width", C.c_int),
        ("split_beta", C.c_float),
        ("packet_levels", C.c_int),
        ("group_max", C.c_int),
        ("max_batch_rays", C.c_longlong),
        ("max_batches_in_flight", C.c_int),
        ("rank0_share_a", C.c_int),
        ("rank0_share_b", C.c_int),
        ("packet_budget", C.c_int),
        ("subtree_level", C.c_int),
        ("call_order", C.c_int),
        ("tile_order", C.c_int),
        ("host_export", C.c_int),
        ("peer_wait_ms", C.c_int),
    ]


class Stats(C.Structure):
    _fields_ = [
        ("rays_primary", C.c_uint64),
        ("rays_shadow", C.c_uint64),
        ("rays_reflect", C.c_uint64),
        ("rays_refract", C.c_uint64),
        ("node_visits", C.c_uint64),
        ("tri_tests", C.c_uint64),
        ("ms_total", C.c_double),
        ("ms_raygen", C.c_double),
        ("ms_trace", C.c_double),
        ("ms_shade", C.c_double),
        ("ms_shadow", C.c_double),
        ("ms_combine", C.c_double),
        ("ms_resolve", C.c_double),
        ("ms_gather", C.c_double),
        ("trace_launches", C.c_int),
        ("levels", C.c_int),
        ("overflow_retries", C.c_int),
        ("wide_node_visits", C.c_uint64),
        ("shade_hits", C.c_uint64),
        ("shade_textured_hits", C.c_uint64),
    ]

    def rays(self) -> int:
        return int(self.rays_primary + self.rays_shadow + self.rays_reflect + self.rays_refract)

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class LevelDiag(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("rays", "shadow_rays", "visits", "tests", "max_visits", "max_tests",
                                          "shadow_visits", "shadow_tests", "shadow_max_visits", "shadow_max_tests",
                                          "max_wave_iterations", "max_ray_ticks", "stack_spills", "max_stack",
                                          "lr_visits", "lr_tests", "lr_leaves", "lr_node_cyc64", "lr_leaf_cyc64",
                                          "lr_load_cyc64", "wide_visits")] + [("ms_trace", C.c_double), ("ms_shade", C.c_double),
                                                                  ("packet_steps_hit", C.c_uint64),
                                                                  ("packet_steps_live", C.c_uint64)]


TIMELINE_KINDS = ("raygen", "trace_pkt", "trace", "trace_8g", "trace_resume", "trace_shadow", "shade", "combine",
                  "finish", "export", "unpack", "path_shade", "path_resolve", "subtree", "host_export", "dropped")  # PGRT_TL_*


class TimelineRec(C.Structure):
    """pgrt_timeline_rec: one launch, device wall clock (100 MHz ticks)."""
    _fields_ = [
        ("ticket", C.c_uint64),
        ("slot", C.c_int),
        ("kind", C.c_int),
        ("level", C.c_int),
        ("waves", C.c_int),
        ("start", C.c_uint64),
        ("end", C.c_uint64),
        ("wave_p50", C.c_uint32),
        ("wave_p90", C.c_uint32),
        ("wave_max", C.c_uint32),
        ("last_in", C.c_uint32),
    ]


class BvhInfo(C.Structure):
    _fields_ = [
        ("num_triangles", C.c_int),
        ("num_nodes", C.c_int),
        ("max_depth", C.c_int),
        ("build_ms", C.c_double),
        ("scene_lo", C.c_float * 3),
        ("scene_hi", C.c_float * 3),
        ("device_bytes", C.c_size_t),
        ("builder", C.c_int),
        ("build_iterations", C.c_int),
        ("width", C.c_int),
        ("num_references", C.c_int),
        ("split_beta", C.c_float),
    ]


def fptr(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_float))


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_int))


def make_params(spp_side=1, max_level=5, dof=0, focal_distance=200.0, aperture=5.0, gamma_level=0.5,
                jitter=PGRT_JITTER_NONE, seed=1234, frame=0, rect=(0, 0, 0, 0), profile=0,
                mode=PGRT_MODE_WHITTED) -> RenderParams:
    p = RenderParams()
    p.spp_side = spp_side
    p.max_level = max_level
    p.dof = dof
    p.focal_distance = focal_distance
    p.aperture = aperture
    p.gamma_level = gamma_level
    p.jitter = jitter
    p.seed = seed
    p.frame = frame
    p.rect_x, p.rect_y, p.rect_w, p.rect_h = rect
    p.profile = profile
    p.mode = mode
    return p


def make_camera(width, height, fov_y, view_from, view_at, up=(0.0, 0.0, 1.0)) -> Camera:
    c = Camera()
    c.width = width
    c.height = height
    c.fov_y = fov_y
    for i in range(3):
        c.from_[i] = view_from[i]
        c.at[i] = view_at[i]
        c.up[i] = up[i]
    return c


def deg2rad(x: float) -> float:
    """mymath.h:27-30 -- x * float(M_PI) / 180.0f evaluated in float32."""
    return float(np.float32(x) * np.float32(np.pi) / np.float32(180.0))


def default_camera(width=640, height=480) -> Camera:
    """raytrace_loop's camera (tutorials.cpp:186-191)."""
    return make_camera(width, height, deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 40.0))
