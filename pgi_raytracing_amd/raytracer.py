"""Python host API over libpgrt's C ABI, mirroring the reference's renderer interface.

Reference: ``class Raytracer`` (src/pg/pg1_embree/raytracer.h:15-52) with ``LoadScene``
(raytracer.cpp:48-128), ``get_pixel`` (:396-437, driven per pixel by SimpleGuiDX11::Producer,
simpleguidx11.cpp:86-128), ``gamma_level`` (:23) and ``trace``'s ray query ``get_ray_hit``
(:130-148).  Here a frame is rendered in one call on the GPU (``render``) and ``get_pixel``
reads the last frame; ``intersect`` is the batched ``rtcIntersect1``.

There is no CPU fallback: if libpgrt.so (the gfx950 HIP build) cannot be loaded, importing
this module's ``lib()`` raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import abi
from .scene import LightData, MaterialData, Scene, TextureData

_LIB = None


class PgrtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{abi.ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib():
    """Load libpgrt.so (raises if it is missing -- the product never falls back to the CPU)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(abi.LIB_PATH):
        raise ImportError(f"{abi.LIB_PATH} not built: run `make` (or __graft_entry__.build())")
    L = C.CDLL(abi.LIB_PATH)
    vp, ip, fp = C.c_void_p, C.c_int, C.POINTER(C.c_float)
    sig = {
        "pgrt_version": (C.c_char_p, []),
        "pgrt_device_count": (ip, [C.POINTER(C.c_int)]),
        "pgrt_create": (ip, [ip, C.POINTER(vp)]),
        "pgrt_create_devices": (ip, [C.POINTER(C.c_int), ip, C.POINTER(vp)]),
        "pgrt_destroy": (None, [vp]),
        "pgrt_last_error": (C.c_char_p, [vp]),
        "pgrt_get_config": (ip, [vp, C.POINTER(abi.Config)]),
        "pgrt_set_config": (ip, [vp, C.POINTER(abi.Config)]),
        "pgrt_set_scene": (ip, [vp, C.POINTER(abi.SceneDesc)]),
        "pgrt_bvh_get_info": (ip, [vp, C.POINTER(abi.BvhInfo)]),
        "pgrt_set_camera": (ip, [vp, C.POINTER(abi.Camera)]),
        "pgrt_render": (ip, [vp, C.POINTER(abi.RenderParams), fp, C.POINTER(abi.Stats)]),
        "pgrt_render_device": (ip, [vp, C.POINTER(abi.RenderParams), vp, C.POINTER(abi.Stats)]),
        "pgrt_device_alloc": (ip, [vp, C.c_size_t, C.POINTER(vp)]),
        "pgrt_device_free": (ip, [vp, vp]),
        "pgrt_copy_to_host": (ip, [vp, vp, vp, C.c_size_t]),
        "pgrt_synchronize": (ip, [vp]),
        "pgrt_intersect_closest": (ip, [vp, fp, ip, fp]),
        "pgrt_intersect_closest_soa": (ip, [vp, fp, ip, fp]),
        "pgrt_occluded": (ip, [vp, fp, ip, C.POINTER(C.c_int)]),
        "pgrt_accumulate_reset": (ip, [vp]),
        "pgrt_render_accumulate": (ip, [vp, C.POINTER(abi.RenderParams), fp, C.POINTER(C.c_int),
                                        C.POINTER(abi.Stats)]),
        "pgrt_set_frames_in_flight": (ip, [vp, ip]),
        "pgrt_render_device_async": (ip, [vp, C.POINTER(abi.RenderParams), vp, C.POINTER(C.c_ulonglong)]),
        "pgrt_render_distributed_device_async": (ip, [vp, C.POINTER(abi.RenderParams), vp,
                                                      C.POINTER(C.c_ulonglong)]),
        "pgrt_render_wait": (ip, [vp, C.c_ulonglong, C.POINTER(abi.Stats)]),
        "pgrt_render_frames_device_async": (ip, [vp, C.POINTER(abi.RenderParams), ip, vp,
                                                 C.POINTER(C.c_ulonglong)]),
        "pgrt_render_frames_device": (ip, [vp, C.POINTER(abi.RenderParams), ip, vp, C.POINTER(abi.Stats)]),
        "pgrt_render_frames_distributed_device_async": (ip, [vp, C.POINTER(abi.RenderParams), ip, vp,
                                                             C.POINTER(C.c_ulonglong)]),
        "pgrt_render_frames_host_async": (ip, [vp, C.POINTER(abi.RenderParams), ip, fp, C.POINTER(C.c_ulonglong)]),
        "pgrt_host_alloc": (ip, [vp, C.c_size_t, C.POINTER(vp)]),
        "pgrt_host_free": (ip, [vp, vp]),
        "pgrt_tile_count": (ip, [ip, ip, ip, ip, ip]),
        "pgrt_tile_index": (ip, [ip, ip, ip, ip, ip, ip]),
        "pgrt_tile_share": (ip, [ip, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "pgrt_tile_rect": (ip, [ip, ip, ip, ip, C.POINTER(C.c_int)]),
        "pgrt_unpack_tiles_host": (ip, [ip, ip, ip, ip, fp, fp]),
        "pgrt_gather_tail": (ip, [ip, ip, C.c_uint, C.POINTER(C.c_int)]),
        "pgrt_gather_tail_verdict": (ip, [C.POINTER(C.c_int), C.POINTER(C.c_uint), ip, C.c_uint, C.POINTER(C.c_int),
                                          C.POINTER(C.c_int)]),
        "pgrt_tile_count_ex": (ip, [ip, ip, ip, ip, ip, ip, ip]),
        "pgrt_tile_index_ex": (ip, [ip, ip, ip, ip, ip, ip, ip, ip]),
        "pgrt_unpack_tiles_host_ex": (ip, [ip, ip, ip, ip, ip, ip, fp, fp]),
        "pgrt_comm_unique_id": (ip, [C.c_char_p]),
        "pgrt_comm_init": (ip, [vp, ip, ip, C.c_char_p]),
        "pgrt_comm_info": (ip, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "pgrt_tune_distribution": (ip, [vp, C.POINTER(abi.RenderParams), ip, vp, ip, C.POINTER(C.c_int),
                                        C.POINTER(C.c_int)]),
        "pgrt_unpack_tiles_device": (ip, [vp, ip, ip, ip, ip, ip, vp, vp]),
        "pgrt_render_tiles_device": (ip, [vp, C.POINTER(abi.RenderParams), ip, ip, vp, C.POINTER(abi.Stats)]),
        "pgrt_render_distributed": (ip, [vp, C.POINTER(abi.RenderParams), fp, C.POINTER(abi.Stats)]),
        "pgrt_render_distributed_device": (ip, [vp, C.POINTER(abi.RenderParams), vp, C.POINTER(abi.Stats)]),
        "pgrt_obj_load": (ip, [C.c_char_p, ip, C.POINTER(vp)]),
        "pgrt_obj_free": (None, [vp]),
        "pgrt_obj_error": (C.c_char_p, []),
        "pgrt_obj_scene": (ip, [vp, C.POINTER(abi.SceneDesc)]),
        "pgrt_obj_counts": (ip, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "pgrt_obj_texture_path": (C.c_char_p, [vp, ip]),
        "pgrt_obj_material_name": (C.c_char_p, [vp, ip]),
        "pgrt_obj_surface_range": (ip, [vp, ip, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "pgrt_selftest_math": (ip, [vp, fp, ip, fp]),
        "pgrt_selftest_srgb": (ip, [vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)]),
        "pgrt_frame_diag": (ip, [vp, C.POINTER(abi.LevelDiag), ip]),
        "pgrt_timeline_enable": (ip, [vp, ip]),
        "pgrt_timeline_read": (ip, [vp, C.POINTER(abi.TimelineRec), ip, C.POINTER(C.c_int)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name, None)
        if f is None:  # an older build (PGRT_LIB A/B): calling it raises AttributeError
            continue
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def device_count() -> int:
    n = C.c_int(0)
    lib().pgrt_device_count(C.byref(n))
    return n.value


def _check(ctx, rc: int):
    if rc != abi.PGRT_OK:
        msg = lib().pgrt_last_error(ctx).decode() if ctx else ""
        raise PgrtError(rc, msg)


class Context:
    """One libpgrt context on one HIP device (one process per GPU), or with `devices` a
    single-process multi-device context (pgrt_create_devices): rank r renders its image tiles on
    devices[r], every frame is gathered on devices[0]."""

    def __init__(self, device: int = 0, devices=None):
        self.L = lib()
        h = C.c_void_p()
        if devices is not None:
            ids = (C.c_int * len(devices))(*devices)
            rc = self.L.pgrt_create_devices(ids, len(devices), C.byref(h))
            if rc != abi.PGRT_OK:
                raise PgrtError(rc, f"pgrt_create_devices({list(devices)})")
            device = devices[0]
        else:
            rc = self.L.pgrt_create(device, C.byref(h))
            if rc != abi.PGRT_OK:
                raise PgrtError(rc, f"pgrt_create(device={device})")
        self.h = h
        self.device = device
        self.scene = None
        self.camera = None

    def close(self):
        if getattr(self, "h", None):
            self.L.pgrt_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def get_config(self) -> abi.Config:
        cfg = abi.Config()
        _check(self.h, self.L.pgrt_get_config(self.h, C.byref(cfg)))
        return cfg

    def configure(self, **kw) -> abi.Config:
        """pgrt_set_config with the given fields changed (others kept); returns the previous config.
        BVH fields take effect at the next set_scene."""
        old = self.get_config()
        cfg = abi.Config.from_buffer_copy(old)
        for k, v in kw.items():
            if not hasattr(cfg, k):
                raise AttributeError(f"pgrt_config has no field {k}")
            setattr(cfg, k, v)
        _check(self.h, self.L.pgrt_set_config(self.h, C.byref(cfg)))
        return old

    def set_config(self, cfg: abi.Config):
        _check(self.h, self.L.pgrt_set_config(self.h, C.byref(cfg)))

    def set_scene(self, scene: Scene):
        d = scene.desc()
        _check(self.h, self.L.pgrt_set_scene(self.h, C.byref(d)))
        self.scene = scene

    def bvh_info(self) -> abi.BvhInfo:
        info = abi.BvhInfo()
        _check(self.h, self.L.pgrt_bvh_get_info(self.h, C.byref(info)))
        return info

    def set_camera(self, cam: abi.Camera):
        _check(self.h, self.L.pgrt_set_camera(self.h, C.byref(cam)))
        self.camera = cam

    def render(self, params: abi.RenderParams, out: np.ndarray | None = None):
        """One frame to a host framebuffer (pgrt_render); `out` (h, w, 4) float32, e.g. pinned
        memory from host_array, is written in place."""
        w = params.rect_w if params.rect_w > 0 else self.camera.width
        h = params.rect_h if params.rect_h > 0 else self.camera.height
        if out is None:
            out = np.empty((h, w, 4), np.float32)
        assert out.dtype == np.float32 and out.flags.c_contiguous and out.size == h * w * 4
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render(self.h, C.byref(params), abi.fptr(out), C.byref(st)))
        return out, st

    def render_device(self, params: abi.RenderParams, dev_ptr: int):
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render_device(self.h, C.byref(params), C.c_void_p(dev_ptr), C.byref(st)))
        return st

    def alloc(self, nbytes: int) -> int:
        p = C.c_void_p()
        _check(self.h, self.L.pgrt_device_alloc(self.h, nbytes, C.byref(p)))
        return p.value

    def free(self, ptr: int):
        _check(self.h, self.L.pgrt_device_free(self.h, C.c_void_p(ptr)))

    def host_array(self, shape) -> np.ndarray:
        """float32 array in page-locked host memory (pgrt_host_alloc); free with host_free."""
        n = int(np.prod(shape))
        p = C.c_void_p()
        _check(self.h, self.L.pgrt_host_alloc(self.h, n * 4, C.byref(p)))
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_float)), shape=(n,)).reshape(shape)

    def host_free(self, arr: np.ndarray):
        _check(self.h, self.L.pgrt_host_free(self.h, C.c_void_p(arr.ctypes.data)))

    def to_host(self, ptr: int, shape, dtype=np.float32) -> np.ndarray:
        out = np.empty(shape, dtype)
        _check(self.h, self.L.pgrt_copy_to_host(self.h, out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr),
                                                out.nbytes))
        return out

    def synchronize(self):
        _check(self.h, self.L.pgrt_synchronize(self.h))

    def intersect(self, rays: np.ndarray) -> np.ndarray:
        """rtcIntersect1 over a batch: rays (n, 8) {org, tnear, dir, tfar} -> (n, 4) {t, u, v, prim}."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        hits = np.zeros((rays.shape[0], 4), np.float32)
        _check(self.h, self.L.pgrt_intersect_closest(self.h, abi.fptr(rays), rays.shape[0], abi.fptr(hits)))
        return hits

    def intersect_soa(self, rays_soa: np.ndarray) -> np.ndarray:
        """The same query on SoA streams: rays_soa (8, n) -> hits (4, n) {t, u, v, prim bits}."""
        rays_soa = np.ascontiguousarray(rays_soa, np.float32).reshape(8, -1)
        hits = np.zeros((4, rays_soa.shape[1]), np.float32)
        _check(self.h, self.L.pgrt_intersect_closest_soa(self.h, abi.fptr(rays_soa), rays_soa.shape[1],
                                                         abi.fptr(hits)))
        return hits

    def accumulate_reset(self) -> None:
        _check(self.h, self.L.pgrt_accumulate_reset(self.h))

    def render_accumulate(self, params: abi.RenderParams):
        """One more frame into the progressive average; returns (mean image, frames in the sum)."""
        w = params.rect_w if params.rect_w > 0 else self.camera.width
        h = params.rect_h if params.rect_h > 0 else self.camera.height
        out = np.empty((h, w, 4), np.float32)
        frames = C.c_int(0)
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render_accumulate(self.h, C.byref(params), abi.fptr(out), C.byref(frames),
                                                     C.byref(st)))
        return out, frames.value

    def occluded(self, rays: np.ndarray) -> np.ndarray:
        """rtcOccluded1 over a batch: rays (n, 8) -> (n,) bool, any hit in (tnear, tfar]."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 8)
        occ = np.zeros(rays.shape[0], np.int32)
        _check(self.h, self.L.pgrt_occluded(self.h, abi.fptr(rays), rays.shape[0],
                                            occ.ctypes.data_as(C.POINTER(C.c_int))))
        return occ.astype(bool)

    def timeline_enable(self, on: bool = True):
        """pgrt_timeline_enable: every later frame's launches stamp the device clock."""
        _check(self.h, self.L.pgrt_timeline_enable(self.h, 1 if on else 0))

    def timeline_read(self) -> list:
        """pgrt_timeline_read: the launch records collected so far (and clears them), as dicts with
        us_start / us_end in microseconds of the device clock."""
        out = []
        arr = (abi.TimelineRec * 4096)()
        while True:
            n = C.c_int(0)
            _check(self.h, self.L.pgrt_timeline_read(self.h, arr, 4096, C.byref(n)))
            for i in range(n.value):
                r = arr[i]
                out.append({"ticket": int(r.ticket), "slot": r.slot, "kind": abi.TIMELINE_KINDS[r.kind]
                            if 0 <= r.kind < len(abi.TIMELINE_KINDS) else str(r.kind), "level": r.level,
                            "waves": r.waves, "start": int(r.start), "end": int(r.end),
                            "us_start": r.start / 100.0, "us_end": r.end / 100.0,
                            "wave_us": (r.wave_p50 / 100.0, r.wave_p90 / 100.0, r.wave_max / 100.0),
                            "last_in_us": r.last_in / 100.0})
            if n.value < 4096:
                return out

    def frame_diag(self) -> list:
        """Per-level counters of the last frame (traversal counts need params.profile == 2)."""
        arr = (abi.LevelDiag * 16)()
        n = self.L.pgrt_frame_diag(self.h, arr, 16)
        if n < 0:
            raise PgrtError(n, "pgrt_frame_diag")
        return [{k: (float if k.startswith("ms_") else int)(getattr(arr[i], k)) for k, _ in abi.LevelDiag._fields_}
                for i in range(n)]

    def selftest_math(self, pairs: np.ndarray) -> np.ndarray:
        pairs = np.ascontiguousarray(pairs, np.float32).reshape(-1, 2)
        out = np.zeros((pairs.shape[0], 8), np.float32)
        _check(self.h, self.L.pgrt_selftest_math(self.h, abi.fptr(pairs), pairs.shape[0], abi.fptr(out)))
        return out

    def selftest_srgb(self, first_bits: int, count: int):
        """(expand, compress) mismatches of the kernels' sRGB functions vs their exact form over the
        floats with bit patterns [first_bits, first_bits + count)."""
        m = (C.c_uint64 * 2)()
        _check(self.h, self.L.pgrt_selftest_srgb(self.h, first_bits, count, m))
        return int(m[0]), int(m[1])

    # ---- frames in flight ----
    def set_frames_in_flight(self, n: int):
        _check(self.h, self.L.pgrt_set_frames_in_flight(self.h, n))

    def render_device_async(self, params, dev_ptr: int) -> int:
        """Enqueue a frame (pgrt_render_device_async); returns its ticket."""
        t = C.c_ulonglong()
        _check(self.h, self.L.pgrt_render_device_async(self.h, C.byref(params), C.c_void_p(dev_ptr), C.byref(t)))
        return t.value

    def render_distributed_device_async(self, params, dev_ptr: int | None) -> int:
        t = C.c_ulonglong()
        _check(self.h, self.L.pgrt_render_distributed_device_async(self.h, C.byref(params), C.c_void_p(dev_ptr or 0),
                                                                   C.byref(t)))
        return t.value

    def render_frames_device_async(self, params, nframes: int, dev_ptr: int) -> int:
        """Enqueue nframes consecutive frames in one pass (pgrt_render_frames_device_async)."""
        t = C.c_ulonglong()
        _check(self.h, self.L.pgrt_render_frames_device_async(self.h, C.byref(params), nframes, C.c_void_p(dev_ptr),
                                                              C.byref(t)))
        return t.value

    def render_frames_device(self, params, nframes: int, dev_ptr: int):
        """nframes consecutive frames in one synchronous pass (pgrt_render_frames_device)."""
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render_frames_device(self.h, C.byref(params), nframes, C.c_void_p(dev_ptr),
                                                        C.byref(st)))
        return st

    def render_frames_host_async(self, params, nframes: int, out: np.ndarray) -> int:
        """Enqueue nframes frames whose pixels are copied to the host array `out` (nframes, h, w, 4)
        behind them (pgrt_render_frames_host_async); `out` must live until the ticket is waited."""
        assert out.dtype == np.float32 and out.flags.c_contiguous
        t = C.c_ulonglong()
        _check(self.h, self.L.pgrt_render_frames_host_async(self.h, C.byref(params), nframes, abi.fptr(out),
                                                            C.byref(t)))
        return t.value

    def render_frames_distributed_device_async(self, params, nframes: int, dev_ptr: int | None) -> int:
        t = C.c_ulonglong()
        _check(self.h, self.L.pgrt_render_frames_distributed_device_async(self.h, C.byref(params), nframes,
                                                                          C.c_void_p(dev_ptr or 0), C.byref(t)))
        return t.value

    def render_wait(self, ticket: int):
        """Complete the frames up to `ticket`; returns that frame's Stats."""
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render_wait(self.h, C.c_ulonglong(ticket), C.byref(st)))
        return st

    # ---- multi-GPU ----
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        rc = lib().pgrt_comm_unique_id(buf)
        if rc != abi.PGRT_OK:
            raise PgrtError(rc, "pgrt_comm_unique_id")
        return buf.raw

    def comm_init(self, world: int, rank: int, uid: bytes):
        _check(self.h, self.L.pgrt_comm_init(self.h, world, rank, C.c_char_p(uid)))

    def comm_info(self) -> tuple[int, int]:
        """(ranks, rank) of the context's RCCL communicator (ncclCommCount / ncclCommUserRank)."""
        n, r = C.c_int(), C.c_int()
        _check(self.h, self.L.pgrt_comm_info(self.h, C.byref(n), C.byref(r)))
        return n.value, r.value

    def tune_distribution(self, params, nframes: int, dev_ptr: int | None, calls: int = 4) -> tuple[int, int]:
        """Collective: pick rank 0's tile share a/b from measured distributed calls (kept in the config)."""
        a, b = C.c_int(), C.c_int()
        _check(self.h, self.L.pgrt_tune_distribution(self.h, C.byref(params), nframes, C.c_void_p(dev_ptr or 0), calls,
                                                      C.byref(a), C.byref(b)))
        return a.value, b.value

    def unpack_tiles_device(self, width: int, height: int, world: int, share, tiles_dev: int, rgba_dev: int):
        _check(self.h, self.L.pgrt_unpack_tiles_device(self.h, width, height, world, share[0], share[1],
                                                       C.c_void_p(tiles_dev), C.c_void_p(rgba_dev)))

    def render_tiles_device(self, params, rank: int, world: int, dev_ptr: int):
        """This rank's tiles into a tile-compact device buffer (pgrt_render_tiles_device)."""
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render_tiles_device(self.h, C.byref(params), rank, world, C.c_void_p(dev_ptr),
                                                       C.byref(st)))
        return st

    def render_distributed_device(self, params, dev_ptr: int | None):
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render_distributed_device(self.h, C.byref(params),
                                                             C.c_void_p(dev_ptr or 0), C.byref(st)))
        return st

    def render_distributed(self, params):
        out = np.empty((self.camera.height, self.camera.width, 4), np.float32)
        st = abi.Stats()
        _check(self.h, self.L.pgrt_render_distributed(self.h, C.byref(params), abi.fptr(out), C.byref(st)))
        return out, st


# ---------------------------------------------------------------- scene ingest (product path)

def load_obj(obj_path: str, flip_yz: bool = False) -> Scene:
    """LoadOBJ/LoadMTL (objloader.cpp:53-507) through the C++ loader in libpgrt, textures
    decoded host-side (Texture::Texture, texture.cpp:5-54)."""
    L = lib()
    h = C.c_void_p()
    rc = L.pgrt_obj_load(obj_path.encode(), int(flip_yz), C.byref(h))
    if rc != abi.PGRT_OK:
        raise PgrtError(rc, L.pgrt_obj_error().decode())
    try:
        d = abi.SceneDesc()
        L.pgrt_obj_scene(h, C.byref(d))
        n = d.num_triangles

        def arr(ptr, size, dtype):  # an OBJ without faces has no arrays at all (NULL pointers)
            return np.ctypeslib.as_array(ptr, shape=(size,)).copy() if size else np.zeros(0, dtype)

        pos = arr(d.positions, 9 * n, np.float32)
        nrm = arr(d.normals, 9 * n, np.float32)
        uv = arr(d.uvs, 6 * n, np.float32)
        mid = arr(d.material_ids, n, np.int32)
        ns, nm, nt = C.c_int(), C.c_int(), C.c_int()
        L.pgrt_obj_counts(h, C.byref(ns), C.byref(nm), C.byref(nt))
        mats = []
        for i in range(nm.value):
            m = d.materials[i]
            mats.append(MaterialData(L.pgrt_obj_material_name(h, i).decode(), tuple(m.diffuse), tuple(m.specular),
                                     m.shininess, m.ior, m.type, m.diffuse_tex))
        textures = []
        for i in range(nt.value):  # a map_Kd that does not decode fails the load (the reference reads garbage)
            path = L.pgrt_obj_texture_path(h, i).decode()
            try:
                textures.append(TextureData.from_file(path))
            except (OSError, ValueError, RuntimeError) as e:
                raise PgrtError(-7, f"texture {path}: {e}") from e
        surfaces = []
        for i in range(ns.value):
            f, c = C.c_int(), C.c_int()
            L.pgrt_obj_surface_range(h, i, C.byref(f), C.byref(c))
            surfaces.append(("", f.value, c.value))
    finally:
        L.pgrt_obj_free(h)
    return Scene(pos, nrm, uv, mid, mats, textures, -1, [LightData()], surfaces)


class Raytracer:
    """Raytracer(width, height, fov_y, view_from, view_at) (raytracer.h:18-20)."""

    def __init__(self, width: int, height: int, fov_y: float, view_from, view_at, device: int = 0):
        self.ctx = Context(device)
        self.camera = abi.make_camera(width, height, fov_y, view_from, view_at)
        self.ctx.set_camera(self.camera)
        self.gamma_level = 0.5  # UI slider default (raytracer.cpp:450,464-465)
        self.frame = None
        self.scene = None

    def LoadScene(self, object_file_name: str, background_file_name: str | None = None):  # noqa: N802
        sc = load_obj(object_file_name)
        if background_file_name:
            sc.set_environment(background_file_name)
        self.load_scene(sc)

    def load_scene(self, scene: Scene):
        self.ctx.set_scene(scene)
        self.scene = scene

    def render(self, params: abi.RenderParams | None = None, **kw):
        if params is None:
            kw.setdefault("gamma_level", self.gamma_level)
            params = abi.make_params(**kw)
        self.frame, st = self.ctx.render(params)
        return self.frame, st

    def render_progressive(self, frames: int, first_frame: int = 0, **kw):
        """Producer loop as a frame sink (simpleguidx11.cpp:86-128): `frames` renders with
        params.frame = first_frame, first_frame+1, ... averaged on the device; returns the mean."""
        kw.setdefault("gamma_level", self.gamma_level)
        self.ctx.accumulate_reset()
        mean, n = None, 0
        for f in range(first_frame, first_frame + frames):
            mean, n = self.ctx.render_accumulate(abi.make_params(frame=f, **kw))
        self.frame = mean
        return mean, n

    def get_pixel(self, x: int, y: int, t: float = 0.0):  # noqa: ARG002 (t is unused, as in the reference)
        if self.frame is None:
            self.render()
        return self.frame[y, x].copy()

    def intersect(self, rays):
        return self.ctx.intersect(rays)

    def occluded(self, rays):
        return self.ctx.occluded(rays)
