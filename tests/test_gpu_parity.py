"""GPU parity: libpgrt's HIP path (through the C ABI) against the CPU restatement (oracle).

Bar: RGBA after gamma within 1e-4 of the oracle, NaN at the same places.
Integer/index results (hit primitive ids) must be bit-exact.  GPU and oracle share the float
operation order and pgrt_detmath.h, so in practice every pixel is bit-identical; the tests
report the exact-match fraction and require it to be 1 for the hit records.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from conftest import assert_frames_match
from pgi_raytracing_amd import abi
from pgi_raytracing_amd.scene import LightData, single_triangle_scene

pytestmark = pytest.mark.gpu

FLT_MIN = np.float32(1.17549435e-38)
FLT_MAX = np.float32(3.402823466e38)


def _oracle(scene, cache={}):  # noqa: B006 (per-session cache keyed by scene id)
    k = id(scene)
    if k not in cache:
        cache[k] = (scene, pyoracle.OracleScene(scene, accel=1))
    return cache[k][1]


def test_device_math_bit_exact(gpu_ctx):
    rng = np.random.default_rng(7)
    a = np.concatenate([rng.uniform(0, 2, 4000), rng.uniform(-1, 1, 2000), rng.uniform(0, 1e-3, 500),
                        np.array([0.0, -0.0, 1.0, 0.5, 1e-38, 3e38])]).astype(np.float32)
    b = np.concatenate([rng.uniform(-3, 40, 4000), rng.uniform(0.1, 3, 2000), rng.uniform(1, 2, 500),
                        np.array([2.0, 3.0, 0.0, 32.0, 2.4, 0.5])]).astype(np.float32)
    # k_finish's gamma fast path (column 2 is gamma_pow == pg_powf): y = 0.5 on special and random x
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, -1.0, 1.0, 1e-45, 3.4e38], np.float32)
    a = np.concatenate([a, sp, rng.uniform(0, 4, 1000).astype(np.float32)]).astype(np.float32)
    b = np.concatenate([b, np.full(len(sp) + 1000, 0.5, np.float32)]).astype(np.float32)
    pairs = np.stack([a, b], 1)
    dev = gpu_ctx.selftest_math(pairs)
    host = np.zeros_like(dev)
    pyoracle.lib().orc_detmath_eval(abi.fptr(np.ascontiguousarray(pairs.reshape(-1))), pairs.shape[0],
                                    abi.fptr(host.reshape(-1)))
    same = (dev.view(np.uint32) == host.view(np.uint32)) | (np.isnan(dev) & np.isnan(host))
    bad = np.argwhere(~same)
    assert same.all(), f"{len(bad)} mismatches, first {bad[:5]}: dev {dev[tuple(bad[0])]} host {host[tuple(bad[0])]}"


def test_env_angles_fast_path_bit_exact(gpu_ctx):
    """The env-map lookup's atan2f / asinf (columns 4, 5: a double-precision approximation with
    Ziv's rounding test, the exact pgrt_detmath.h function when undecided) equal the host's exact
    functions bit for bit on 4M unit-vector-like arguments -- about 3e-5 of them take the exact
    fallback, so both branches run -- plus signed zeros, tiny, huge and near-1 values."""
    rng = np.random.default_rng(11)
    v = rng.normal(size=(1 << 22, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    a = v[:, 0].astype(np.float32)
    b = v[:, 2].astype(np.float32)
    edge = np.array([0.0, -0.0, 1e-31, -1e-31, 1e-20, 0.9998999, 0.9999, -0.9999001, 1.0, -1.0, 1e31, 3e38,
                     np.inf, -np.inf, np.nan, 0.5, -0.5], np.float32)
    ea, eb = np.meshgrid(edge, edge)
    pairs = np.ascontiguousarray(np.stack([np.concatenate([a, ea.ravel()]), np.concatenate([b, eb.ravel()])], 1))
    dev = gpu_ctx.selftest_math(pairs)[:, 4:6]
    host = np.zeros((pairs.shape[0], 8), np.float32)
    pyoracle.lib().orc_detmath_eval(abi.fptr(pairs.reshape(-1)), pairs.shape[0], abi.fptr(host.reshape(-1)))
    host = host[:, 4:6]
    same = (dev.view(np.uint32) == host.view(np.uint32)) | (np.isnan(dev) & np.isnan(host))
    bad = np.argwhere(~same)
    assert same.all(), f"{len(bad)} mismatches, first {bad[:5]}: pairs {pairs[bad[:5, 0]]}"


def test_srgb_fast_path_exhaustive(gpu_ctx):
    """The kernels' sRGB expand / compress (mix_srgb: a float exp2(log2) estimate, two Newton steps
    in double, Ziv's rounding test with the exact pg_pow_d form as fallback) equal the exact form
    bit for bit on EVERY float in [0, 1] (bit patterns 0 .. 0x3f800000, ~1.07e9 inputs each) and
    on a band above 1 -- the proof that the fast path cannot change a pixel."""
    end = 0x3F800000 + (1 << 20)
    first = 0
    while first < end:
        n = min(1 << 28, end - first)
        me, mc = gpu_ctx.selftest_srgb(first, n)
        assert (me, mc) == (0, 0), f"bits [{first:#x}, {first + n:#x}): {me} expand, {mc} compress mismatches"
        first += n


def test_tutorial1_kat_on_gpu(gpu_ctx):
    gpu_ctx.set_scene(single_triangle_scene())
    ray = np.array([0.1, 0.2, 2.0, FLT_MIN, 0.0, 0.0, -1.0, FLT_MAX], np.float32)
    t, u, v, prim = gpu_ctx.intersect(ray)[0]
    assert prim.view(np.int32) == 0 and t == np.float32(2.0)
    assert f"{u:0.3f}" == "0.050" and abs(v - 1 / 15) < 1e-6


def _random_rays(scene, n, seed):
    rng = np.random.default_rng(seed)
    lo = np.array([-150, -150, -50], np.float32)
    hi = np.array([150, 150, 150], np.float32)
    org = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r1 = np.concatenate([org, np.full((n, 1), 0.01, np.float32), d, np.full((n, 1), FLT_MAX, np.float32)], 1)
    p = scene.positions.reshape(-1, 3, 3)
    m = n // 4
    idx = rng.integers(0, p.shape[0], size=m)
    w = rng.uniform(0, 1, size=(m, 1)).astype(np.float32)
    target = w * p[idx, 0] + (1 - w) * p[idx, 1]  # points on triangle edges (ties, grazing)
    o2 = np.array([-140, -175, 80], np.float32) + rng.normal(size=(m, 3)).astype(np.float32)
    r2 = np.concatenate([o2, np.full((m, 1), 0.001, np.float32), (target - o2).astype(np.float32),
                         np.full((m, 1), FLT_MAX, np.float32)], 1)
    # shadow-style rays: from the light along hit-position vectors, finite tfar
    r3 = r2.copy()
    r3[:, 0:3] = np.array([-500, -100, 500], np.float32)
    r3[:, 4:7] = target
    r3[:, 7] = np.linalg.norm(r3[:, 0:3] - target, axis=1)
    return np.concatenate([r1, r2, r3]).astype(np.float32)


def test_closest_hit_bit_exact_vs_oracle(gpu_ctx, avenger_scene):
    gpu_ctx.set_scene(avenger_scene)
    info = gpu_ctx.bvh_info()
    assert info.num_triangles == avenger_scene.num_triangles and info.max_depth > 0
    rays = _random_rays(avenger_scene, 40000, 3)
    hg = gpu_ctx.intersect(rays)
    ho = _oracle(avenger_scene).intersect(rays)
    eq = (hg.view(np.int32) == ho.view(np.int32)).all(1)
    assert eq.all(), f"{(~eq).sum()} / {len(eq)} hit records differ, e.g. {np.argwhere(~eq)[:3].ravel()}"
    assert (hg[:, 3].view(np.int32) >= 0).sum() > 10000


def test_soa_query_equals_aos(gpu_ctx, avenger_scene):
    """pgrt_intersect_closest_soa (SURVEY 8b's SoA streams) returns the AoS query's hit records."""
    gpu_ctx.set_scene(avenger_scene)
    rays = _random_rays(avenger_scene, 8000, 9)
    aos = gpu_ctx.intersect(rays)
    soa = gpu_ctx.intersect_soa(np.ascontiguousarray(rays.T))
    assert (soa.T.view(np.int32) == aos.view(np.int32)).all()


CONFIGS = [
    dict(spp_side=1, max_level=1),
    dict(spp_side=1, max_level=5),
    dict(spp_side=1, max_level=7),
    dict(spp_side=2, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH),
    dict(spp_side=3, max_level=7, dof=1, jitter=abi.PGRT_JITTER_HASH_CORRELATED, seed=99, frame=3),
    dict(spp_side=2, max_level=0, jitter=abi.PGRT_JITTER_HASH, gamma_level=0.45),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "-".join(f"{k}{v}" for k, v in c.items()))
def test_avenger_frame_parity(gpu_ctx, avenger_scene, cfg):
    gpu_ctx.set_scene(avenger_scene)
    cam = abi.default_camera(128, 96)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(**cfg)
    ref, sto = _oracle(avenger_scene).render(cam, p)
    # default (one-frame batches: levels >= 3 as whole ray trees) and one launch per level
    for sub in (0, -1):
        old = gpu_ctx.configure(subtree_level=sub)
        try:
            img, st = gpu_ctx.render(p)
        finally:
            gpu_ctx.set_config(old)
        diff, exact = assert_frames_match(img, ref)
        assert exact == 1.0, f"subtree_level {sub}: max diff {diff}, exact fraction {exact}"
        assert (st.rays_primary, st.rays_shadow, st.rays_reflect, st.rays_refract) == \
            (sto.rays_primary, sto.rays_shadow, sto.rays_reflect, sto.rays_refract)


@pytest.mark.parametrize("cfg", CONFIGS[1:3] + CONFIGS[4:5], ids=["d5", "d7", "S3d7dof"])
def test_geosphere_glass_parity(gpu_ctx, geosphere_scene, cfg):
    """All-glass icosphere (geosphere.mtl, shader 4): deep refraction trees, TIR, queue growth."""
    gpu_ctx.set_scene(geosphere_scene)
    cam = abi.make_camera(96, 72, abi.deg2rad(90.0), (2.0, 0.0, 0.0), (0.0, 0.0, 0.0))  # tutorials.cpp:194
    gpu_ctx.set_camera(cam)
    p = abi.make_params(**cfg)
    img, st = gpu_ctx.render(p)
    ref, sto = _oracle(geosphere_scene).render(cam, p)
    diff, exact = assert_frames_match(img, ref)
    assert exact == 1.0
    assert st.rays_refract == sto.rays_refract > 0


def test_empty_scene_renders_environment(gpu_ctx, avenger_scene):
    """A scene without triangles (an OBJ with no faces: Embree commits it, every rtcIntersect1
    misses) renders the environment map in every pixel, Whitted and path mode, bit-exact with the
    oracle's empty scene; the closest-hit query reports misses; no material is required."""
    from pgi_raytracing_amd.scene import Scene

    env = avenger_scene.textures[avenger_scene.env_texture]
    sc = Scene(np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.int32),
               [], [env], 0, [LightData()])
    gpu_ctx.set_scene(sc)
    assert gpu_ctx.bvh_info().num_triangles == 0
    cam = abi.default_camera(90, 60)
    gpu_ctx.set_camera(cam)
    orc = pyoracle.OracleScene(sc, accel=1)
    for p in (abi.make_params(max_level=5), abi.make_params(spp_side=2, max_level=3, dof=1, jitter=abi.PGRT_JITTER_HASH),
              abi.make_params(max_level=5, mode=abi.PGRT_MODE_PATH)):
        img, st = gpu_ctx.render(p)
        ref, sto = orc.render(cam, p)
        _, exact = assert_frames_match(img, ref)
        assert exact == 1.0
        assert st.rays_primary == sto.rays_primary and st.rays_shadow == 0 and st.rays_reflect == 0
    hits = gpu_ctx.intersect(_random_rays(avenger_scene, 1000, 5))
    assert (hits[:, 3].view(np.int32) == -1).all()


@pytest.mark.parametrize("wh", [(1, 1), (65, 1), (1, 70), (129, 3)])
def test_degenerate_image_sizes(gpu_ctx, avenger_scene, wh):
    """Single-pixel, single-row and single-column images (ragged 64x64 tiles of one pixel's
    width): bit-exact with the oracle, synchronous and batched."""
    W, H = wh
    gpu_ctx.set_scene(avenger_scene)
    cam = abi.make_camera(W, H, abi.deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 40.0))
    gpu_ctx.set_camera(cam)
    p = abi.make_params(spp_side=2, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH)
    img, st = gpu_ctx.render(p)
    ref, sto = _oracle(avenger_scene).render(cam, p)
    _, exact = assert_frames_match(img, ref)
    assert exact == 1.0 and st.rays_primary == sto.rays_primary == 4 * W * H
    buf = gpu_ctx.alloc(3 * W * H * 16)
    try:
        gpu_ctx.render_frames_device(p, 3, buf)
        out = gpu_ctx.to_host(buf, (3, H, W, 4))
        same = (out[0] == img) | (np.isnan(out[0]) & np.isnan(img))
        assert same.all()
    finally:
        gpu_ctx.free(buf)


def test_maximum_depth_and_samples(gpu_ctx, avenger_scene, geosphere_scene):
    """The largest parameters pgrt_render_params accepts: max_level 14 (kMaxLevels - 2) on the
    all-glass geosphere (refraction trees as deep as the queues allow, re-grown on overflow) and
    spp_side 64 (4096 samples per pixel, many sample batches) on a few pixels -- bit-exact with
    the oracle."""
    gpu_ctx.set_scene(geosphere_scene)
    cam = abi.make_camera(48, 36, abi.deg2rad(90.0), (2.0, 0.0, 0.0), (0.0, 0.0, 0.0))
    gpu_ctx.set_camera(cam)
    p = abi.make_params(spp_side=2, max_level=14, jitter=abi.PGRT_JITTER_HASH)
    img, st = gpu_ctx.render(p)
    ref, sto = _oracle(geosphere_scene).render(cam, p)
    _, exact = assert_frames_match(img, ref)
    assert exact == 1.0 and st.levels == 15
    assert (st.rays_reflect, st.rays_refract) == (sto.rays_reflect, sto.rays_refract)
    gpu_ctx.set_scene(avenger_scene)
    cam = abi.default_camera(8, 4)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(spp_side=64, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH)
    img, st = gpu_ctx.render(p)
    ref, sto = _oracle(avenger_scene).render(cam, p)
    _, exact = assert_frames_match(img, ref)
    assert exact == 1.0 and st.rays_primary == sto.rays_primary == 4096 * 32


def test_rect_render_equals_crop(gpu_ctx, avenger_scene):
    gpu_ctx.set_scene(avenger_scene)
    cam = abi.default_camera(200, 150)
    gpu_ctx.set_camera(cam)
    full, _ = gpu_ctx.render(abi.make_params(max_level=5))
    sub, _ = gpu_ctx.render(abi.make_params(max_level=5, rect=(37, 21, 101, 70)))
    assert (np.nan_to_num(sub, nan=9) == np.nan_to_num(full[21:91, 37:138], nan=9)).all()


def test_scene_without_env_and_lights(gpu_ctx, avenger_scene):
    from pgi_raytracing_amd.scene import Scene

    sc = Scene(avenger_scene.positions, avenger_scene.normals, avenger_scene.uvs, avenger_scene.material_ids,
               avenger_scene.materials, avenger_scene.textures[:2], -1, [])
    gpu_ctx.set_scene(sc)
    cam = abi.default_camera(64, 48)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(max_level=3)
    img, st = gpu_ctx.render(p)
    ref, _ = pyoracle.OracleScene(sc).render(cam, p)
    assert_frames_match(img, ref)
    assert st.rays_shadow == 0


def test_multiple_lights(gpu_ctx, avenger_scene):
    from pgi_raytracing_amd.scene import Scene

    lights = [LightData((-500.0, -100.0, 500.0)), LightData((300.0, -400.0, 200.0), (0.8, 0.2, 0.2), (0.8, 0.2, 0.2)),
              LightData((0.0, 0.0, -300.0), (0.2, 0.2, 0.8), (0.2, 0.8, 0.2))]
    sc = Scene(avenger_scene.positions, avenger_scene.normals, avenger_scene.uvs, avenger_scene.material_ids,
               avenger_scene.materials, avenger_scene.textures, avenger_scene.env_texture, lights)
    gpu_ctx.set_scene(sc)
    cam = abi.default_camera(80, 60)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(max_level=5)
    img, st = gpu_ctx.render(p)
    ref, sto = pyoracle.OracleScene(sc).render(cam, p)
    _, exact = assert_frames_match(img, ref)
    assert exact == 1.0 and st.rays_shadow == sto.rays_shadow


def test_distributed_world1_equals_render(gpu_ctx, avenger_scene):
    gpu_ctx.set_scene(avenger_scene)
    cam = abi.default_camera(150, 100)
    gpu_ctx.set_camera(cam)
    uid = gpu_ctx.comm_unique_id()
    gpu_ctx.comm_init(1, 0, uid)
    p = abi.make_params(max_level=5, spp_side=2, jitter=abi.PGRT_JITTER_HASH)
    a, _ = gpu_ctx.render(p)
    b, _ = gpu_ctx.render_distributed(p)
    assert (np.nan_to_num(a, nan=5) == np.nan_to_num(b, nan=5)).all()
    # batched frames through the RCCL gather: one ncclGather for all frames of the call
    F = 3
    refs = [gpu_ctx.render(abi.make_params(max_level=5, spp_side=2, jitter=abi.PGRT_JITTER_HASH, frame=4 + f))[0]
            for f in range(F)]
    buf = gpu_ctx.alloc(F * 150 * 100 * 16)
    try:
        gpu_ctx.set_frames_in_flight(2)
        q = abi.make_params(max_level=5, spp_side=2, jitter=abi.PGRT_JITTER_HASH, frame=4)
        gpu_ctx.render_wait(gpu_ctx.render_frames_distributed_device_async(q, F, buf))
        out = gpu_ctx.to_host(buf, (F, 100, 150, 4))
        for f in range(F):
            assert (np.nan_to_num(out[f], nan=5) == np.nan_to_num(refs[f], nan=5)).all(), f"frame {f}"
    finally:
        gpu_ctx.set_frames_in_flight(1)
        gpu_ctx.free(buf)
    # distributed calls in flight that reuse frame sets: a set's next frame waits for its own gather
    # only (not for the gathers of the calls submitted after it), and every frame still lands intact
    calls, F2 = 7, 2
    refs = [gpu_ctx.render(abi.make_params(max_level=5, spp_side=1, jitter=abi.PGRT_JITTER_HASH, frame=f))[0]
            for f in range(calls * F2)]
    bufs = [gpu_ctx.alloc(F2 * 150 * 100 * 16) for _ in range(calls)]
    try:
        gpu_ctx.set_frames_in_flight(3)
        pend = []

        def check(c, t):
            gpu_ctx.render_wait(t)
            out = gpu_ctx.to_host(bufs[c], (F2, 100, 150, 4))
            for f in range(F2):
                ref = refs[c * F2 + f]
                assert (np.nan_to_num(out[f], nan=5) == np.nan_to_num(ref, nan=5)).all(), f"call {c} frame {f}"

        for c in range(calls):
            if len(pend) == 3:
                check(*pend.pop(0))
            q = abi.make_params(max_level=5, spp_side=1, jitter=abi.PGRT_JITTER_HASH, frame=c * F2)
            pend.append((c, gpu_ctx.render_frames_distributed_device_async(q, F2, bufs[c])))
        for c, t in pend:
            check(c, t)
    finally:
        gpu_ctx.set_frames_in_flight(1)
        for b in bufs:
            gpu_ctx.free(b)


@pytest.mark.parametrize("ranks", [1, 2, 3, 8])
def test_multi_device_context_equals_render(gpu_ctx, avenger_scene, ranks):
    """pgrt_create_devices (SURVEY 8b's single-process multi-device context).  One device: its
    own RCCL communicator from ncclCommInitAll (the RCCL path at world 1).  Several ranks listed
    on this one GPU (the pool has one GPU per box): every rank renders its tile deal on its own
    streams and rank 0 gathers by device copies -- the single-thread submission, the grouped
    gather, the lockstep frame sets and the host overflow agreement at world > 1.  Frames are
    bit-identical to one context's render, synchronous, batched and in flight."""
    from pgi_raytracing_amd.raytracer import Context, PgrtError

    W, H = 330, 200  # 6 x 4 tiles, ragged edge tiles
    gpu_ctx.set_scene(avenger_scene)
    gpu_ctx.set_camera(abi.default_camera(W, H))
    params = [abi.make_params(max_level=5, spp_side=1 + f % 2, dof=f % 2, jitter=abi.PGRT_JITTER_HASH, frame=f)
              for f in range(4)]
    refs = [gpu_ctx.render(p) for p in params]
    g = Context(devices=[0] * ranks)
    try:
        assert g.comm_info() == (ranks, 0)
        g.set_scene(avenger_scene)
        g.set_camera(abi.default_camera(W, H))
        for p, (ref, st_ref) in zip(params, refs):
            img, st = g.render(p)
            same = (img == ref) | (np.isnan(img) & np.isnan(ref))
            assert same.all(), f"{(~same).sum()} pixels differ"
            assert st.rays() == st_ref.rays() and st.rays_shadow == st_ref.rays_shadow
        with pytest.raises(PgrtError):  # whole frames only
            g.render(abi.make_params(max_level=5, rect=(0, 0, 64, 64)))
        # batched frames, two calls in flight
        F = 3
        q = abi.make_params(max_level=5, spp_side=1, jitter=abi.PGRT_JITTER_HASH, frame=0)
        fr = [gpu_ctx.render(abi.make_params(max_level=5, spp_side=1, jitter=abi.PGRT_JITTER_HASH, frame=f))[0]
              for f in range(2 * F)]
        bufs = [g.alloc(F * W * H * 16) for _ in range(2)]
        g.set_frames_in_flight(2)
        t0 = g.render_frames_device_async(q, F, bufs[0])
        q.frame = F
        t1 = g.render_frames_device_async(q, F, bufs[1])
        for t, b, base in ((t0, bufs[0], 0), (t1, bufs[1], F)):
            st = g.render_wait(t)
            assert st.rays_primary == F * W * H
            out = g.to_host(b, (F, H, W, 4))
            for f in range(F):
                same = (out[f] == fr[base + f]) | (np.isnan(out[f]) & np.isnan(fr[base + f]))
                assert same.all(), f"frame {base + f}: {(~same).sum()} pixels differ"
        for b in bufs:
            g.free(b)
    finally:
        g.close()


@pytest.mark.parametrize("builder,width,split,group", [
    (abi.PGRT_BVH_LBVH, 2, 0.0, -1), (abi.PGRT_BVH_PLOC, 8, 0.0, -1), (abi.PGRT_BVH_LBVH, 8, 0.0, -1),
    (abi.PGRT_BVH_PLOC, 2, 0.0, -1), (abi.PGRT_BVH_PLOC, 2, 1.0, -1), (abi.PGRT_BVH_PLOC, 8, 0.5, -1),
    (abi.PGRT_BVH_PLOC, 2, 0.0, 1 << 30), (abi.PGRT_BVH_LBVH, 2, 0.5, 1 << 30),
    (abi.PGRT_BVH_PLOC, 2, 0.5, 1 << 30), (abi.PGRT_BVH_PLOC, 8, 0.0, 1 << 30)])
def test_bvh_layouts_bit_exact(gpu_ctx, avenger_scene, builder, width, split, group):
    """Every BVH builder / traversal layout / split budget (pgrt_config) gives the same closest
    hits and frames: the hit is order-independent (ties to the smaller triangle index,
    conservative box tests), and split references cover their triangle.  group: queues up to it
    take 8 (4) lanes per ray over the 8-wide BVH (-1 never)."""
    old = gpu_ctx.configure(bvh_builder=builder, bvh_width=width, split_beta=split, group_max=group)
    try:
        gpu_ctx.set_scene(avenger_scene)
        info = gpu_ctx.bvh_info()
        assert info.width == width and info.builder == builder
        if builder == abi.PGRT_BVH_PLOC and split > 0:
            assert info.num_references > info.num_triangles
        else:
            assert info.num_references == info.num_triangles
        rays = _random_rays(avenger_scene, 20000, 11)
        hg = gpu_ctx.intersect(rays)
        ho = _oracle(avenger_scene).intersect(rays)
        eq = (hg.view(np.int32) == ho.view(np.int32)).all(1)
        assert eq.all(), f"{(~eq).sum()} / {len(eq)} hit records differ"
        cam = abi.default_camera(96, 64)
        gpu_ctx.set_camera(cam)
        p = abi.make_params(spp_side=2, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH)
        img, _ = gpu_ctx.render(p)
        ref, _ = _oracle(avenger_scene).render(cam, p)
        _, exact = assert_frames_match(img, ref)
        assert exact == 1.0
    finally:
        gpu_ctx.set_config(old)
        gpu_ctx.set_scene(avenger_scene)


@pytest.mark.parametrize("packets", [abi.PGRT_PACKETS_OFF, 1, abi.PGRT_PACKETS_AUTO, 16])
def test_packet_levels_bit_exact(gpu_ctx, avenger_scene, packets):
    """Every packet-traversal depth (none: k_raygen + one lane per ray; level 0 only, which
    generates its rays in the traversal; the default; every level) renders the oracle's frame bit
    for bit, frames in flight and batched frames included."""
    gpu_ctx.set_scene(avenger_scene)
    old = gpu_ctx.configure(packet_levels=packets)
    try:
        W, H = 96, 64
        cam = abi.default_camera(W, H)
        gpu_ctx.set_camera(cam)
        for p in (abi.make_params(spp_side=1, max_level=5),
                  abi.make_params(spp_side=2, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=3)):
            img, _ = gpu_ctx.render(p)
            ref, _ = _oracle(avenger_scene).render(cam, p)
            _, exact = assert_frames_match(img, ref)
            assert exact == 1.0
        buf = gpu_ctx.alloc(3 * W * H * 16)
        try:
            gpu_ctx.set_frames_in_flight(2)
            p = abi.make_params(spp_side=1, max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=7)
            gpu_ctx.render_wait(gpu_ctx.render_frames_device_async(p, 3, buf))
            out = gpu_ctx.to_host(buf, (3, H, W, 4))
            for f in range(3):
                ref, _ = _oracle(avenger_scene).render(
                    cam, abi.make_params(spp_side=1, max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=7 + f))
                _, exact = assert_frames_match(out[f], ref)
                assert exact == 1.0, f"batched frame {f}"
        finally:
            gpu_ctx.set_frames_in_flight(1)
            gpu_ctx.free(buf)
    finally:
        gpu_ctx.set_config(old)


@pytest.mark.parametrize("budget", [1, 24, 200])
def test_packet_budget_deferral_bit_exact(gpu_ctx, avenger_scene, budget):
    """Bounce-level packets with a step budget: waves out of steps store their rays' closest hits so
    far and hand the rays to the 8-lanes-per-ray kernel, which resumes from those hits.  A tiny
    budget defers nearly every wave (every ray resumed), a middling one a mix; packets on every
    level, DoF samples and the all-glass geosphere included, oracle bit for bit."""
    gpu_ctx.set_scene(avenger_scene)
    old = gpu_ctx.configure(packet_levels=16, packet_budget=budget)
    try:
        W, H = 96, 64
        cam = abi.default_camera(W, H)
        gpu_ctx.set_camera(cam)
        for p in (abi.make_params(spp_side=1, max_level=5),
                  abi.make_params(spp_side=2, max_level=7, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=5)):
            img, _ = gpu_ctx.render(p)
            ref, _ = _oracle(avenger_scene).render(cam, p)
            _, exact = assert_frames_match(img, ref)
            assert exact == 1.0
        rays = _random_rays(avenger_scene, 4000, 3)
        hg = gpu_ctx.intersect(rays)
        ho = _oracle(avenger_scene).intersect(rays)
        assert (hg.view(np.int32) == ho.view(np.int32)).all()
    finally:
        gpu_ctx.set_config(old)


@pytest.mark.parametrize("sub,packets", [(1, abi.PGRT_PACKETS_AUTO), (2, abi.PGRT_PACKETS_AUTO), (3, 16),
                                         (5, abi.PGRT_PACKETS_OFF), (7, abi.PGRT_PACKETS_AUTO)])
def test_subtree_levels_bit_exact(gpu_ctx, avenger_scene, geosphere_scene, sub, packets):
    """Levels >= sub as whole ray trees in one launch (subtree.hip: reflection, refraction and shadow
    rays of each level-sub ray traced and shaded depth first, as the reference's recursive trace
    does): the avenger at d = 5 / 7 (pinhole, DoF samples), the all-glass geosphere at d = 8 (total
    internal reflection chains), batched frames in flight -- oracle bit for bit, and the same ray
    counts per kind."""
    old = gpu_ctx.configure(subtree_level=sub, packet_levels=packets)
    try:
        for scene, cfgs in ((avenger_scene, (dict(spp_side=1, max_level=5), dict(spp_side=1, max_level=7),
                                             dict(spp_side=2, max_level=7, dof=1, jitter=abi.PGRT_JITTER_HASH,
                                                  frame=2))),
                            (geosphere_scene, (dict(spp_side=2, max_level=8, jitter=abi.PGRT_JITTER_HASH),))):
            gpu_ctx.set_scene(scene)
            W, H = 96, 64
            cam = (abi.default_camera(W, H) if scene is avenger_scene else
                   abi.make_camera(W, H, abi.deg2rad(90.0), (2.0, 0.0, 0.0), (0.0, 0.0, 0.0)))  # tutorials.cpp:194
            gpu_ctx.set_camera(cam)
            for c in cfgs:
                p = abi.make_params(**c)
                img, st = gpu_ctx.render(p)
                ref, sto = _oracle(scene).render(cam, p)
                _, exact = assert_frames_match(img, ref)
                assert exact == 1.0, f"{c}"
                assert (st.rays_primary, st.rays_shadow, st.rays_reflect, st.rays_refract) == \
                    (sto.rays_primary, sto.rays_shadow, sto.rays_reflect, sto.rays_refract), f"{c}"
        gpu_ctx.set_scene(avenger_scene)
        cam = abi.default_camera(96, 64)
        gpu_ctx.set_camera(cam)
        buf = gpu_ctx.alloc(3 * 96 * 64 * 16)
        try:
            gpu_ctx.set_frames_in_flight(2)
            p = abi.make_params(spp_side=1, max_level=6, jitter=abi.PGRT_JITTER_HASH, frame=11)
            gpu_ctx.render_wait(gpu_ctx.render_frames_device_async(p, 3, buf))
            out = gpu_ctx.to_host(buf, (3, 64, 96, 4))
            for f in range(3):
                ref, _ = _oracle(avenger_scene).render(
                    cam, abi.make_params(spp_side=1, max_level=6, jitter=abi.PGRT_JITTER_HASH, frame=11 + f))
                _, exact = assert_frames_match(out[f], ref)
                assert exact == 1.0, f"batched frame {f}"
        finally:
            gpu_ctx.set_frames_in_flight(1)
            gpu_ctx.free(buf)
    finally:
        gpu_ctx.set_config(old)
        gpu_ctx.set_scene(avenger_scene)


@pytest.mark.parametrize("order", [0, -1])
def test_tile_order_bit_exact(gpu_ctx, avenger_scene, order):
    """Synchronous frames after the first of a size deal the tiles whose primary rays hit a
    dielectric in the previous frame to the first pipeline slot (pgrt_config.tile_order 0) or
    round-robin (-1); a different camera makes the recorded tiles stale -- every frame equals the
    oracle bit for bit, with the same ray counts per kind."""
    old = gpu_ctx.configure(tile_order=order)
    gpu_ctx.set_scene(avenger_scene)
    try:
        W, H = 448, 320  # 7 x 5 tiles: the canopy covers some of them
        for k, (pos, c) in enumerate((((0.0, 0.0, 0.0), dict(spp_side=1, max_level=5)),
                                      ((0.0, 0.0, 0.0), dict(spp_side=1, max_level=5, jitter=abi.PGRT_JITTER_HASH,
                                                             frame=4)),
                                      ((0.0, 0.0, 0.0), dict(spp_side=2, max_level=4)),
                                      ((30.0, -20.0, 10.0), dict(spp_side=1, max_level=6)))):
            cam = abi.default_camera(W, H)
            if k == 3:  # moved camera: the deal follows the last frame's tiles (stale, speed only)
                cam = abi.make_camera(W, H, abi.deg2rad(42.185), (-140.0 + pos[0], -175.0 + pos[1], 80.0 + pos[2]),
                                      (0.0, 0.0, 0.0))
            gpu_ctx.set_camera(cam)
            p = abi.make_params(**c)
            for rep in range(2):
                img, st = gpu_ctx.render(p)
                ref, sto = _oracle(avenger_scene).render(cam, p)
                _, exact = assert_frames_match(img, ref)
                assert exact == 1.0, f"{c} rep {rep}"
                assert (st.rays_primary, st.rays_shadow, st.rays_reflect, st.rays_refract) == \
                    (sto.rays_primary, sto.rays_shadow, sto.rays_reflect, sto.rays_refract), f"{c}"
    finally:
        gpu_ctx.set_config(old)


def test_auto_probe_frames_unchanged(gpu_ctx, avenger_scene):
    """PGRT_PACKETS_AUTO re-probes a level that is off packets every 32 collected calls with a side
    packet launch over the level's first rays (hit records discarded): 70 calls of the same frame
    (several probes) stay bit-identical to the oracle, and the probe launch really runs -- in some
    frame, a level traced one lane per ray also has a packet launch (the device timeline).  The deep
    levels are traced per level (subtree_level -1): with the one-frame default the subtree launch
    takes level 3, the level AUTO probes first."""
    gpu_ctx.set_scene(avenger_scene)  # AUTO starts over per scene
    old = gpu_ctx.configure(packet_levels=abi.PGRT_PACKETS_AUTO, subtree_level=-1)
    gpu_ctx.timeline_enable(True)
    try:
        cam = abi.default_camera(80, 48)
        gpu_ctx.set_camera(cam)
        p = abi.make_params(spp_side=1, max_level=6, jitter=abi.PGRT_JITTER_HASH, frame=4)
        ref, _ = _oracle(avenger_scene).render(cam, p)
        for k in range(70):
            img, _ = gpu_ctx.render(p)
            _, exact = assert_frames_match(img, ref)
            assert exact == 1.0, f"call {k}"
        recs = gpu_ctx.timeline_read()
    finally:
        gpu_ctx.timeline_enable(False)
        gpu_ctx.set_config(old)
    by = {}
    for r in recs:
        by.setdefault((r["ticket"], r["level"]), set()).add(r["kind"])
    probed = [key for key, kinds in by.items() if key[1] >= 1 and "trace_pkt" in kinds and kinds & {"trace", "trace_8g"}]
    assert probed, "no frame ran AUTO's probe launch beside a level's one-lane trace"


def test_timeline_records_and_frames_unchanged(gpu_ctx, avenger_scene):
    """pgrt_timeline_enable: a stamped frame is the oracle's frame bit for bit, every launch of it
    leaves one record (wave-ordered spans on the device clock, percentiles within the span), and
    reading removes the records."""
    gpu_ctx.set_scene(avenger_scene)
    cam = abi.default_camera(96, 64)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(spp_side=1, max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=2)
    ref, _ = _oracle(avenger_scene).render(cam, p)
    gpu_ctx.timeline_enable(True)
    try:
        img, _ = gpu_ctx.render(p)
        recs = gpu_ctx.timeline_read()
    finally:
        gpu_ctx.timeline_enable(False)
    _, exact = assert_frames_match(img, ref)
    assert exact == 1.0
    kinds = {r["kind"] for r in recs}
    assert {"shade", "finish", "export"} <= kinds, kinds
    assert any(r["kind"].startswith("trace") and r["level"] == 0 for r in recs)
    for r in recs:
        span = r["end"] - r["start"]
        assert r["waves"] > 0 and span >= 0
        p50, p90, mx = r["wave_us"]
        assert p50 <= p90 <= mx <= span / 100.0 + 1e-6
        assert 0 <= r["last_in_us"] <= span / 100.0 + 1e-6
    assert gpu_ctx.timeline_read() == []
    img2, _ = gpu_ctx.render(p)  # off again: no records
    assert gpu_ctx.timeline_read() == []
    assert np.array_equal(img2, img)


@pytest.mark.parametrize("octant", range(8))
def test_packet_sign_octants_bit_exact(gpu_ctx, avenger_scene, octant):
    """The packet kernel runs one of 8 node loops per direction-sign combination (near / far
    planes fixed at compile time) and a min / max loop for mixed-sign waves: a camera in each
    octant around the model sends the primary waves through every combination (the waves on the
    image's sign boundaries through the mixed loop), packets on every level, oracle bit for bit."""
    gpu_ctx.set_scene(avenger_scene)
    old = gpu_ctx.configure(packet_levels=16)
    try:
        W, H = 64, 48
        sx, sy, sz = (1 if octant & 1 else -1), (1 if octant & 2 else -1), (1 if octant & 4 else -1)
        cam = abi.make_camera(W, H, abi.deg2rad(42.185), (160.0 * sx, 190.0 * sy, 40.0 + 110.0 * sz),
                              (0.0, 0.0, 40.0))
        gpu_ctx.set_camera(cam)
        p = abi.make_params(spp_side=1, max_level=3)
        img, _ = gpu_ctx.render(p)
        ref, _ = _oracle(avenger_scene).render(cam, p)
        _, exact = assert_frames_match(img, ref)
        assert exact == 1.0
    finally:
        gpu_ctx.set_config(old)


def test_occluded_matches_closest_hit(gpu_ctx, avenger_scene):
    """rtcOccluded1 analogue: any hit in (tnear, tfar] exactly when the closest-hit query (oracle)
    finds one -- including finite-tfar shadow-style rays that stop short of the geometry."""
    gpu_ctx.set_scene(avenger_scene)
    rays = _random_rays(avenger_scene, 20000, 21)
    short = rays.copy()
    short[:, 7] = np.float32(5.0)  # tfar 5: most rays stop before any triangle
    rays = np.concatenate([rays, short])
    occ = gpu_ctx.occluded(rays)
    ho = _oracle(avenger_scene).intersect(rays)
    expect = ho[:, 3].view(np.int32) >= 0
    assert (occ == expect).all(), f"{(occ != expect).sum()} differ"
    assert 1000 < occ.sum() < len(occ) - 1000


def test_progressive_accumulation_is_mean_of_frames(gpu_ctx, avenger_scene):
    """Frame sink: the device running mean of 4 jittered DoF frames equals the float32 mean of
    the same frames rendered one by one (same summation order), and a reset restarts it."""
    gpu_ctx.set_scene(avenger_scene)
    cam = abi.default_camera(96, 64)
    gpu_ctx.set_camera(cam)
    frames = []
    for f in range(4):
        p = abi.make_params(spp_side=1, max_level=3, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=f)
        img, _ = gpu_ctx.render(p)
        frames.append(img)
    gpu_ctx.accumulate_reset()
    for f in range(4):
        mean, n = gpu_ctx.render_accumulate(abi.make_params(spp_side=1, max_level=3, dof=1,
                                                             jitter=abi.PGRT_JITTER_HASH, frame=f))
    assert n == 4
    acc = frames[0].copy()
    for fr in frames[1:]:
        acc = acc + fr
    ref = acc / np.float32(4)
    same = (mean == ref) | (np.isnan(mean) & np.isnan(ref))
    assert same.all()
    assert not (frames[0] == frames[1]).all()  # the jitter differs per frame
    gpu_ctx.accumulate_reset()
    m1, n1 = gpu_ctx.render_accumulate(abi.make_params(spp_side=1, max_level=3, dof=1, jitter=abi.PGRT_JITTER_HASH,
                                                       frame=0))
    assert n1 == 1 and ((m1 == frames[0]) | (np.isnan(m1) & np.isnan(frames[0]))).all()


def test_batched_frames_match_single(gpu_ctx, avenger_scene):
    """pgrt_render_frames_device_async: nframes frames in one pass (ragged 200x120 frame, so
    padded edge tiles repeat per frame) are bit-identical to single renders with frame index
    base + f; the distributed form (world 1) unpacks every frame; nframes outside [1, 64] is
    refused."""
    from pgi_raytracing_amd.raytracer import PgrtError

    gpu_ctx.set_scene(avenger_scene)
    W, H = 200, 120
    gpu_ctx.set_camera(abi.default_camera(W, H))
    for spp_side, dof, F, rect in ((1, 0, 3, (0, 0, 0, 0)), (2, 1, 5, (0, 0, 0, 0)), (1, 1, 2, (30, 20, 100, 70))):
        def params(frame):
            return abi.make_params(max_level=5, spp_side=spp_side, dof=dof, jitter=abi.PGRT_JITTER_HASH,
                                   frame=frame, rect=rect)

        p = params(11)
        w, h = (rect[2], rect[3]) if rect[2] else (W, H)
        frame_bytes = w * h * 16
        refs = [gpu_ctx.render(params(11 + f)) for f in range(F)]
        buf = gpu_ctx.alloc(F * frame_bytes)
        dbuf = gpu_ctx.alloc(F * frame_bytes)
        try:
            gpu_ctx.set_frames_in_flight(2)
            t0 = gpu_ctx.render_frames_device_async(p, F, buf)
            st0 = gpu_ctx.render_wait(t0)
            assert st0.rays() == sum(st.rays() for _, st in refs)
            out = gpu_ctx.to_host(buf, (F, h, w, 4))
            checks = [("frames", out)]
            st1 = gpu_ctx.render_frames_device(params(11), F, dbuf)  # synchronous form
            assert st1.rays() == st0.rays()
            checks.append(("synchronous frames", gpu_ctx.to_host(dbuf, (F, h, w, 4))))
            if not rect[2]:  # the distributed form renders the whole camera image
                gpu_ctx.render_wait(gpu_ctx.render_frames_distributed_device_async(p, F, dbuf))
                checks.append(("distributed frames", gpu_ctx.to_host(dbuf, (F, H, W, 4))))
            # host output (pinned): two calls in flight, then one call on the 2-slot synchronous set
            for n_in_flight in (2, 1):
                gpu_ctx.set_frames_in_flight(n_in_flight)
                hb = [gpu_ctx.host_array((F, h, w, 4)) for _ in range(2)]
                try:
                    for a in hb:
                        a.fill(-7.0)
                    ts = [gpu_ctx.render_frames_host_async(p, F, a) for a in hb]
                    assert gpu_ctx.render_wait(ts[-1]).rays() == st0.rays()
                    for k, a in enumerate(hb):
                        checks.append((f"host frames {n_in_flight}/{k}", a.copy()))
                finally:
                    for a in hb:
                        gpu_ctx.host_free(a)
            gpu_ctx.set_frames_in_flight(2)
            for f, (ref, _) in enumerate(refs):
                for name, o in ((n, a[f]) for n, a in checks):
                    same = (o == ref) | (np.isnan(o) & np.isnan(ref))
                    assert same.all(), f"{name} S={spp_side} frame {f}: {(~same).sum()} pixels differ"
            if F > 1:
                assert not np.array_equal(out[0], out[1])  # the frames really differ (jitter)
            for bad in (0, 65):
                with pytest.raises(PgrtError):
                    gpu_ctx.render_frames_device_async(p, bad, buf)
        finally:
            gpu_ctx.set_frames_in_flight(1)
            gpu_ctx.free(buf)
            gpu_ctx.free(dbuf)


def test_full_size_c2_batched_bit_exact(gpu_ctx, avenger_scene):
    """BASELINE C2 at its full size through the bench's path (batched frames, frames in flight,
    packets on levels 0-2, block-level queue allocation): every pixel of both frames of a
    2-frame call equals the CPU restatement's frame bit for bit; plus a 2x2-spp DoF frame."""
    gpu_ctx.set_scene(avenger_scene)
    W, H = 1920, 1080
    cam = abi.default_camera(W, H)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(max_level=5)
    ref, st_ref = _oracle(avenger_scene).render(cam, p, threads=16)
    buf = gpu_ctx.alloc(2 * W * H * 16)
    try:
        gpu_ctx.set_frames_in_flight(6)
        st = gpu_ctx.render_wait(gpu_ctx.render_frames_device_async(p, 2, buf))
        assert st.rays() == 2 * st_ref.rays()
        out = gpu_ctx.to_host(buf, (2, H, W, 4))
        for f in range(2):
            _, exact = assert_frames_match(out[f], ref)
            assert exact == 1.0, f"frame {f}"
    finally:
        gpu_ctx.set_frames_in_flight(1)
        gpu_ctx.free(buf)
    q = abi.make_params(max_level=5, spp_side=2, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=5)
    img, _ = gpu_ctx.render(q)
    ref2, _ = _oracle(avenger_scene).render(cam, q, threads=16)
    _, exact = assert_frames_match(img, ref2)
    assert exact == 1.0


def test_full_size_c2_distinct_frames_bit_exact(gpu_ctx, avenger_scene):
    """The bench's default C2 workload (bench.py --frames distinct): a 2-frame call with hash
    jitter at 1 spp (get_pixel's sub-pixel jitter, raytracer.cpp:407-413) and its own frame
    indices, 3 calls in flight into separate framebuffers -- every frame equals the CPU
    restatement's frame with the same frame index bit for bit, and the frames differ."""
    gpu_ctx.set_scene(avenger_scene)
    W, H = 1920, 1080
    cam = abi.default_camera(W, H)
    gpu_ctx.set_camera(cam)
    F, calls = 2, 3
    bufs = [gpu_ctx.alloc(F * W * H * 16) for _ in range(calls)]
    try:
        gpu_ctx.set_frames_in_flight(calls)
        tickets = [gpu_ctx.render_frames_device_async(
            abi.make_params(max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=F * k), F, b) for k, b in enumerate(bufs)]
        for t in tickets:
            gpu_ctx.render_wait(t)
        outs = [gpu_ctx.to_host(b, (F, H, W, 4)) for b in bufs]
    finally:
        gpu_ctx.set_frames_in_flight(1)
        for b in bufs:
            gpu_ctx.free(b)
    for f in (0, 3, 5):  # first frame of call 0, second of call 1, last of call 2
        ref, _ = _oracle(avenger_scene).render(cam, abi.make_params(max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=f),
                                               threads=16)
        _, exact = assert_frames_match(outs[f // F][f % F], ref)
        assert exact == 1.0, f"frame {f}"
    assert not np.array_equal(outs[0][0], outs[0][1])


def test_distributed_frame_after_host_output_leaves_host_buffer_alone(gpu_ctx, avenger_scene):
    """Regression (r2 advisor): a synchronous distributed frame reuses frame set 0, which the
    default one-frame-in-flight pgrt_render_frames_host_async also uses -- its host destination
    must not be kept: the distributed frame would copy into a buffer the caller may have freed.
    The old host buffer is refilled with a sentinel after its call and must keep it."""
    gpu_ctx.set_scene(avenger_scene)
    W, H = 128, 64
    gpu_ctx.set_camera(abi.default_camera(W, H))
    uid = gpu_ctx.comm_unique_id()
    gpu_ctx.comm_init(1, 0, uid)
    p = abi.make_params(max_level=3)
    hb = gpu_ctx.host_array((1, H, W, 4))
    fb = gpu_ctx.alloc(W * H * 16)
    try:
        gpu_ctx.set_frames_in_flight(1)
        gpu_ctx.render_wait(gpu_ctx.render_frames_host_async(p, 1, hb))
        ref, _ = gpu_ctx.render(p)
        assert ((hb[0] == ref) | (np.isnan(hb[0]) & np.isnan(ref))).all()
        hb.fill(-7.0)
        gpu_ctx.render_distributed_device(p, fb)
        out, _ = gpu_ctx.render_distributed(p)
        gpu_ctx.synchronize()
        assert (hb == -7.0).all(), "the distributed frame wrote the previous call's host buffer"
        assert ((out == ref) | (np.isnan(out) & np.isnan(ref))).all()
    finally:
        gpu_ctx.host_free(hb)
        gpu_ctx.free(fb)


def test_new_frame_sets_start_clean(avenger_scene):
    """Regression (r1h): the first frame on each new frame set must see zeroed queue counters
    -- they were zeroed by a NULL-stream hipMemset, unordered with the slot streams, and a set's
    first frame could lose its secondary rays.  A fresh context, 6 sets, 720p frames."""
    from pgi_raytracing_amd.raytracer import Context

    ctx = Context(0)
    try:
        ctx.set_scene(avenger_scene)
        W, H = 1280, 720
        ctx.set_camera(abi.default_camera(W, H))
        p = abi.make_params(max_level=5)
        _, st_ref = ctx.render(p)
        fb = ctx.alloc(W * H * 16)
        ctx.set_frames_in_flight(6)
        tickets = [ctx.render_device_async(p, fb) for _ in range(6)]
        for t in tickets:
            st = ctx.render_wait(t)
            assert st.rays() == st_ref.rays() and st.rays_shadow == st_ref.rays_shadow
        ctx.free(fb)
    finally:
        ctx.close()


def test_frames_in_flight_match_synchronous(gpu_ctx, avenger_scene):
    """Asynchronous frames (3 in flight, different depth / spp / DoF / seed per frame, the
    distributed form included) are bit-identical to synchronous renders; a recycled ticket is
    refused."""
    from pgi_raytracing_amd.raytracer import PgrtError

    gpu_ctx.set_scene(avenger_scene)
    W, H = 200, 120
    gpu_ctx.set_camera(abi.default_camera(W, H))
    params = [abi.make_params(max_level=5 if f % 2 == 0 else 3, spp_side=2 if f % 3 == 2 else 1, dof=f % 2,
                              jitter=abi.PGRT_JITTER_HASH, frame=f) for f in range(7)]
    refs = [gpu_ctx.render(p) for p in params]
    bufs = [gpu_ctx.alloc(W * H * 16) for _ in params]
    try:
        gpu_ctx.set_frames_in_flight(3)
        tickets = [gpu_ctx.render_device_async(p, b) if f != 4 else gpu_ctx.render_distributed_device_async(p, b)
                   for f, (p, b) in enumerate(zip(params, bufs))]
        with pytest.raises(PgrtError):
            gpu_ctx.render_wait(tickets[0])  # its frame set was reused by tickets[3]
        stats = [gpu_ctx.render_wait(t) for t in tickets[4:]]
        for (ref, st_ref), st in zip(refs[4:], stats):
            assert st.rays() == st_ref.rays()
        for f, (b, (ref, _)) in enumerate(zip(bufs, refs)):
            out = gpu_ctx.to_host(b, (H, W, 4))
            same = (out == ref) | (np.isnan(out) & np.isnan(ref))
            assert same.all(), f"frame {f}: {(~same).sum()} pixels differ"
    finally:
        gpu_ctx.set_frames_in_flight(1)
        for b in bufs:
            gpu_ctx.free(b)


def test_host_framebuffer_pinned_sync_equals_device(gpu_ctx, avenger_scene):
    """pgrt_render into page-locked host memory: every pipeline slot exports its finished tiles
    itself (k_export_tiles, the bulk slot while the deep-tile slot still renders) -- the host frame
    equals the device-resident frame and the pageable-memory path bit for bit, at C2's full size
    (the second frame takes the deep-tiles-first deal) and for a render rect."""
    gpu_ctx.set_scene(avenger_scene)
    W, H = 1920, 1080
    gpu_ctx.set_camera(abi.default_camera(W, H))
    gpu_ctx.set_frames_in_flight(1)
    try:
        for mode in (0, 1, -1, 2):  # pgrt_config.host_export: default, export kernels, one copy, split
            gpu_ctx.configure(host_export=mode)
            _host_frames_equal_device(gpu_ctx, W, H)
    finally:
        gpu_ctx.configure(host_export=0)


def test_host_framebuffer_in_flight_modes_equal_device(gpu_ctx, avenger_scene):
    """pgrt_render_frames_host_async (3 frames per call, 2 calls in flight) into page-locked
    memory under every host_export mode -- one DMA copy, export kernels, and the split copy (a blit
    kernel's share on a side stream beside the DMA copy of the rest) -- equals the device frames."""
    gpu_ctx.set_scene(avenger_scene)
    W, H, F = 640, 360, 3
    gpu_ctx.set_camera(abi.default_camera(W, H))
    params = [abi.make_params(max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=20 + 3 * k) for k in range(2)]
    dev = gpu_ctx.alloc(F * W * H * 16)
    refs = []
    try:
        for p in params:
            gpu_ctx.render_frames_device(p, F, dev)
            refs.append(gpu_ctx.to_host(dev, (F, H, W, 4)))
        gpu_ctx.set_frames_in_flight(2)
        for mode in (0, 1, -1, 2):
            gpu_ctx.configure(host_export=mode)
            hb = [gpu_ctx.host_array((F, H, W, 4)) for _ in params]
            try:
                for a in hb:
                    a.fill(-7.0)
                ts = [gpu_ctx.render_frames_host_async(p, F, a) for p, a in zip(params, hb)]
                for t in ts:
                    gpu_ctx.render_wait(t)
                for k, (a, ref) in enumerate(zip(hb, refs)):
                    same = (a == ref) | (np.isnan(a) & np.isnan(ref))
                    assert same.all(), f"host_export {mode} call {k}: {(~same).sum()} pixels differ"
            finally:
                for a in hb:
                    gpu_ctx.host_free(a)
    finally:
        gpu_ctx.configure(host_export=0)
        gpu_ctx.set_frames_in_flight(1)
        gpu_ctx.free(dev)


def _host_frames_equal_device(gpu_ctx, W, H):
    for p, (w, h) in ((abi.make_params(max_level=5), (W, H)),
                      (abi.make_params(max_level=5, jitter=abi.PGRT_JITTER_HASH, frame=3), (W, H)),
                      (abi.make_params(max_level=5, rect=(101, 37, 333, 190)), (333, 190))):
        fb = gpu_ctx.alloc(w * h * 16)
        hb = gpu_ctx.host_array((h, w, 4))
        try:
            for _ in range(2):  # the second synchronous frame deals the deep tiles to slot 0
                hb.fill(-7.0)
                gpu_ctx.render(p, out=hb)
            gpu_ctx.render_device(p, fb)
            dev = gpu_ctx.to_host(fb, (h, w, 4))
            pageable, _ = gpu_ctx.render(p)
            for name, o in (("pinned", hb), ("pageable", pageable)):
                same = (o == dev) | (np.isnan(o) & np.isnan(dev))
                assert same.all(), f"{name} {w}x{h}: {(~same).sum()} pixels differ"
        finally:
            gpu_ctx.host_free(hb)
            gpu_ctx.free(fb)


def test_config_size_is_checked(gpu_ctx):
    """pgrt_config carries its size (abi 2; abi 3 added peer_wait_ms): pgrt_get_config fills it, pgrt_set_config rejects a
    struct of another layout instead of writing its fields into the wrong places."""
    from pgi_raytracing_amd.raytracer import PgrtError

    cfg = gpu_ctx.get_config()
    assert cfg.size == C.sizeof(abi.Config)
    assert b"abi 3" in gpu_ctx.L.pgrt_version()
    bad = abi.Config.from_buffer_copy(cfg)
    bad.size = cfg.size - 4
    with pytest.raises(PgrtError, match="pgrt_config.size"):
        gpu_ctx.set_config(bad)
    bad = abi.Config.from_buffer_copy(cfg)
    bad.host_export = 5
    with pytest.raises(PgrtError):
        gpu_ctx.set_config(bad)
    bad = abi.Config.from_buffer_copy(cfg)
    bad.peer_wait_ms = -1
    with pytest.raises(PgrtError, match="peer_wait_ms"):
        gpu_ctx.set_config(bad)
    gpu_ctx.set_config(cfg)


def test_distributed_overflow_on_one_rank(geosphere_scene):
    """A queue overflow on ONE rank of a distributed frame (verdict r4 #5): the all-glass geosphere
    fills rank 1's tile only (128x64 = two tiles, rank r renders tile r), so rank 1's level-1 queue
    (sized for its 4096 primary rays) overflows on the first frame while rank 0's never does.  Rank
    1 re-renders its tiles with grown queues and rank 0 gathers them again: the frame equals the
    oracle bit for bit, the re-render is reported, and the next frame (grown queues) needs none.
    Ranks on this one GPU gather by device copies (the multi-process RCCL form of the same protocol
    -- overflow flag and frame sequence at the tail of each send -- needs one GPU per rank)."""
    from pgi_raytracing_amd.raytracer import Context

    W, H = 128, 64
    cam = abi.make_camera(W, H, abi.deg2rad(90.0), (2.0, 0.0, 0.0), (0.0, -1.3, 0.0))
    p = abi.make_params(max_level=5)
    ref, sto = _oracle(geosphere_scene).render(cam, p)
    g = Context(devices=[0, 0])
    try:
        g.set_scene(geosphere_scene)
        g.set_camera(cam)
        for frame in range(2):
            img, st = g.render(p)
            _, exact = assert_frames_match(img, ref)
            assert exact == 1.0, f"frame {frame}"
            assert (st.rays_primary, st.rays_reflect, st.rays_refract, st.rays_shadow) == \
                (sto.rays_primary, sto.rays_reflect, sto.rays_refract, sto.rays_shadow), f"frame {frame}"
            assert (st.overflow_retries >= 1) == (frame == 0), f"frame {frame}: {st.overflow_retries} re-renders"
    finally:
        g.close()
