"""GPU parity on the BASELINE configs C3, C4 and C5 through the product path.

Bar: bit-exact frames (exact-match fraction 1, i.e. within the 1e-4 tolerance with 0 slack) and
equal ray counts against the CPU restatement (oracle/) on the same pixels.  The oracle is timed
in seconds only on a subset of each frame: C3 on a reduced image (every sample batch of the
multi-batch path), C4 on whole 64x64 tiles of a rank's share, C5 on rows (every 256th row).
"""
import numpy as np
import pytest

import pyoracle
from conftest import ENV_MAP, assert_frames_match
from pgi_raytracing_amd import abi

pytestmark = pytest.mark.gpu


def _frames_equal(a, b):
    return bool(((a == b) | (np.isnan(a) & np.isnan(b))).all())


def test_c3_multi_batch_64spp_dof(gpu_ctx, avenger_scene):
    """C3's defining path -- 64 spp DoF split into sample batches, the parallel level-0 combine
    (k_combine over level 0) and the batched k_finish accumulation -- at 128x96: with
    max_batch_rays 16384 every batch holds 2 of the 64 samples of the slot's pixels (32 batches
    per slot), and the frame equals the oracle's bit for bit; so does the same frame through
    frames in flight and with the default batching (one batch)."""
    gpu_ctx.set_scene(avenger_scene)
    W, H = 128, 96
    cam = abi.default_camera(W, H)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(spp_side=8, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=2)
    ref, sto = pyoracle.OracleScene(avenger_scene).render(cam, p, threads=16)
    one, st1 = gpu_ctx.render(p)  # default: the whole frame in one sample batch
    old = gpu_ctx.configure(max_batch_rays=16384)
    try:
        img, st = gpu_ctx.render(p)
        for name, out, s in (("multi-batch", img, st), ("single batch", one, st1)):
            _, exact = assert_frames_match(out, ref)
            assert exact == 1.0, name
            assert (s.rays_primary, s.rays_shadow, s.rays_reflect, s.rays_refract) == \
                (sto.rays_primary, sto.rays_shadow, sto.rays_reflect, sto.rays_refract), name
        buf = gpu_ctx.alloc(W * H * 16)
        try:
            gpu_ctx.set_frames_in_flight(3)
            tickets = [gpu_ctx.render_device_async(p, buf) for _ in range(3)]
            for t in tickets:
                assert gpu_ctx.render_wait(t).rays() == sto.rays()
            assert _frames_equal(gpu_ctx.to_host(buf, (H, W, 4)), ref)
        finally:
            gpu_ctx.set_frames_in_flight(1)
            gpu_ctx.free(buf)
    finally:
        gpu_ctx.set_config(old)


def test_c3_full_size_default_batching_rows(gpu_ctx, avenger_scene):
    """C3 at its full size (1920x1080, DoF, 64 spp) through the default sample batching (32M
    level-0 rays per batch: several batches per frame, each frame's accumulation over them) and
    frames in flight: every 64th row equals the CPU restatement's bit for bit, and those rows
    rendered as GPU rects give the oracle's ray counts per kind exactly (raytracer.cpp:396-437)."""
    gpu_ctx.set_scene(avenger_scene)
    W, H = 1920, 1080
    cam = abi.default_camera(W, H)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(spp_side=8, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=3)
    assert gpu_ctx.get_config().max_batch_rays == 0  # the default batching
    osc = pyoracle.OracleScene(avenger_scene)
    ref, sto = osc.render(cam, p, row_step=64, threads=16)
    rows = np.arange(0, H, 64)
    bufs = [gpu_ctx.alloc(W * H * 16) for _ in range(2)]
    try:
        gpu_ctx.set_frames_in_flight(2)
        tickets = [gpu_ctx.render_device_async(p, b) for b in bufs]
        stats = [gpu_ctx.render_wait(t) for t in tickets]
        imgs = [gpu_ctx.to_host(b, (H, W, 4)) for b in bufs]
    finally:
        gpu_ctx.set_frames_in_flight(1)
        for b in bufs:
            gpu_ctx.free(b)
    assert stats[0].rays() == stats[1].rays()
    for img in imgs:
        _, exact = assert_frames_match(img[rows], ref[rows])
        assert exact == 1.0
    got = np.zeros(4, np.int64)
    for y in rows:
        _, s = gpu_ctx.render(abi.make_params(spp_side=8, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=3,
                                              rect=(0, int(y), W, 1)))
        got += (s.rays_primary, s.rays_shadow, s.rays_reflect, s.rays_refract)
    assert tuple(got) == (sto.rays_primary, sto.rays_shadow, sto.rays_reflect, sto.rays_refract)
    assert stats[0].rays_primary == W * H * 64


def _tile_rect(W, H, t):
    tx = (W + 63) // 64
    x0, y0 = (t % tx) * 64, (t // tx) * 64
    return x0, y0, min(64, W - x0), min(64, H - y0)


def test_c4_rank_tiles_4k_dof_64spp(gpu_ctx, avenger_scene):
    """C4 (3840x2160, DoF, 64 spp) as ranks 0 and 5 of 8 render it: pgrt_render_tiles_device
    (the rank-local half of the distributed frame) into tile-compact buffers; whole tiles of
    each rank's share (its first tile, one over the glass canopy, its last) equal the oracle's
    rect renders bit for bit, and the two ranks' ray counts sum with the other six to the
    full frame's (rendered once through pgrt_render_device)."""
    from pgi_raytracing_amd.raytracer import lib

    gpu_ctx.set_scene(avenger_scene)
    W, H, world = 3840, 2160, 8
    cam = abi.default_camera(W, H)
    gpu_ctx.set_camera(cam)
    p = abi.make_params(spp_side=8, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=1)
    L = lib()
    osc = pyoracle.OracleScene(avenger_scene)
    rank_rays = 0
    for rank in range(world):
        n = L.pgrt_tile_count(W, H, 64, rank, world)
        assert n > 0
        buf = gpu_ctx.alloc(n * 64 * 64 * 16)
        try:
            st = gpu_ctx.render_tiles_device(p, rank, world, buf)
            rank_rays += st.rays()
            if rank not in (0, 5):
                continue
            tiles = gpu_ctx.to_host(buf, (n, 64, 64, 4))
            idx = [L.pgrt_tile_index(W, H, 64, rank, world, j) for j in range(n)]
            canopy = min(range(n), key=lambda j: abs(idx[j] - (H // 2 // 64) * ((W + 63) // 64) - (W // 2 // 64)))
            for j in sorted({0, canopy, n - 1}):
                x0, y0, w, h = _tile_rect(W, H, idx[j])
                q = abi.make_params(spp_side=8, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=1,
                                    rect=(x0, y0, w, h))
                ref, _ = osc.render(cam, q, threads=16)
                _, exact = assert_frames_match(tiles[j, :h, :w], ref)
                assert exact == 1.0, f"rank {rank} tile {idx[j]}"
        finally:
            gpu_ctx.free(buf)
    fb = gpu_ctx.alloc(W * H * 16)
    try:
        full = gpu_ctx.render_device(p, fb)
    finally:
        gpu_ctx.free(fb)
    assert full.rays() == rank_rays


def test_c4_frames_in_flight_uncapped(gpu_ctx, avenger_scene):
    """Regression (r1d fault, root cause fixed in r1h): C4 frames (32 sample batches each) with
    6 frames in flight and no bound on the queued batches -- every frame set's first frame must
    see zeroed counters, else shadow hit records past the (wrongly reset) shadow count are read
    and their garbage triangle index faults in the shadow resolve.  All 6 frames equal the
    synchronous frame bit for bit."""
    gpu_ctx.set_scene(avenger_scene)
    W, H = 3840, 2160
    gpu_ctx.set_camera(abi.default_camera(W, H))
    p = abi.make_params(spp_side=8, max_level=5, dof=1, jitter=abi.PGRT_JITTER_HASH, frame=9)
    assert gpu_ctx.get_config().max_batches_in_flight == 0  # no bound by default
    ref_buf = gpu_ctx.alloc(W * H * 16)
    bufs = [gpu_ctx.alloc(W * H * 16) for _ in range(6)]
    try:
        st_ref = gpu_ctx.render_device(p, ref_buf)
        ref = gpu_ctx.to_host(ref_buf, (H, W, 4))
        gpu_ctx.set_frames_in_flight(6)
        tickets = [gpu_ctx.render_device_async(p, b) for b in bufs]
        for t in tickets:
            assert gpu_ctx.render_wait(t).rays() == st_ref.rays()
        for k, b in enumerate(bufs):
            assert _frames_equal(gpu_ctx.to_host(b, (H, W, 4)), ref), f"frame {k}"
    finally:
        gpu_ctx.set_frames_in_flight(1)
        gpu_ctx.free(ref_buf)
        for b in bufs:
            gpu_ctx.free(b)


@pytest.fixture(scope="module")
def c5_scene():
    import scenes

    return scenes.random_scene(1_000_000, 42, ENV_MAP)


def test_c5_random_1m_4096_d8(gpu_ctx, c5_scene):
    """C5 (10^6 random triangles, 4096x4096, d = 8) at full size: the frame rendered through the
    batched / in-flight path, every 256th row (16 rows x 4096 pixels) compared with the oracle bit
    for bit; those rows rendered as GPU rects give the oracle's ray counts per kind exactly."""
    gpu_ctx.set_scene(c5_scene)
    info = gpu_ctx.bvh_info()
    assert info.num_triangles == 1_000_000
    W = H = 4096
    cam = abi.make_camera(W, H, abi.deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 0.0))
    gpu_ctx.set_camera(cam)
    p = abi.make_params(max_level=8)
    osc = pyoracle.OracleScene(c5_scene)
    ref, sto = osc.render(cam, p, row_step=256, threads=16)
    fb = gpu_ctx.alloc(W * H * 16)
    try:
        gpu_ctx.set_frames_in_flight(2)
        st = gpu_ctx.render_wait(gpu_ctx.render_device_async(p, fb))
        img = gpu_ctx.to_host(fb, (H, W, 4))
    finally:
        gpu_ctx.set_frames_in_flight(1)
        gpu_ctx.free(fb)
    assert st.rays_refract > 0 and st.rays_shadow > 0
    rows = np.arange(0, H, 256)
    _, exact = assert_frames_match(img[rows], ref[rows])
    assert exact == 1.0
    got = np.zeros(4, np.int64)
    for y in rows:
        _, s = gpu_ctx.render(abi.make_params(max_level=8, rect=(0, int(y), W, 1)))
        got += (s.rays_primary, s.rays_shadow, s.rays_reflect, s.rays_refract)
    assert tuple(got) == (sto.rays_primary, sto.rays_shadow, sto.rays_reflect, sto.rays_refract)


@pytest.mark.parametrize("share", [(0, 0), (20, 8), (3, 8)])
def test_device_unpack_eight_ranks(gpu_ctx, avenger_scene, share):
    """The multi-GPU assembly with world 8 on one GPU: every rank's tiles rendered through
    pgrt_render_tiles_device into its slot of a rank-major buffer (exactly pgrt_tile_count_ex
    tiles per rank), unpacked by the device kernel (pgrt_unpack_tiles_device), equal the full
    frame bit for bit -- for the default deal and explicit rank-0 shares above and below 1."""
    from pgi_raytracing_amd.raytracer import lib

    gpu_ctx.set_scene(avenger_scene)
    W, H, world = 700, 450, 8
    gpu_ctx.set_camera(abi.default_camera(W, H))
    p = abi.make_params(max_level=5, spp_side=2, jitter=abi.PGRT_JITTER_HASH, frame=6)
    L = lib()
    old = gpu_ctx.configure(rank0_share_a=share[0], rank0_share_b=share[1])
    counts = [L.pgrt_tile_count_ex(W, H, 64, r, world, *share) for r in range(world)]
    assert sum(counts) == (-(-W // 64)) * (-(-H // 64))
    tile_bytes = 64 * 64 * 16
    g = gpu_ctx.alloc(sum(counts) * tile_bytes)
    fb = gpu_ctx.alloc(W * H * 16)
    try:
        off = 0
        for r in range(world):
            gpu_ctx.render_tiles_device(p, r, world, g + off * tile_bytes)
            off += counts[r]
        gpu_ctx.unpack_tiles_device(W, H, world, share, g, fb)
        out = gpu_ctx.to_host(fb, (H, W, 4))
        ref, _ = gpu_ctx.render(p)
        assert _frames_equal(out, ref)
        assert gpu_ctx.tune_distribution(p, 1, fb) == (1, 1)  # one rank: nothing to tune
    finally:
        gpu_ctx.set_config(old)
        gpu_ctx.free(g)
        gpu_ctx.free(fb)
