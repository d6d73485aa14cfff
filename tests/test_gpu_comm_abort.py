"""Rank 0's bounded wait for the peers' tiles (csrc/distributed.cpp rank0_await_peers).

A peer that died or never submitted a distributed frame would leave rank 0's ncclRecv pending on
the context stream forever.  The wait is bounded by pgrt_config.peer_wait_ms; when it runs out the
communicator is aborted (ncclCommAbort), the call returns PGRT_ERR_RCCL, every later distributed
call fails at once, frames that are not distributed still render, and pgrt_destroy returns.

Two forms:
* one GPU (runs on the pool's boxes): rank 0 of an emulated world of 2 (PGRT_EMULATE_RANK=0/2)
  with the diagnostics stall PGRT_DEBUG_PEER_STALL=1, which takes the same timeout / abort path
  without a communicator (one GPU cannot host a world-2 RCCL communicator);
* two GPUs (skipped on one): a real world-2 RCCL communicator whose rank 1 initialises and then
  never submits, so rank 0's ncclRecv stays pending until the wait runs out and the abort ends it.

Each runs in child processes (the environment switches are read once per process) under a time
limit, so a regression shows up as a failure instead of a hung suite.
"""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, %r)
    sys.path.insert(0, os.path.join(%r, "tools"))
    import scenes
    from pgi_raytracing_amd import abi
    from pgi_raytracing_amd.raytracer import Context, PgrtError, load_obj
    if not os.path.exists(scenes.AVENGER_OBJ):
        scenes.write_avenger_proxy()
    scene = load_obj(scenes.AVENGER_OBJ)
    W, H = 256, 128
    cam = abi.default_camera(W, H)
    p = abi.make_params(max_level=3)
""" % (ROOT, ROOT))

ONE_GPU = PRELUDE + textwrap.dedent("""
    ctx = Context(0)
    ctx.set_scene(scene)
    ctx.set_camera(cam)
    ctx.configure(peer_wait_ms=300)
    fb = ctx.alloc(W * H * 16)
    t0 = time.time()
    try:
        ctx.render_distributed_device(p, fb)
        raise SystemExit("the distributed frame returned although no peer sent its tiles")
    except PgrtError as e:
        assert e.code == abi.PGRT_ERR_RCCL, e
        assert "communicator aborted" in str(e), e
    waited = time.time() - t0
    assert 0.25 <= waited < 30, waited
    t0 = time.time()
    for call in (lambda: ctx.render_distributed_device(p, fb),
                 lambda: ctx.render_frames_distributed_device_async(p, 2, fb)):
        try:
            call()
            raise SystemExit("a distributed call after the abort returned")
        except PgrtError as e:
            assert e.code == abi.PGRT_ERR_RCCL and "was aborted" in str(e), e
    assert time.time() - t0 < 0.25, "later distributed calls must fail at once"
    img, st = ctx.render(p)  # a frame that is not distributed still renders
    assert st.rays_primary == W * H
    ctx.free(fb)
    t0 = time.time()
    ctx.close()
    assert time.time() - t0 < 15
    print("OK")
""")

TWO_GPU = PRELUDE + textwrap.dedent("""
    rank = int(sys.argv[1])
    uid_path = sys.argv[2]
    if rank == 0:
        uid = Context.comm_unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(uid_path + ".tmp", uid_path)
    else:
        while not os.path.exists(uid_path):
            time.sleep(0.05)
        uid = open(uid_path, "rb").read()
    ctx = Context(rank)
    ctx.set_scene(scene)
    ctx.set_camera(cam)
    ctx.comm_init(2, rank, uid)
    if rank == 1:  # initialised, then never submits: rank 0's receive has no sender
        while not os.path.exists(uid_path + ".done"):
            time.sleep(0.05)
        os._exit(0)
    ctx.configure(peer_wait_ms=2000)
    fb = ctx.alloc(W * H * 16)
    t0 = time.time()
    try:
        ctx.render_distributed_device(p, fb)
        raise SystemExit("the distributed frame returned although rank 1 never sent")
    except PgrtError as e:
        assert e.code == abi.PGRT_ERR_RCCL and "communicator aborted" in str(e), e
    assert time.time() - t0 < 60
    try:
        ctx.render_distributed_device(p, fb)
        raise SystemExit("a distributed call after the abort returned")
    except PgrtError as e:
        assert e.code == abi.PGRT_ERR_RCCL and "was aborted" in str(e), e
    t0 = time.time()
    ctx.close()
    assert time.time() - t0 < 15
    open(uid_path + ".done", "w").close()
    print("OK")
""")


def _env(**kw):
    env = dict(os.environ)
    env.update(kw)
    return env


@pytest.mark.gpu
def test_peer_wait_times_out_and_aborts_one_gpu():
    r = subprocess.run([sys.executable, "-c", ONE_GPU], capture_output=True, text=True, timeout=240,
                       env=_env(PGRT_EMULATE_RANK="0/2", PGRT_DEBUG_PEER_STALL="1"))
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_peer_never_submits_world2_rccl(tmp_path):
    from pgi_raytracing_amd.raytracer import device_count

    if device_count() < 2:
        pytest.skip("a world-2 RCCL communicator needs two GPUs (this box has one)")
    uid = str(tmp_path / "uid")
    procs = [subprocess.Popen([sys.executable, "-c", TWO_GPU, str(r), uid], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True, env=_env(HIP_VISIBLE_DEVICES="0,1"))
             for r in (0, 1)]
    outs = []
    try:
        for pr in procs:
            outs.append(pr.communicate(timeout=240))
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
    assert procs[0].returncode == 0 and "OK" in outs[0][0], outs[0][0][-2000:] + outs[0][1][-2000:]
    assert procs[1].returncode == 0, outs[1][1][-2000:]
