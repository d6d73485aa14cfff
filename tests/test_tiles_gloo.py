"""Multi-GPU path on CPU: world_size 2 over gloo.

Each rank renders the 64x64 tiles it owns (the deal of pgrt_tile_count / pgrt_tile_index /
pgrt_tile_rect: rank 0 takes a smaller share, it also unpacks) into a tile-compact buffer, the buffers are gathered on rank 0
(gloo standing in for libpgrt's ncclGather) and unpacked with pgrt_unpack_tiles_host; the result
must equal a single-process full-frame render bit for bit.  The per-tile renders use the CPU
restatement (no GPU here); the device path runs the same plan (tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

W, H, T = 200, 130, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, obj, env, q):
    import ctypes as C
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle")):
        sys.path.insert(0, p)
    import pyoracle
    from pgi_raytracing_amd import abi
    from pgi_raytracing_amd.raytracer import lib, load_obj

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = lib()
    sc = load_obj(obj)
    sc.set_environment(env)
    osc = pyoracle.OracleScene(sc)
    cam = abi.default_camera(W, H)
    counts = [L.pgrt_tile_count(W, H, T, r, world) for r in range(world)]
    per_rank = max(counts)
    mine = [L.pgrt_tile_index(W, H, T, rank, world, j) for j in range(L.pgrt_tile_count(W, H, T, rank, world))]
    buf = np.zeros((per_rank, T, T, 4), np.float32)
    rect = (C.c_int * 4)()
    for j, t in enumerate(mine):
        L.pgrt_tile_rect(W, H, T, t, rect)
        x, y, w, h = rect
        img, _ = osc.render(cam, abi.make_params(max_level=5, spp_side=2, jitter=abi.PGRT_JITTER_HASH,
                                                 rect=(x, y, w, h)), threads=2)
        buf[j, :h, :w] = img
    t_buf = torch.from_numpy(buf.reshape(-1))
    gathered = [torch.zeros_like(t_buf) for _ in range(world)] if rank == 0 else None
    dist.gather(t_buf, gathered, dst=0)
    if rank == 0:
        # rank-major, exactly pgrt_tile_count tiles per rank (the gather pads to equal sizes)
        g = np.ascontiguousarray(np.concatenate([x.numpy().reshape(per_rank, -1)[:counts[r]]
                                                 for r, x in enumerate(gathered)]).reshape(-1))
        out = np.zeros((H, W, 4), np.float32)
        assert L.pgrt_unpack_tiles_host(W, H, T, world, abi.fptr(g), abi.fptr(out.reshape(-1))) == 0
        full, _ = osc.render(cam, abi.make_params(max_level=5, spp_side=2, jitter=abi.PGRT_JITTER_HASH), threads=2)
        q.put(bool((np.nan_to_num(out, nan=3) == np.nan_to_num(full, nan=3)).all()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_tile_gather_matches_full_frame(avenger_obj):
    from conftest import ENV_MAP

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, avenger_obj, ENV_MAP, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
