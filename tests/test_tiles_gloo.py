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


# ---- the overflow protocol of distributed frames, world 3 over gloo ----
# Each rank sends its tiles plus the two-int tail pgrt_gather_tail forms (flag, frame sequence);
# rank 0 reads the tails with pgrt_gather_tail_verdict -- the function collect_frame runs -- and
# receives again only from the ranks it names, which re-send on their own (no message from rank 0,
# as in libpgrt).  Tile pixels are synthetic (a function of the global tile index and the frame): a
# rank whose queues "overflow" first sends a damaged render.  Scenarios per frame: all good; rank 2
# overflows once; ranks 1 and 2 overflow (rank 2 twice); rank 1 sends the tiles of another frame
# (PGRT_ERR_RCCL at rank 0); rank 2 gives up (poison: PGRT_ERR_OUT_OF_MEMORY at rank 0).
PW, PH = 300, 200
SCENARIOS = [  # (frame sequence, {rank: overflowing attempts}, {rank: sequence it sends}, poisoned rank)
    (1, {}, {}, None),
    (2, {2: 1}, {}, None),
    (3, {1: 1, 2: 2}, {}, None),
    (4, {}, {1: 5}, None),
    (5, {2: 1}, {}, 2),
]


def _tile_pixels(t, seq, damaged=False):
    rng = np.random.default_rng(1000 * t + seq)
    px = rng.random((T, T, 4), dtype=np.float32)
    if damaged:
        px[::3] = -1.0
    return px


def _protocol_worker(rank, world, port, q):
    import ctypes as C
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from pgi_raytracing_amd import abi
    from pgi_raytracing_amd.raytracer import lib

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    L = lib()
    counts = [L.pgrt_tile_count(PW, PH, T, r, world) for r in range(world)]
    tiles = [[L.pgrt_tile_index(PW, PH, T, r, world, j) for j in range(counts[r])] for r in range(world)]

    def send_buf(r, seq, damaged, poison, sent_seq):
        px = np.stack([_tile_pixels(t, seq, damaged) for t in tiles[r]]).reshape(-1)
        tail = (C.c_int * 2)()
        assert L.pgrt_gather_tail(int(damaged), int(poison), sent_seq, tail) == 0
        return np.concatenate([px, np.array([tail[0], tail[1]], np.int32).view(np.float32)])

    results = []
    for seq, overflow, wrong_seq, poisoned in SCENARIOS:
        if rank != 0:
            bad = overflow.get(rank, 0)
            sent = wrong_seq.get(rank, seq)
            if poisoned == rank:  # every attempt overflows; after the last it sends with the poison flag
                dist.send(torch.from_numpy(send_buf(rank, seq, True, True, sent)), 0)
            else:
                for attempt in range(bad + 1):  # damaged renders first, then the good one
                    dist.send(torch.from_numpy(send_buf(rank, seq, attempt < bad, False, sent)), 0)
            continue
        gathered = {0: np.stack([_tile_pixels(t, seq) for t in tiles[0]]).reshape(-1)}
        pending = list(range(1, world))
        status, rounds = 0, 0
        while pending:
            flags = (C.c_int * world)()
            seqs = (C.c_uint * world)()
            for r in pending:
                buf = torch.zeros(counts[r] * T * T * 4 + 2)
                dist.recv(buf, r)
                b = buf.numpy()
                gathered[r] = b[:-2].copy()
                flags[r], seqs[r] = (int(v) for v in b[-2:].view(np.int32))
            regather = (C.c_int * world)()
            badr = C.c_int(-1)
            status = L.pgrt_gather_tail_verdict(flags, seqs, world, seq, regather, C.byref(badr))
            if status != 0:
                break
            pending = [r for r in range(1, world) if regather[r]]
            rounds += 1
        if status != 0:
            results.append((seq, status, badr.value, rounds, None))
            continue
        g = np.concatenate([gathered[r] for r in range(world)])
        out = np.zeros((PH, PW, 4), np.float32)
        assert L.pgrt_unpack_tiles_host(PW, PH, T, world, abi.fptr(g), abi.fptr(out.reshape(-1))) == 0
        expect = np.zeros_like(out)
        rect = (C.c_int * 4)()
        for r in range(world):
            for t in tiles[r]:
                L.pgrt_tile_rect(PW, PH, T, t, rect)
                x, y, w, h = rect
                expect[y:y + h, x:x + w] = _tile_pixels(t, seq)[:h, :w]
        results.append((seq, status, -1, rounds, bool((out == expect).all())))
    if rank == 0:
        q.put(results)
    dist.barrier()
    dist.destroy_process_group()


def test_three_rank_overflow_protocol():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_protocol_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = {seq: rest for seq, *rest in q.get(timeout=5)}
    PGRT_ERR_RCCL, PGRT_ERR_OOM = -6, -3
    assert res[1] == [0, -1, 1, True]            # one round, frame exact
    assert res[2] == [0, -1, 2, True]            # rank 2 received again
    assert res[3] == [0, -1, 3, True]            # rank 1 once more, rank 2 twice more
    assert res[4][:2] == [PGRT_ERR_RCCL, 1]      # rank 1 sent frame 5's tiles at frame 4
    assert res[5][:2] == [PGRT_ERR_OOM, 2]       # rank 2 gave up (poison), rank 0 fails too


def test_gather_tail_abi_edges():
    import ctypes as C

    from pgi_raytracing_amd.raytracer import lib

    L = lib()
    tail = (C.c_int * 2)()
    assert L.pgrt_gather_tail(0, 0, 7, tail) == 0 and list(tail) == [0, 7]
    assert L.pgrt_gather_tail(1, 0, 7, tail) == 0 and list(tail) == [1, 7]
    assert L.pgrt_gather_tail(1, 1, 7, tail) == 0 and list(tail) == [2, 7]
    assert L.pgrt_gather_tail(0, 0, 0, tail) < 0  # sequence numbers start at 1
    flags = (C.c_int * 4)(9, 0, 1, 0)
    seqs = (C.c_uint * 4)(0, 3, 3, 0)  # rank 3 not received in this gather; rank 0's entry ignored
    reg = (C.c_int * 4)()
    bad = C.c_int(-5)
    assert L.pgrt_gather_tail_verdict(flags, seqs, 4, 3, reg, C.byref(bad)) == 0
    assert list(reg) == [0, 0, 1, 0] and bad.value == -1
    assert L.pgrt_gather_tail_verdict(flags, seqs, 4, 0, reg, C.byref(bad)) < 0
    assert L.pgrt_gather_tail_verdict(flags, seqs, 0, 3, reg, C.byref(bad)) < 0
