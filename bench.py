#!/usr/bin/env python3
"""Benchmark of the Whitted trace hot path (BASELINE.json metric: Mrays/s + ms/frame, avenger
1920x1080 Whitted d=5, 1/2/4/8 GPU).

One step = one frame of BASELINE config C2 (avenger-proxy, 1920x1080, 1 spp pinhole, Whitted
depth 5, spherical env map) rendered into an HBM-resident framebuffer (--config C3/C4/C5 select
the other BASELINE configs).  Rays = every closest-hit query (primary + shadow + reflect +
refract).  Frames are submitted in batches of --frames-per-call consecutive frames (one launch
sequence covers all of them, pgrt_render_frames_device_async; every frame is fully traced into
its own framebuffer) with up to --in-flight calls overlapping on the device (throughput =
ms_per_step); the latency of one synchronous frame is reported beside it (frame_latency_ms).

N > 1 GPUs: one process per GPU.  `python bench.py --gpus N` without a launcher environment starts
the N rank processes itself (subprocess, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set; this
parent never touches a GPU); under torch.distributed.run the ranks come from the environment.
64x64 image tiles are dealt to ranks (csrc/tiles.hpp), every rank renders its tiles of the
call's frames, ONE ncclGather (RCCL over xGMI, libpgrt's own communicator) moves them to rank
0, where one kernel unpacks every frame into its framebuffer.  The frame is fixed as N grows
(strong scaling); value = all ranks' rays / the max over ranks of the timed region.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time
from collections import deque

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# one hardware queue per frame in flight (+ the context stream): HIP's default of 4 would make
# frames share queues; read by the HIP runtime at its initialisation, i.e. before libpgrt loads
# (r1i C2, 8 frames per call: 8 queues / 6 in flight 0.197 ms; 12 / 6 0.191; 12 / 8 0.186;
# 16 / 8-14 0.185-0.187).  The GPU boxes export GPU_MAX_HW_QUEUES=4 (HIP's default): raise it.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path.insert(0, os.path.join(ROOT, "tools"))

METRIC = "Mrays/sec + ms/frame, avenger 1920x1080 Whitted d=5, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes: ray in 32 B + hit out 16 B per ray, 64 B per binary BVH
# node visited, 80 B per 8-wide node visited (small queues), 48 B per triangle tested (our
# triangle record: v0|id, e1, e2)
RAY_BYTES, NODE_BYTES, WIDE_NODE_BYTES, TRI_BYTES = 48, 64, 80, 48
# level-0 rays of the packet traversal are generated in registers (k_trace_pkt<GEN>): no 32-B ray
# read; it stores what the level-0 shade reads back -- the 16-B direction (pinhole: origin, tnear
# and medium come from the camera) or origin + direction + medium (36 B, DoF) -- and the 16-B hit
L0_PINHOLE_BYTES, L0_DOF_BYTES = 16 + 16, 36 + 16
# closest-hit launches in the device timeline (pgrt_timeline_enable; abi.TIMELINE_KINDS)
TRACE_KINDS = ("trace_pkt", "trace", "trace_8g", "trace_resume", "trace_shadow", "subtree")
# B_shade per shaded ray / hit / textured hit or env lookup / emitted ray
SHADE_RAY_BYTES, SHADE_HIT_BYTES, SHADE_COLOUR_BYTES = 48, 16, 16
SHADE_ATTR_BYTES, SHADE_TEXEL_BYTES, SHADE_EMIT_BYTES = 64, 12, 48

# BASELINE.json configs (SURVEY.md §8d "Concrete inputs"); C2 is the headline bench line
CONFIGS = {
    "C2": dict(width=1920, height=1080, max_level=5, spp_side=1, dof=0, scene="avenger", in_flight=8),
    # r1h: C3 14.4 / 15.0 / 12.6 ms at 2 / 4 / 6 in flight
    "C3": dict(width=1920, height=1080, max_level=5, spp_side=8, dof=1, scene="avenger"),
    # r2a: 47.4 ms/frame at 6 in flight (32 sample batches per frame, no batch bound)
    "C4": dict(width=3840, height=2160, max_level=5, spp_side=8, dof=1, scene="avenger"),
    # r1h: 23.4 / 23.8 / 22.3 ms at 2 / 4 / 6 in flight
    "C5": dict(width=4096, height=4096, max_level=8, spp_side=1, dof=0, scene="random1m"),
}
# PMC-measured HBM traffic per closest-hit launch of the bench's profiled configuration
# (tools/profile.sh + tools/traffic.py, committed under profiles/)
TRAFFIC = {"C2": "profiles/r6/r6fin3/traffic_C2.json", "C3": "profiles/r6/r6fin/traffic_C3.json",
           "C4": "profiles/r6/r6fin/traffic_C4.json", "C5": "profiles/r6/r6fin3/traffic_C5.json",
           "C2-path": "profiles/r6/r6fin/traffic_C2-path.json"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # frames timed; default for C2 600 x world (N GPUs batch 8 x N frames per call: 75 calls
    # either way, ~10x the 8 calls in flight, so pipeline fill and drain stay a small part of the
    # timed region at every N; r1i C2: 200 frames 0.207 ms/frame, 960 frames 0.186)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--max-level", type=int, default=None)
    ap.add_argument("--spp-side", type=int, default=None)
    ap.add_argument("--dof", type=int, default=None)
    ap.add_argument("--mode", default="whitted", choices=["whitted", "path"],
                    help="render mode: the reference's Whitted trace (the metric) or PGRT_MODE_PATH "
                         "(the README to-do path tracer; a separate workload line)")
    ap.add_argument("--dist-path", action="store_true",
                    help="validation only: the multi-GPU code path (RCCL communicator, distributed frames, "
                         "tuned tile share, gather + unpack) also at world 1")
    ap.add_argument("--frames", default="distinct", choices=["distinct", "identical"],
                    help="distinct (default): every frame gets its own frame index and hash jitter (get_pixel's "
                         "sub-pixel jitter, raytracer.cpp:407-413), so no two frames of the timed region are the same "
                         "image, and every call in flight writes its own framebuffers; identical: the r2 workload "
                         "(no jitter, one framebuffer shared by every call) -- A/B only")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the synchronous-frame latency after the timed region (profiles of the timed calls only)")
    ap.add_argument("--hw-queues", type=int, default=None,
                    help="A/B only: GPU_MAX_HW_QUEUES for this process (default: 16, as the C++ drop-in sets it; "
                         "HIP reads it at its first call, after this)")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the profiled roofline frames (the run profiles/ rocprofv3 summaries are taken of)")
    ap.add_argument("--in-flight", type=int, default=None,
                    help="calls in flight (pgrt_set_frames_in_flight); default 8 for C2, 6 otherwise")
    ap.add_argument("--frames-per-call", type=int, default=None,
                    help="frames per submission (pgrt_render_frames_*_async, 1..64); default for C2 8 x world, "
                         "32 x world (at most 64) for jobs of >= 256 frames per rank; 1 otherwise")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (multi-thread leg)")
    ap.add_argument("--packet-levels", type=int, default=None,
                    help="A/B only: pgrt_config.packet_levels (default AUTO: chosen per level by libpgrt)")
    ap.add_argument("--group-max", type=int, default=None,
                    help="A/B only: pgrt_config.group_max (queues up to it: 8 lanes per ray)")
    ap.add_argument("--remainder-first", action="store_true",
                    help="submit the short call (steps %% frames-per-call frames) first instead of last")
    ap.add_argument("--cfg", action="append", default=[],
                    help="A/B only: pgrt_config field=value (repeatable), e.g. --cfg bvh_width=8")
    a = ap.parse_args()
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    return a


# ------------------------------------------------------------------ rank launcher (N > 1)

def visible_gpus() -> int:
    """GPUs this process may use, without initialising HIP: the *_VISIBLE_DEVICES lists, else the
    KFD topology nodes that have SIMDs (the GPU agents)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(f) as fh:
                props = dict(line.split() for line in fh if len(line.split()) == 2)
            n += int(props.get("simd_count", "0")) > 0
        except (OSError, ValueError):
            pass
    return n


def launch_ranks(n: int) -> int:
    """Start N rank processes of this script (fresh processes: this one never touched a GPU) and
    forward rank 0's stdout; the first failing rank stops the others."""
    have = visible_gpus()
    if have < n:
        print(f"bench.py: --gpus {n} needs {n} GPUs, {have} visible on this node", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:  # the others would wait for the failed rank forever
                    q.terminate()
        time.sleep(0.05)
    return rc


# ------------------------------------------------------------------ CPU baseline

def cpu_share() -> dict:
    """Host cores: the machine's (nproc), this process's affinity mask and the cgroup CPU quota;
    the baseline runs on all cores this process may use."""
    info = {"nproc": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, period = fh.read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    info["cgroup_quota"] = quota
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    info["threads"] = max(1, min(info["affinity"] or 1, int(quota) if quota else 1 << 30))
    return info


def cpu_baseline(args, scene, cam, params):
    """The CPU restatement (oracle/, test infrastructure: timed only here) on the host cores.
    C2: whole frames until the budget is spent; C3-C5: every 16th row."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # cpu_baseline leg only: the checker, timed as the baseline

    share = cpu_share()
    threads = share["threads"]
    t0 = time.perf_counter()
    osc = pyoracle.OracleScene(scene)
    build_s = time.perf_counter() - t0
    row_step = 1 if args.config == "C2" else 16

    def timed(nthreads, budget_s):
        frames = rays_c = 0
        t1 = time.perf_counter()
        while True:
            _, sc = osc.render(cam, params, row_step=row_step, threads=nthreads)
            rays_c += sc.rays()
            frames += 1
            dt_c = time.perf_counter() - t1
            if dt_c >= budget_s:
                return rays_c / dt_c / 1e6, frames, rays_c, dt_c

    # the reference's own per-sample RNG work, reported separately: two wall-clock
    # seeded std::mt19937 per sample (raytracer.cpp:407-410, PinHoleCamera.cpp:77-80), 2 draws each
    import ctypes as C
    ol = pyoracle.lib()
    ol.orc_mt19937_reseed.restype = C.c_uint32
    ol.orc_mt19937_reseed.argtypes = [C.c_int, C.c_uint32]
    n_rs, t_rs = 0, time.perf_counter()
    while time.perf_counter() - t_rs < 0.5:
        ol.orc_mt19937_reseed(20000, n_rs)
        n_rs += 20000
    reseed_us = (time.perf_counter() - t_rs) / n_rs * 1e6
    samples = args.width * args.height * args.spp_side ** 2
    what = "whole C2 frames" if row_step == 1 else f"{args.config} frames, every 16th row"
    v_mt, f_mt, r_mt, t_mt = timed(threads, args.cpu_seconds)
    v_st, f_st, r_st, t_st = timed(1, args.cpu_seconds / 2)
    return {"value": round(v_mt, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{f_mt} x {what} ({r_mt} rays, {t_mt:.1f} s) on {threads} host threads (OpenMP over rows); "
                      f"oracle/ CPU restatement with its own SAH BVH (built in {build_s:.1f} s, not timed)",
            "host": share,
            "reference_rng": {"reseed_us": round(reseed_us, 3), "reseeds_per_sample": 2,
                              "ms_per_frame_1_thread": round(reseed_us * 2 * samples / 1e3, 1),
                              "note": "std::mt19937 seeding + 2 draws, restated in C (oracle/ orc_mt19937_reseed), "
                                      "the reference's per-sample RNG cost on one thread, beside the restatement's "
                                      "deterministic counter hash"},
            "single_thread_value": round(v_st, 3),
            "single_thread_sample": f"{f_st} x {what} ({r_st} rays, {t_st:.1f} s), 1 thread (the reference's "
                                    f"single Producer thread)"}


def workload(args) -> str:
    return (f"{args.config} {'avenger-proxy' if args.scene == 'avenger' else '1M random triangles'} "
            f"{args.width}x{args.height} {'path tracing' if args.mode == 'path' else 'Whitted'} d={args.max_level} "
            f"+ env map, "
            f"{args.spp_side ** 2} spp {'DoF' if args.dof else 'pinhole'}")


# ------------------------------------------------------------------ main

class _stdout_to_stderr:
    """fd 1 -> fd 2 while native libraries initialise: stdout carries only rank 0's JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def main():
    args = parse()
    if args.hw_queues is not None:  # before the first HIP call (Context below)
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.steps is None:
        args.steps = 600 * world if args.config == "C2" else 20
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only; the frame gather is RCCL in libpgrt

        dist.init_process_group("gloo", init_method="env://")
    import scenes
    from pgi_raytracing_amd import abi
    from pgi_raytracing_amd.raytracer import Context, load_obj

    env = os.path.join(ROOT, "assets", "spherical_map_windows.jpg")
    if args.scene == "avenger":
        if rank == 0 and not os.path.exists(scenes.AVENGER_OBJ):
            scenes.write_avenger_proxy()
        if dist:
            dist.barrier()
        scene = load_obj(scenes.AVENGER_OBJ)
        scene.set_environment(env)
        cam = abi.default_camera(args.width, args.height)
    else:  # C5: 10^6 random triangles, camera from (-140,-175,80) at the origin
        scene = scenes.random_scene(1_000_000, 42, env)
        cam = abi.make_camera(args.width, args.height, abi.deg2rad(42.185), (-140.0, -175.0, 80.0), (0.0, 0.0, 0.0))
    distinct = args.frames == "distinct"
    params = abi.make_params(spp_side=args.spp_side, max_level=args.max_level, dof=args.dof,
                             jitter=abi.PGRT_JITTER_HASH if (args.spp_side > 1 or args.dof or distinct)
                             else abi.PGRT_JITTER_NONE,
                             mode=abi.PGRT_MODE_PATH if args.mode == "path" else abi.PGRT_MODE_WHITTED)
    ctx = Context(local_rank)
    if args.packet_levels is not None:
        ctx.configure(packet_levels=args.packet_levels)
    if args.group_max is not None:
        ctx.configure(group_max=args.group_max)
    for kv in args.cfg:
        k, v = kv.split("=", 1)
        ctx.configure(**{k: float(v) if "." in v else int(v)})
    ctx.set_scene(scene)
    ctx.set_camera(cam)
    bvh = ctx.bvh_info()
    # frames per call: ~22 M rays per call per rank (8 C2 frames on 1 GPU, 8 x world frames of a
    # rank's 1/world share at N GPUs); r1e scans: N=1 F=8 0.255 ms/frame (F=16 with 6 in flight
    # 0.39), emulated N=8 rank F=64 0.040 ms/frame (F=16 0.045)
    # (C3/C4/C5 frames are 15-250x heavier than C2's and fill the GPU on their own: 1 per call)
    # A long C2 job (>= 256 frames per rank) goes in calls of 32 frames' worth of rays per rank:
    # fewer, wider launches per frame (r6q, 600 frames: 0.1413 -> 0.1333 ms/frame; 64 per call with
    # 8 in flight does not fit one GPU's memory); a short one keeps 8 so several calls overlap (r6m:
    # the driver's 20 frames in one call 0.183-0.189 vs 0.166 ms/frame in 8 + 8 + 4)
    per_rank = 32 if args.steps >= 256 * world else 8
    F = max(1, min(64, args.frames_per_call or (per_rank * world if args.config == "C2" else 1)))
    # the profiled roofline calls and the host-framebuffer calls keep the short-job size (the
    # committed rocprofv3 traffic is per 8-frame launch; 8 calls of 32 host frames would pin 8.5 GB)
    F_aux = min(F, max(1, min(64, args.frames_per_call or (8 * world if args.config == "C2" else 1))))
    # calls in flight: a step is one whole frame (every rank's tiles rendered, gathered and
    # unpacked on rank 0); up to `in_flight` calls overlap on the device, so one call's
    # latency-bound deep levels share the CUs with the next call's wide levels
    in_flight = args.in_flight or CONFIGS[args.config].get("in_flight", 6)
    call_bytes = F * args.width * args.height * 16
    # distinct frames: one framebuffer set per call in flight (a pending frame's framebuffer is
    # never reused, pgrt.h); call k writes set k % in_flight, which call k - in_flight released
    ring = in_flight if distinct else 1
    fb = ctx.alloc(ring * call_bytes) if rank == 0 or world == 1 else None
    comm_ranks = 1
    distributed = world > 1 or args.dist_path
    if distributed:
        with _stdout_to_stderr():  # RCCL prints its version banner on stdout at init
            uid = [Context.comm_unique_id() if rank == 0 else None]
            if dist:
                dist.broadcast_object_list(uid, src=0)
            ctx.comm_init(world, rank, uid[0])
        comm_ranks, _ = ctx.comm_info()

    def frame(p):  # synchronous frame (latency, profiled frames)
        if distributed:
            return ctx.render_distributed_device(p, fb)
        return ctx.render_device(p, fb)

    ctx.set_frames_in_flight(in_flight)
    gather_ms = []

    next_frame = [0]  # frame index of the next submitted frame (jitter key of distinct frames)

    def run_frames(n, record=False):
        pending, rays_n = deque(), 0

        def wait_one():
            st = ctx.render_wait(pending.popleft())
            if record and distributed:
                gather_ms.append(st.ms_gather)
            return st.rays()

        # call sizes: F frames each, the remainder of n / F either last or (--remainder-first) first
        sizes = [F] * (n // F)
        if n % F:
            sizes = [n % F] + sizes if args.remainder_first else sizes + [n % F]
        for k, nf in enumerate(sizes):
            pc = params
            out = fb
            if distinct:
                pc = abi.RenderParams.from_buffer_copy(params)
                pc.frame = next_frame[0]
                out = fb + (k % ring) * call_bytes if fb else fb
            next_frame[0] += nf
            pending.append(ctx.render_frames_distributed_device_async(pc, nf, out) if distributed
                           else ctx.render_frames_device_async(pc, nf, out))
            if len(pending) >= in_flight:
                rays_n += wait_one()
        while pending:
            rays_n += wait_one()
        return rays_n

    if args.roofline_only:  # the profiled calls below, after two unprofiled ones (AUTO's start frame)
        args.warmup, args.steps = 2 * F, 0
    # untimed set-up (not warm-up): one call of F frames per call slot in flight, so every frame
    # set's queues and framebuffers are allocated before the warm-up and the timed region (a first
    # use would hipMalloc inside the timed calls); then exactly --warmup untimed frames
    setup_frames = 0 if args.roofline_only else in_flight * F
    run_frames(setup_frames)
    run_frames(args.warmup)
    share = None
    if distributed and not args.roofline_only:
        # rank 0's tile share from measured calls (libpgrt collective): its rendering against the
        # xGMI gather it receives and the unpack it runs
        share = ctx.tune_distribution(params, F, fb, calls=4)
    ctx.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    rays = run_frames(args.steps, record=True)
    ctx.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    # frame latency (one synchronous frame at a time, the reference's Producer loop,
    # simpleguidx11.cpp:95-124), reported beside the throughput: the context set up for it --
    # one frame in flight, so a frame gets the two pipeline slots and the deep-tiles-first deal
    # (pgrt_config.tile_order), which needs one earlier frame of the same size (2 warm-ups)
    lat = []
    ctx.set_frames_in_flight(1)
    for k in range(0 if args.no_latency else min(args.steps, 30) + 2):
        t1 = time.perf_counter()
        frame(params)
        if k >= 2:
            lat.append(time.perf_counter() - t1)
    ctx.set_frames_in_flight(in_flight)
    latency_ms = sorted(lat)[len(lat) // 2] * 1e3 if lat else None
    total_rays = rays
    per_rank_ms = [elapsed / max(1, args.steps) * 1e3]
    if dist:
        g = [None] * world
        dist.all_gather_object(g, {"elapsed": elapsed, "rays": rays, "latency_ms": latency_ms})
        per_rank_ms = [x["elapsed"] / max(1, args.steps) * 1e3 for x in g]
        elapsed = max(x["elapsed"] for x in g)  # max over ranks
        total_rays = sum(x["rays"] for x in g)
        latency_ms = max(x["latency_ms"] or 0.0 for x in g)

    roof = None
    if not args.no_roofline:
        # live per-kernel timing: HIP events on libpgrt's own stream around every closest-hit
        # launch (profile=1), and the instrumented traversal counts (profile=2, separate call)
        # (1 GPU: the timed configuration, F frames per launch sequence; N GPUs: one frame)
        def prof_call(p):
            return ctx.render_frames_device(p, F_aux, fb) if world == 1 else frame(p)

        frames_per_prof = F_aux if world == 1 else 1
        # level 0 on packets generates its rays in registers (k_trace_pkt<GEN>): 16-B direction
        # write instead of a 32-B ray read.  Whether it did is read off the launch timeline of one
        # unprofiled call of the same configuration (packets can be off by --packet-levels, --cfg
        # packet_levels / bvh_width, or a BVH too deep for the packet stack).  Before the profiled
        # calls: tools/traffic.py takes the calls ahead of the last (profile=2) one
        ctx.timeline_enable(True)
        try:
            prof_call(params)
            l0_kinds = {r["kind"] for r in ctx.timeline_read()
                        if r["level"] == 0 and r["waves"] > 0 and r["kind"] in TRACE_KINDS}
        finally:
            ctx.timeline_enable(False)
        p1 = abi.RenderParams.from_buffer_copy(params)
        p1.profile = 1
        reps = 5 if args.config == "C2" else 2
        ms_trace = 0.0
        launches = 0
        for _ in range(reps):
            s1 = prof_call(p1)
            ms_trace += s1.ms_trace
            launches += s1.trace_launches
        p1.profile = 2
        s2 = prof_call(p1)
        frame_rays = s2.rays()
        fused_l0 = "trace_pkt" in l0_kinds
        l0_bytes = (L0_DOF_BYTES if args.dof else L0_PINHOLE_BYTES) if fused_l0 else RAY_BYTES
        alg_bytes = (RAY_BYTES * (frame_rays - s2.rays_primary) + l0_bytes * s2.rays_primary
                     + NODE_BYTES * s2.node_visits + WIDE_NODE_BYTES * s2.wide_node_visits + TRI_BYTES * s2.tri_tests)
        avg_launch_ms = ms_trace / max(1, launches)
        per_launch_bytes = alg_bytes / max(1, launches / reps)
        achieved = per_launch_bytes / (avg_launch_ms * 1e-3) / 1e9
        roof = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": "closest hit: k_trace_pkt (wave packets; level 0 generates its rays) + k_trace / k_trace8g "
                      "(one / 8 lanes per ray: deeper levels, the shadow queue)",
            "avg_launch_ms": round(avg_launch_ms, 4),
            "frames_per_launch": frames_per_prof,
            "launches_per_call": launches // reps,
            "trace_ms_per_frame": round(ms_trace / reps / frames_per_prof, 4),
            "node_visits_per_ray": round(s2.node_visits / max(1, frame_rays), 2),
            "wide_node_visits_per_ray": round(s2.wide_node_visits / max(1, frame_rays), 2),
            "tri_tests_per_ray": round(s2.tri_tests / max(1, frame_rays), 2),
            "bytes_per_ray": round(alg_bytes / max(1, frame_rays), 1),
            "level0_bytes_per_ray": l0_bytes,
            "level0_kernels": sorted(l0_kinds),
            "timing": "HIP events around every closest-hit launch of " + str(reps) + " profile=1 calls of "
                      + str(frames_per_prof) + " frame(s), synchronous (rocprofv3 trace of exactly these calls: "
                      "tools/profile.sh + tools/traffic.py)",
        }
        if world == 1 and args.steps:
            # the closest-hit launches in the TIMED configuration (calls of F frames, `in_flight` of
            # them in flight): the device-stamped launch timeline of a separate run of such calls;
            # the union of the closest-hit launches' wave spans is the time closest-hit kernels
            # occupy the device per frame (<= the frame time by construction)
            ncalls = max(2 * in_flight, min(max(1, args.steps // F), 4 * in_flight))
            ctx.timeline_enable(True)
            try:
                run_frames(ncalls * F)
                recs = ctx.timeline_read()
            finally:
                ctx.timeline_enable(False)
            recs = [r for r in recs if r["waves"] > 0]  # (a "dropped" marker: stamp buffer full)
            iv = sorted((r["us_start"], r["us_end"]) for r in recs if r["kind"] in TRACE_KINDS)
            busy, cur = 0.0, None
            for a, b in iv:
                if cur is None or a > cur[1]:
                    if cur:
                        busy += cur[1] - cur[0]
                    cur = [a, b]
                else:
                    cur[1] = max(cur[1], b)
            if cur:
                busy += cur[1] - cur[0]
            span = (max(r["us_end"] for r in recs) - min(r["us_start"] for r in recs)) if recs else 0.0
            nfr = ncalls * F
            if busy > 0:
                busy_ms = busy / 1e3 / nfr
                ta = alg_bytes / frames_per_prof / (busy_ms * 1e-3) / 1e9
                roof["timed"] = {
                    "achieved": round(ta, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ta / HBM_PEAK_GBS, 4),
                    "trace_busy_ms_per_frame": round(busy_ms, 4), "span_ms_per_frame": round(span / 1e3 / nfr, 4),
                    "frames": nfr, "calls": ncalls, "frames_per_call": F, "in_flight": in_flight,
                    "note": "closest-hit bytes per frame over the union of the closest-hit launches' wave spans "
                            "(device timeline, pgrt_timeline_enable) while calls of the timed configuration run "
                            "in flight -- a separate run with the stamps on (busy <= its own span per frame; "
                            "capped at ms_per_step if it exceeds the unstamped line's frame time)",
                }
        if args.mode == "whitted":
            # whole-frame algorithmic bytes (B = 32 + 16 + 64 N_node + 36 N_tri + B_shade)
            # over the timed region's ms per frame: the closest-hit bytes above (every level and the
            # shadow queue) plus B_shade per shaded ray (every primary / reflection / refraction ray
            # is shaded once, raytracer.cpp:241-393): ray + meta 48, hit 16, colour record 16; per
            # hit the 64-B attribute record (n0 n1 n2 uv0 uv1 uv2 + material, rtcInterpolate0 and
            # the geometry user data); 12 B of texel taps per textured hit and per environment
            # lookup (every miss, SphericalMap::get_texel); 48 B per emitted child / shadow ray
            shaded = s2.rays_primary + s2.rays_reflect + s2.rays_refract
            misses = shaded - s2.shade_hits
            emitted = s2.rays_reflect + s2.rays_refract + s2.rays_shadow
            shade_bytes = ((SHADE_RAY_BYTES + SHADE_HIT_BYTES + SHADE_COLOUR_BYTES) * shaded
                           + SHADE_ATTR_BYTES * s2.shade_hits + SHADE_TEXEL_BYTES * (s2.shade_textured_hits + misses)
                           + SHADE_EMIT_BYTES * emitted)
            frame_bytes = (alg_bytes + shade_bytes) / frames_per_prof
            ms_frame = elapsed / max(1, args.steps) * 1e3 if args.steps else None
            if ms_frame:
                fa = frame_bytes / (ms_frame * 1e-3) / 1e9
                roof["frame"] = {
                    "achieved": round(fa, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(fa / HBM_PEAK_GBS, 4),
                    "bytes_per_frame": int(frame_bytes),
                    "trace_bytes_per_frame": int(alg_bytes / frames_per_prof),
                    "shade_bytes_per_frame": int(shade_bytes / frames_per_prof),
                    "ms_per_frame": round(ms_frame, 4),
                    "shaded_rays_per_frame": int(shaded / frames_per_prof),
                    "hits_per_frame": int(s2.shade_hits / frames_per_prof),
                    "textured_hits_per_frame": int(s2.shade_textured_hits / frames_per_prof),
                    "note": "SURVEY 8(d) B incl. B_shade (ray+meta 48, hit 16, colour 16 per shaded ray; attributes 64 "
                            "per hit; texel taps 12 per textured hit and per env lookup; 48 per emitted child/shadow "
                            "ray) over the timed region's ms per frame (every kernel of the frame, overlapped)",
                }
        tkey = args.config if args.mode == "whitted" else f"{args.config}-path"
        tf = os.path.join(ROOT, TRAFFIC.get(tkey, "-"))
        if world == 1 and os.path.exists(tf):
            with open(tf) as fh:
                t = json.load(fh)
            roof["traffic"] = t.get("bytes_per_launch")
            roof["traffic_source"] = f"{TRAFFIC[tkey]} ({t.get('round')}; FETCH_SIZE x2 + WRITE_SIZE per launch)"
            roof["traffic_frac"] = round(roof["traffic"] / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            if t.get("frame") and roof.get("frame"):  # whole-frame DRAM bytes (every kernel of the call)
                fb = t["frame"]["bytes_per_frame"]
                roof["frame"]["traffic"] = fb
                roof["frame"]["traffic_frac"] = round(fb / (roof["frame"]["ms_per_frame"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                roof["frame"]["traffic_by_kernel"] = t["frame"].get("by_kernel_bytes_per_frame")
            if t.get("valu_issue"):
                roof["valu_issue"] = t["valu_issue"]
                roof["valu_issue_note"] = t.get("valu_issue_note")

        # consistency rule (verdict r5 #5): the headline frac's closest-hit time per frame must not
        # exceed the timed region's ms per frame.  The synchronous profiled calls run one call alone,
        # so when the timed calls in flight overlap their levels (C3-C5: one frame per call) the
        # synchronous launch time per frame can exceed ms_per_step; the headline then is the timed
        # configuration's figure (device timeline), and the synchronous HIP-event figure (which the
        # committed rocprofv3 averages match) stays under "sync"
        ms_step = elapsed / max(1, args.steps) * 1e3 if args.steps else None
        tm = roof.get("timed")
        if tm and ms_step and tm["trace_busy_ms_per_frame"] > ms_step:
            # the stamped run is a little slower than the timed one (C5: busy 15.80 vs 15.62 ms per
            # frame): the closest-hit launches of a frame cannot be busy longer than the frame, so the
            # denominator is capped at ms_per_step -- a lower bound of the unstamped run's achieved
            # rate (its true busy time is <= ms_per_step)
            ta = tm["achieved"] * tm["trace_busy_ms_per_frame"] / ms_step
            tm["measured_busy_ms_per_frame"] = tm["trace_busy_ms_per_frame"]
            tm["trace_busy_ms_per_frame"] = round(ms_step, 4)
            tm["achieved"], tm["frac"] = round(ta, 1), round(ta / HBM_PEAK_GBS, 4)
            tm["busy_capped"] = "the stamped run's busy time per frame exceeded ms_per_step: capped at it"
        roof["sync"] = {k: roof[k] for k in ("achieved", "frac", "avg_launch_ms", "trace_ms_per_frame")}
        roof["frac_source"] = "sync"
        if ms_step and roof["trace_ms_per_frame"] > ms_step and roof.get("timed"):
            roof["achieved"], roof["frac"] = roof["timed"]["achieved"], roof["timed"]["frac"]
            roof["frac_source"] = "timed"
        roof["frac_source_note"] = (
            "sync: algorithmic closest-hit bytes per launch / HIP-event launch time of synchronous profile=1 calls; "
            "timed: closest-hit bytes per frame / busy time of the closest-hit launches in the timed configuration "
            "(used when the synchronous closest-hit time per frame exceeds ms_per_step)")

    if args.roofline_only:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "config": args.config, "workload": workload(args), "roofline": roof}),
                  flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    host = None
    if world == 1 and not args.no_roofline:
        # host-framebuffer figures (PCIe-inclusive; never the headline value).  SURVEY §8(d)'s
        # ms/frame: pgrt_render from camera upload to the framebuffer on the host, median of >= 10
        # frames after 2 warm-ups (into page-locked memory, as a D3D upload heap would be);
        # throughput: pgrt_render_frames_host_async, F_aux frames per call, their D2H copy (W*H*16 B
        # per frame) queued behind them and overlapped with the calls in flight
        fb_host = ctx.host_array((args.height, args.width, 4))
        try:
            ctx.set_frames_in_flight(1)  # synchronous frames: as the latency above
            for _ in range(2):
                ctx.render(params, out=fb_host)
            lat_h = []
            for _ in range(max(10, min(args.steps, 30))):
                t1 = time.perf_counter()
                ctx.render(params, out=fb_host)
                lat_h.append(time.perf_counter() - t1)
        finally:
            ctx.set_frames_in_flight(in_flight)
            ctx.host_free(fb_host)
        ring = min(in_flight, 4)
        bufs = [ctx.host_array((F_aux, args.height, args.width, 4)) for _ in range(ring)]
        try:
            ctx.set_frames_in_flight(ring)
            calls = max(2 * ring, 96 // F_aux)

            def host_calls(n):
                pend = deque()
                for k in range(n):
                    pend.append(ctx.render_frames_host_async(params, F_aux, bufs[k % ring]))
                    if len(pend) >= ring:
                        ctx.render_wait(pend.popleft())
                while pend:
                    ctx.render_wait(pend.popleft())

            host_calls(ring)
            t1 = time.perf_counter()
            host_calls(calls)
            dt = time.perf_counter() - t1
        finally:
            ctx.set_frames_in_flight(in_flight)
            for b in bufs:
                ctx.host_free(b)
        fb_bytes = args.width * args.height * 16
        host = {
            "ms_per_frame_sync_median": round(sorted(lat_h)[len(lat_h) // 2] * 1e3, 4),
            "ms_per_frame_async": round(dt / (calls * F_aux) * 1e3, 4),
            "async_frames": calls * F_aux,
            "async_calls_in_flight": ring,
            "frame_bytes": fb_bytes,
            "pcie_d2h_gbs": round(calls * F_aux * fb_bytes / dt / 1e9, 2),
            "note": "sync: SURVEY 8(d) definition (pgrt_render into a page-locked host framebuffer, median of "
                    f"{len(lat_h)} after 2 warm-ups); async: pgrt_render_frames_host_async throughput, bound by "
                    "the device-to-host copy of W*H*16 B per frame",
        }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, scene, cam, params)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(total_rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "setup_frames": setup_frames,
            "setup_note": "untimed set-up before the warm-up: one call of frames_per_call frames per call slot in "
                          "flight, so every frame set is allocated before the timed region (not counted as warm-up)",
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "frames_in_flight": in_flight,
            "frames_per_call": F,
            "frame_latency_ms": round(latency_ms, 4) if latency_ms else None,
            "higher_is_better": True,
            "frames_distinct": distinct,
            "frames_note": ("every frame its own frame index and hash jitter (get_pixel's sub-pixel jitter), every call "
                            "in flight its own framebuffers" if distinct else
                            "identical frames (no jitter) into one shared framebuffer: A/B only"),
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic: avenger-proxy OBJ (reference OBJ absent) + spherical_map_windows.jpg"
                     if args.scene == "avenger" else "synthetic: 10^6 random triangles (seed 42) + env map"),
            "config": {
                "workload": workload(args),
                "triangles": bvh.num_triangles,
                "rays_per_frame": int(total_rays / args.steps),
                "parallelism": f"image tiles 64x64 over {world} GPU(s), ncclGather to rank 0" if world > 1
                else "1 GPU",
            },
            "world": world,
            "rccl_ranks": comm_ranks,
            "per_rank_ms_per_step": [round(x, 4) for x in per_rank_ms],
            "gather_ms_per_call": round(sum(gather_ms) / len(gather_ms), 4) if gather_ms else None,
            "rank0_share": f"{share[0]}/{share[1]}" if share else None,
            "roofline": roof,
            "host_framebuffer_ms_per_step": host["ms_per_frame_sync_median"] if host else None,
            "host_framebuffer": host,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
