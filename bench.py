#!/usr/bin/env python3
"""Benchmark of the Whitted trace hot path (BASELINE.json metric: Mrays/s + ms/frame, avenger
1920x1080 Whitted d=5, 1/2/4/8 GPU).

One step = one frame of BASELINE config C2 (avenger-proxy, 1920x1080, 1 spp pinhole, Whitted
depth 5, spherical env map) rendered into an HBM-resident framebuffer (--config C3/C4/C5 select
the other BASELINE configs for the records in DESIGN.md).  N > 1: one process
per GPU (torch.distributed launcher env), 64x64 image tiles dealt round-robin to ranks, one
ncclGather (RCCL over xGMI) to rank 0 and an unpack kernel there -- the total frame is fixed
(strong scaling).  Rays = every closest-hit query (primary + shadow + reflect + refract).
Frames are submitted in batches of --frames-per-call consecutive frames (one launch sequence
covers all of them, pgrt_render_frames_device_async; every frame is fully traced into its own
framebuffer) with up to --in-flight calls overlapping on the device (throughput = ms_per_step);
the latency of one synchronous frame is reported beside it (frame_latency_ms).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import deque

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# one hardware queue per frame in flight (+ the context stream): HIP's default of 4 would make
# frames share queues; read by the HIP runtime at its initialisation, i.e. before libpgrt loads
# (r1i C2, 8 frames per call: 8 queues / 6 in flight 0.197 ms; 12 / 6 0.191; 12 / 8 0.186;
# 16 / 8-14 0.185-0.187)
# (the GPU boxes export GPU_MAX_HW_QUEUES=4, HIP's default: raise it, a setdefault would not)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path.insert(0, os.path.join(ROOT, "tools"))

METRIC = "Mrays/sec + ms/frame, avenger 1920x1080 Whitted d=5, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic bytes: ray in 32 B + hit out 16 B per ray, 64 B per binary BVH
# node visited, 80 B per 8-wide node visited (small queues), 48 B per triangle tested (our
# triangle record: v0|id, e1, e2)
RAY_BYTES, NODE_BYTES, WIDE_NODE_BYTES, TRI_BYTES = 48, 64, 80, 48


# BASELINE.json configs (SURVEY.md §8d "Concrete inputs"); C2 is the headline bench line, the
# others are measured with --config and recorded in DESIGN.md / profiles/
CONFIGS = {
    "C2": dict(width=1920, height=1080, max_level=5, spp_side=1, dof=0, scene="avenger", in_flight=8),
    # (r1h after the counter-zeroing fix: C3 14.4 / 15.0 / 12.6 ms at 2 / 4 / 6 in flight)
    "C3": dict(width=1920, height=1080, max_level=5, spp_side=8, dof=1, scene="avenger"),
    "C4": dict(width=3840, height=2160, max_level=5, spp_side=8, dof=1, scene="avenger"),
    # r1h: 23.4 / 23.8 / 22.3 ms at 2 / 4 / 6 in flight
    "C5": dict(width=4096, height=4096, max_level=8, spp_side=1, dof=0, scene="random1m"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # frames timed; default 600 x world (N GPUs batch 8 x N frames per call: 75 calls either way,
    # ~10x the 8 calls in flight, so pipeline fill and drain stay a small part of the timed region
    # at every N; r1i C2: 200 frames 0.207 ms/frame, 960 frames 0.186)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--max-level", type=int, default=None)
    ap.add_argument("--spp-side", type=int, default=None)
    ap.add_argument("--dof", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the profiled roofline frames (the run profiles/ rocprofv3 summaries are taken of)")
    ap.add_argument("--in-flight", type=int, default=None,
                    help="frames in flight (pgrt_set_frames_in_flight); default 6 (r1 scan, tools/inflight_scan.py)")
    ap.add_argument("--frames-per-call", type=int, default=None,
                    help="frames per submission (pgrt_render_frames_*_async, 1..64); default 8 x world for C2, 1 otherwise (r1e scans)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget (multi-thread leg)")
    a = ap.parse_args()
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k, None) is None:
            setattr(a, k, v)
    return a


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.steps is None:
        args.steps = 600 * world
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
    params = abi.make_params(spp_side=args.spp_side, max_level=args.max_level, dof=args.dof,
                             jitter=abi.PGRT_JITTER_HASH if (args.spp_side > 1 or args.dof) else abi.PGRT_JITTER_NONE)
    ctx = Context(local_rank)
    ctx.set_scene(scene)
    ctx.set_camera(cam)
    bvh = ctx.bvh_info()
    # frames per call: ~22 M rays per call per rank (8 C2 frames on 1 GPU, 8 x world frames of a
    # rank's 1/world share at N GPUs); r1e scans: N=1 F=8 0.255 ms/frame (F=16 with 6 in flight
    # 0.39), emulated N=8 rank F=64 0.040 ms/frame (F=16 0.045)
    # (C3/C4/C5 frames are 15-80x heavier than C2's and fill the GPU on their own: 1 per call)
    F = max(1, min(64, args.frames_per_call or (8 * world if args.config == "C2" else 1)))
    fb = ctx.alloc(F * args.width * args.height * 16) if rank == 0 or world == 1 else None
    if world > 1:
        uid = [Context.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])

    def frame(p):  # synchronous frame (latency, profiled frames)
        if world > 1:
            return ctx.render_distributed_device(p, fb)
        return ctx.render_device(p, fb)

    # frames in flight: a step is one whole frame (every rank's tiles rendered, gathered and
    # unpacked on rank 0); up to `in_flight` consecutive frames overlap on the device, so one
    # frame's latency-bound deep levels share the CUs with the next frame's wide levels
    # (r1g measured C5 at 175 ms/frame with 6 in flight: a new frame set's counters were zeroed
    # by a NULL-stream hipMemset racing the slot streams, fixed in r1h)
    in_flight = args.in_flight or CONFIGS[args.config].get("in_flight", 6)
    ctx.set_frames_in_flight(in_flight)

    def run_frames(n):
        pending, rays_n = deque(), 0
        for f0 in range(0, n, F):
            nf = min(F, n - f0)
            pending.append(ctx.render_frames_distributed_device_async(params, nf, fb) if world > 1
                           else ctx.render_frames_device_async(params, nf, fb))
            if len(pending) >= in_flight:
                rays_n += ctx.render_wait(pending.popleft()).rays()
        while pending:
            rays_n += ctx.render_wait(pending.popleft()).rays()
        return rays_n

    if args.roofline_only:
        args.warmup = args.steps = 0
    if not args.roofline_only:  # every frame set is allocated and warm before the timed region
        args.warmup = max(args.warmup, in_flight * F)
    run_frames(args.warmup)
    ctx.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    rays = run_frames(args.steps)
    ctx.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # frame latency (one synchronous frame at a time), reported beside the throughput
    lat = [0.0]
    for _ in range(min(args.steps, 30)):
        t1 = time.perf_counter()
        frame(params)
        lat.append(time.perf_counter() - t1)
    lat = lat[1:] or lat
    latency_ms = sorted(lat)[len(lat) // 2] * 1e3
    if dist:
        import torch

        lt = torch.tensor([latency_ms], dtype=torch.float64)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        latency_ms = float(lt.item())
    total_rays = rays
    if dist:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.float64)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        total_rays = int(r.item())

    roof = None
    if not args.no_roofline:
        # live per-kernel timing: HIP events on libpgrt's own stream around every closest-hit
        # launch (profile=1), and the instrumented traversal counts (profile=2, separate frame)
        # (1 GPU: the timed configuration, F frames per launch sequence)
        def prof_call(p):
            return ctx.render_frames_device(p, F, fb) if world == 1 else frame(p)

        frames_per_prof = F if world == 1 else 1
        p1 = abi.RenderParams.from_buffer_copy(params)
        p1.profile = 1
        reps = 5
        ms_trace = 0.0
        launches = 0
        for _ in range(reps):
            s1 = prof_call(p1)
            ms_trace += s1.ms_trace
            launches += s1.trace_launches
        p1.profile = 2
        s2 = prof_call(p1)
        frame_rays = s2.rays()
        alg_bytes = (RAY_BYTES * frame_rays + NODE_BYTES * s2.node_visits + WIDE_NODE_BYTES * s2.wide_node_visits
                     + TRI_BYTES * s2.tri_tests)
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
            "kernel": "closest hit: k_trace_pkt (wave packets, levels 0-2; level 0 generates its rays) + k_trace "
                      "(one lane per ray, levels 3-5 and the shadow queue)",
            "avg_launch_ms": round(avg_launch_ms, 4),
            "frames_per_launch": frames_per_prof,
            "launches_per_call": launches // reps,
            "trace_ms_per_frame": round(ms_trace / reps / frames_per_prof, 4),
            "node_visits_per_ray": round(s2.node_visits / max(1, frame_rays), 2),
            "wide_node_visits_per_ray": round(s2.wide_node_visits / max(1, frame_rays), 2),
            "tri_tests_per_ray": round(s2.tri_tests / max(1, frame_rays), 2),
            "bytes_per_ray": round(alg_bytes / max(1, frame_rays), 1),
        }
        tf = os.path.join(ROOT, "profiles", "traffic_c2.json")
        if args.config == "C2" and os.path.exists(tf):
            try:
                roof["traffic"] = json.load(open(tf)).get("bytes_per_launch")
            except Exception:  # noqa: BLE001
                pass

    if args.roofline_only:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "config": args.config, "roofline": roof}), flush=True)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    host_fb = None
    if world == 1 and not args.no_roofline:
        # PCIe-inclusive rate: the same frame through pgrt_render into a host
        # framebuffer (device -> host copy of W*H*16 B per frame); never the headline value
        for _ in range(2):
            ctx.render(params)
        t1 = time.perf_counter()
        nh = max(3, args.steps // 2)
        for _ in range(nh):
            ctx.render(params)
        host_fb = round((time.perf_counter() - t1) / nh * 1e3, 4)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.scene == "avenger":
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle  # cpu_baseline leg only: the CPU restatement timed on the host cores

        osc = pyoracle.OracleScene(scene)
        threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))

        def timed(nthreads, budget_s):  # whole C2 frames, repeated until the budget is spent
            frames = rays_c = 0
            t1 = time.perf_counter()
            while True:
                _, sc = osc.render(cam, params, row_step=1, threads=nthreads)
                rays_c += sc.rays()
                frames += 1
                dt_c = time.perf_counter() - t1
                if dt_c >= budget_s:
                    return rays_c / dt_c / 1e6, frames, rays_c, dt_c

        v_mt, f_mt, r_mt, t_mt = timed(threads, args.cpu_seconds)
        v_st, f_st, r_st, t_st = timed(1, args.cpu_seconds / 2)
        cpu = {"value": round(v_mt, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
               "sample": f"{f_mt} whole C2 frames ({r_mt} rays, {t_mt:.1f} s) on {threads} host threads "
                         f"(OpenMP over rows); oracle/ CPU restatement with its own SAH BVH",
               "single_thread_value": round(v_st, 3),
               "single_thread_sample": f"{f_st} frames ({r_st} rays, {t_st:.1f} s), 1 thread (the reference's "
                                       f"single Producer thread)"}

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(total_rays / elapsed / 1e6, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "frames_in_flight": in_flight,
            "frames_per_call": F,
            "frame_latency_ms": round(latency_ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic: avenger-proxy OBJ (reference OBJ absent) + spherical_map_windows.jpg"
                     if args.scene == "avenger" else "synthetic: 10^6 random triangles (seed 42) + env map"),
            "config": {
                "workload": f"{args.config} {'avenger-proxy' if args.scene == 'avenger' else '1M random triangles'} "
                            f"{args.width}x{args.height} Whitted d={args.max_level} + env map, "
                            f"{args.spp_side ** 2} spp {'DoF' if args.dof else 'pinhole'}",
                "triangles": bvh.num_triangles,
                "rays_per_frame": int(total_rays / args.steps),
                "parallelism": f"image tiles 64x64 over {world} GPU(s), ncclGather to rank 0" if world > 1
                else "1 GPU",
            },
            "roofline": roof,
            "host_framebuffer_ms_per_step": host_fb,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
