"""Every rank of a world-N distributed frame, rendered on ONE GPU (emulated; verdict r5 #7).

For a config (C2: 1920x1080 d=5 1 spp; C4: 3840x2160 d=5 thin lens 64 spp) and N in 2, 4, 8, a
child process per rank r renders rank r's tile deal of the N-GPU frame with calls in flight
through the distributed frame path with PGRT_EMULATE_RANK=r/N: the same tiles bench.py's rank r
renders (64x64 tiles, interleaved deal, rank 0's default share), the RCCL gather replaced by a
device copy of the rank's tiles into a full-size gather buffer; rank 0 also runs the unpack of
the whole frame.  Reported per (config, N): every rank's ms per frame, max / mean (the deal's
imbalance), rank 0's unpack per frame, and the projected N-GPU time = the slowest rank, against
the one-GPU time (world 1).  NOT included: the xGMI transfer into rank 0 (DESIGN.md §6 computes
it) and RCCL itself -- RCCL at world > 1 is unmeasured on hardware (this pool has one GPU per box).

Driver-shaped runs (--frames 20 --warmup 5 --repeat 5, optionally --fpc F): every rank times the same
short job bench.py's N-GPU line times (20 frames after 5 warm-up frames, calls of F frames, the median
of --repeat runs) -- the strong-scaling case, where one call's latency chain is a large part of the job.

usage: python tools/emulate_ranks.py [--configs C2,C4] [--worlds 2,4,8] [--frames N --warmup W --repeat R]
                                     [--fpc F] [--out file.jsonl]
"""
import argparse
import json
import os
import subprocess
import sys
import time
from collections import deque

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = {
    # frames per call: bench.py's 8 x world for C2 (a rank's launches as large as one GPU's), 1 for C4
    "C2": dict(W=1920, H=1080, spp=1, dof=0, in_flight=8, frames=lambda n: 40 * 8 * n, fpc=lambda n: 8 * n),
    "C4": dict(W=3840, H=2160, spp=8, dof=1, in_flight=6, frames=lambda n: 4 + 2 * n, fpc=lambda n: 1),
}


def child(config, world):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
    import scenes  # noqa: E402
    from pgi_raytracing_amd import abi  # noqa: E402
    from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

    c = dict(CFG[config])
    if os.environ.get("EMU_FRAMES"):  # driver-shaped: a short job, warm-up frames, repeats
        nfr, warm, rep = (int(x) for x in os.environ["EMU_FRAMES"].split(":"))
        c["frames"] = lambda n: nfr
    else:
        nfr, warm, rep = None, None, 1
    if os.environ.get("EMU_FPC"):
        c["fpc"] = lambda n: int(os.environ["EMU_FPC"])
    sc = load_obj(scenes.AVENGER_OBJ)
    sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    for kv in filter(None, os.environ.get("EMU_CFG", "").split(",")):  # pgrt_config overrides (--cfg)
        k, v = kv.split("=", 1)
        ctx.configure(**{k: int(v)})
    ctx.set_scene(sc)
    ctx.set_camera(abi.default_camera(c["W"], c["H"]))
    F = c["fpc"](world)
    frames = c["frames"](world)
    p = abi.make_params(spp_side=c["spp"], max_level=5, dof=c["dof"], jitter=abi.PGRT_JITTER_HASH)
    fb = ctx.alloc(F * c["W"] * c["H"] * 16)
    ctx.set_frames_in_flight(c["in_flight"])
    unpack = []

    def run(n, record=False):
        pend, rays = deque(), 0
        for k in range(0, n, F):
            pc = abi.RenderParams.from_buffer_copy(p)
            pc.frame = k
            nf = min(F, n - k)  # a short last call, as bench.py's (8 + 8 + 4 for 20 frames)
            pend.append(ctx.render_frames_distributed_device_async(pc, nf, fb) if world > 1
                        else ctx.render_frames_device_async(pc, nf, fb))
            if len(pend) >= c["in_flight"]:
                st = ctx.render_wait(pend.popleft())
                rays += st.rays()
                if record and world > 1:
                    unpack.append(st.ms_resolve / F)  # (approximate for a short last call)
        while pend:
            st = ctx.render_wait(pend.popleft())
            rays += st.rays()
            if record and world > 1:
                unpack.append(st.ms_resolve / F)
        return rays

    run(c["in_flight"] * F)  # every frame set allocated before the timed region
    ctx.synchronize()
    times = []
    for _ in range(rep):
        if warm:
            run(warm)
            ctx.synchronize()
        t = time.perf_counter()
        rays = run(frames, record=True)
        ctx.synchronize()
        times.append(time.perf_counter() - t)
    dt = sorted(times)[len(times) // 2]
    print(json.dumps({"ms_per_frame": dt / frames * 1e3, "rays_per_frame": rays / frames, "frames": frames,
                      "frames_per_call": F, "repeats": rep,
                      "unpack_ms_per_frame": (sum(unpack) / len(unpack)) if unpack else None}))


def run_child(config, world, rank, args):
    env = dict(os.environ, EMU_CHILD=f"{config}:{world}", GPU_MAX_HW_QUEUES="16")
    if args.frames:
        env["EMU_FRAMES"] = f"{args.frames}:{args.warmup}:{args.repeat}"
    if args.fpc:
        env["EMU_FPC"] = str(args.fpc)
    if args.cfg:
        env["EMU_CFG"] = ",".join(args.cfg)
    if world > 1:
        env["PGRT_EMULATE_RANK"] = f"{rank}/{world}"
    else:
        env.pop("PGRT_EMULATE_RANK", None)
    out = subprocess.run([sys.executable, __file__], env=env, check=True, capture_output=True, text=True,
                         timeout=300).stdout
    return json.loads(out.strip().splitlines()[-1])


def main():
    if os.environ.get("EMU_CHILD"):
        config, world = os.environ["EMU_CHILD"].split(":")
        child(config, int(world))
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C2,C4")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--out", default=None)
    ap.add_argument("--frames", type=int, default=None, help="timed frames per run (driver-shaped: 20)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--fpc", type=int, default=None, help="frames per call (default: CFG's rule)")
    ap.add_argument("--cfg", action="append", default=[], help="pgrt_config override key=int (repeatable)")
    args = ap.parse_args()
    lines = []
    for config in args.configs.split(","):
        one = run_child(config, 1, 0, args)
        shape = {"frames": args.frames, "warmup": args.warmup, "repeat": args.repeat} if args.frames else "steady"
        if args.cfg or args.fpc:
            shape = {"shape": shape, "cfg": args.cfg, "fpc": args.fpc}
        rec = {"config": config, "world": 1, "ms_per_frame": round(one["ms_per_frame"], 4), "job": shape,
               "rays_per_frame": one["rays_per_frame"], "frames_per_call": one["frames_per_call"]}
        print(json.dumps(rec), flush=True)
        lines.append(rec)
        for n in [int(x) for x in args.worlds.split(",")]:
            ranks = []
            for r in range(n):  # one line per rank child (a long silent run looks hung to the box's guard)
                ranks.append(run_child(config, n, r, args))
                print(f"# {config} world {n} rank {r}: {ranks[-1]['ms_per_frame']:.4f} ms/frame", flush=True)
            ms = [r["ms_per_frame"] for r in ranks]
            slow = max(ms)
            rec = {"config": config, "world": n, "emulated": True, "job": shape,
                   "rank_ms_per_frame": [round(x, 4) for x in ms],
                   "rank_rays_per_frame": [int(r["rays_per_frame"]) for r in ranks],
                   "max_over_mean": round(slow / (sum(ms) / n), 3),
                   "slowest_rank": ms.index(slow),
                   "rank0_unpack_ms_per_frame": round(ranks[0]["unpack_ms_per_frame"] or 0.0, 4),
                   "projected_ms_per_frame_without_xgmi": round(slow, 4),
                   "projected_speedup_without_xgmi": round(one["ms_per_frame"] / slow, 3),
                   "frames_per_call": ranks[0]["frames_per_call"],
                   "note": "one GPU renders each rank's tiles in turn (PGRT_EMULATE_RANK); no RCCL, no xGMI transfer"}
            print(json.dumps(rec), flush=True)
            lines.append(rec)
    if args.out:
        with open(args.out, "w") as f:
            for rec in lines:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
