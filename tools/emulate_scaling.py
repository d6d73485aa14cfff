"""Strong-scaling estimate on ONE GPU for bench.py's multi-GPU C2 run.

For N in 1, 2, 4, 8 and a rank r, a child process renders rank r's share of an N-GPU frame
(64x64 tiles dealt round-robin, the same tiles bench.py gives that rank) with frames in flight,
through the distributed frame path with PGRT_EMULATE_RANK=r/N: the RCCL gather is replaced by a
device copy of the rank's tiles into a full-size gather buffer, and rank 0 also runs the unpack.
Prints one JSON line per (N, rank): ms per frame and the speedup T1 / TN of that rank.  The xGMI
transfer (25 MB of RGB per C2 frame into rank 0 at N = 8) is NOT included.

usage: python tools/emulate_scaling.py [frames] [in_flight] [worlds, default 1,2,4,8]
       EMU_FRAMES_PER_CALL=F: F frames per call (pgrt_render_frames_distributed_device_async)
"""
import json
import os
import subprocess
import sys
import time
from collections import deque

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(frames, in_flight):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tools")]
    import scenes  # noqa: E402
    from pgi_raytracing_amd import abi  # noqa: E402
    from pgi_raytracing_amd.raytracer import Context, load_obj  # noqa: E402

    sc = load_obj(scenes.AVENGER_OBJ)
    sc.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    ctx.set_scene(sc)
    W, H = 1920, 1080
    ctx.set_camera(abi.default_camera(W, H))
    F = int(os.environ.get("EMU_FRAMES_PER_CALL", "1"))  # frames per call (batched frames)
    fb = ctx.alloc(F * W * H * 16)
    p = abi.make_params(max_level=5)
    ctx.set_frames_in_flight(in_flight)

    host = [0.0, 0.0]  # seconds inside submit / wait calls

    def run(n):
        pend, rays = deque(), 0
        for _ in range(0, n, F):
            t0 = time.perf_counter()
            pend.append(ctx.render_frames_distributed_device_async(p, F, fb) if F > 1
                        else ctx.render_distributed_device_async(p, fb))
            t1 = time.perf_counter()
            host[0] += t1 - t0
            if len(pend) >= in_flight:
                rays += ctx.render_wait(pend.popleft()).rays()
                host[1] += time.perf_counter() - t1
        while pend:
            rays += ctx.render_wait(pend.popleft()).rays()
        return rays

    run(max(20, 2 * in_flight * F))  # every frame set allocated before the timed region
    ctx.synchronize()
    host[0] = host[1] = 0.0
    t = time.perf_counter()
    rays = run(frames)
    ctx.synchronize()
    dt = time.perf_counter() - t
    print(json.dumps({"ms_per_frame": dt / frames * 1e3, "rays_per_frame": rays / frames,
                      "host_submit_ms": host[0] / frames * 1e3, "host_wait_ms": host[1] / frames * 1e3}))


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    in_flight = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    if os.environ.get("EMU_CHILD"):
        child(frames, in_flight)
        return
    worlds = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,8").split(",")]
    t1 = None
    for n in worlds:
        for r in sorted({0, n - 1}):
            env = dict(os.environ, EMU_CHILD="1", PGRT_EMULATE_RANK=f"{r}/{n}", GPU_MAX_HW_QUEUES="16")
            out = subprocess.run([sys.executable, __file__, str(frames), str(in_flight)], env=env, check=True,
                                 capture_output=True, text=True, timeout=300).stdout
            d = json.loads(out.strip().splitlines()[-1])
            if t1 is None:
                t1 = d["ms_per_frame"] * n  # speedups relative to the first world (x its size)
            d.update(world=n, rank=r, in_flight=in_flight, frames_per_call=os.environ.get("EMU_FRAMES_PER_CALL", "1"), speedup=round(t1 / d["ms_per_frame"], 3),
                     efficiency=round(t1 / d["ms_per_frame"] / n, 3))
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
