"""Per-step latency record of the ray-tree launch (k_subtree) of a synchronous C2 frame.

Needs the diagnostics build (PGRT_STEP_PROFILE=1: `EXTRA_FLAGS=-DPGRT_STEP_PROFILE=1
tools/build_variant.sh stepprof`, run with PGRT_LIB=ablib/stepprof/libpgrt.so): every ray tree the
launch evaluates writes one record -- wall-clock start / end (100 MHz), shader-clock cycles in
all, in 8-wide node steps and in triangle rounds, the part of each spent waiting for the step's
loads (issue -> first use), cycles in the shading between traces, the step / trace counts, and its
wave.  Prints, per launch: the tree-time distribution, the slowest tree's breakdown and the other
groups of its wave, and the per-step cost distribution over all trees.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=3, help="synchronous frames (the last one is recorded)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--cfg", action="append", default=[])
    ap.add_argument("--shade", action="store_true",
                    help="instead: per-wave phase cycles of k_shade over the driver's 20 frames (calls of 8 in flight)")
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
    import scenes
    from pgi_raytracing_amd import abi
    from pgi_raytracing_amd.raytracer import Context, load_obj

    if not os.path.exists(scenes.AVENGER_OBJ):
        scenes.write_avenger_proxy()
    scene = load_obj(scenes.AVENGER_OBJ)
    scene.set_environment(os.path.join(ROOT, "assets", "spherical_map_windows.jpg"))
    ctx = Context(0)
    for kv in args.cfg:
        k, v = kv.split("=", 1)
        ctx.configure(**{k: int(v)})
    ctx.set_scene(scene)
    ctx.set_camera(abi.default_camera(1920, 1080))
    L = ctx.L
    if not hasattr(L, "pgrt_diag_step_profile"):
        sys.exit("this libpgrt.so is not the PGRT_STEP_PROFILE build (set PGRT_LIB=ablib/stepprof/libpgrt.so)")
    L.pgrt_diag_step_profile.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int]
    p = abi.make_params(spp_side=1, max_level=5)
    if args.shade:
        return shade_report(ctx, abi, p, args.out)
    fb = ctx.alloc(1920 * 1080 * 16)
    ctx.set_frames_in_flight(1)
    n = C.c_int(0)
    for f in range(args.frames):
        if f == args.frames - 1:
            L.pgrt_diag_step_profile(None, 0, C.byref(n), 1)  # reset before the recorded frame
        ctx.render_device(p, fb)
    ctx.synchronize()
    L.pgrt_diag_step_profile(None, 0, C.byref(n), 0)
    cnt = min(n.value, 1 << 18)
    rec = np.zeros((cnt, 12), np.uint64)
    L.pgrt_diag_step_profile(rec.ctypes.data, cnt, C.byref(n), 0)
    report = {"trees": int(cnt), "launches": []}
    tags = sorted(set(rec[:, 11].tolist()))
    for tag in tags:
        r = rec[rec[:, 11] == tag]
        w0, w1 = r[:, 0].astype(np.int64), r[:, 1].astype(np.int64)
        t0 = w0.min()
        wall_us = (w1 - w0) / 100.0  # 100 MHz
        cyc = r[:, 2].astype(np.float64)
        node_cyc, node_wait = r[:, 3].astype(np.float64), r[:, 4].astype(np.float64)
        tri_cyc, tri_wait = r[:, 5].astype(np.float64), r[:, 6].astype(np.float64)
        shade_cyc = r[:, 7].astype(np.float64)
        nodes = (r[:, 8] & 0xFFFFFFFF).astype(np.float64)
        tris = (r[:, 8] >> np.uint64(32)).astype(np.float64)
        ntrace = (r[:, 9] & 0xFFFF).astype(np.int64)
        maxsp = ((r[:, 9] >> np.uint64(16)) & 0xFF).astype(np.int64)
        level = int(((r[0, 9] >> np.uint64(24)) & 0xFF))
        G = int((r[0, 9] >> np.uint64(32)) & 0xFF)
        wave = (r[:, 10] & 0xFFFFFFFF).astype(np.int64)
        ghz = cyc.sum() / (wall_us.sum() * 1e3) if wall_us.sum() > 0 else 0.0
        k = int(np.argmax(wall_us))
        same = np.where(wave == wave[k])[0]

        def tree(j):
            return {"wall_us": round(float(wall_us[j]), 2), "start_us": round((w0[j] - t0) / 100.0, 2),
                    "cycles": int(cyc[j]), "traces": int(ntrace[j]), "max_stack": int(maxsp[j]),
                    "node_steps": int(nodes[j]), "tri_rounds": int(tris[j]),
                    "node_cyc_per_step": round(node_cyc[j] / max(1, nodes[j]), 1),
                    "node_wait_per_step": round(node_wait[j] / max(1, nodes[j]), 1),
                    "tri_cyc_per_round": round(tri_cyc[j] / max(1, tris[j]), 1),
                    "tri_wait_per_round": round(tri_wait[j] / max(1, tris[j]), 1),
                    "shade_cyc_per_trace": round(shade_cyc[j] / max(1, ntrace[j]), 1),
                    "other_cyc": int(cyc[j] - node_cyc[j] - tri_cyc[j] - shade_cyc[j])}

        steps = nodes + tris
        ok = steps > 0
        per_step = (node_cyc + tri_cyc)[ok] / steps[ok]
        wait_share = (node_wait + tri_wait)[ok] / np.maximum(1, (node_cyc + tri_cyc)[ok])
        big = wall_us >= np.percentile(wall_us, 99)
        L_ = {"level": level, "lanes_per_ray": G, "trees": int(len(r)),
              "span_us": round((w1.max() - t0) / 100.0, 1), "shader_clock_ghz": round(ghz, 3),
              "tree_wall_us_p50_p90_p99_max": [round(float(np.percentile(wall_us, q)), 1) for q in (50, 90, 99)] +
              [round(float(wall_us.max()), 1)],
              "cyc_per_step_p50_p90_max": [round(float(np.percentile(per_step, q)), 0) for q in (50, 90)] +
              [round(float(per_step.max()), 0)],
              "load_wait_share_p50_p90": [round(float(np.percentile(wait_share, q)), 3) for q in (50, 90)],
              "slowest_1pct_trees": {
                  "traces_mean": round(float(ntrace[big].mean()), 1),
                  "node_steps_mean": round(float(nodes[big].mean()), 1),
                  "tri_rounds_mean": round(float(tris[big].mean()), 1),
                  "node_cyc_per_step": round(float(node_cyc[big].sum() / max(1, nodes[big].sum())), 1),
                  "node_wait_per_step": round(float(node_wait[big].sum() / max(1, nodes[big].sum())), 1),
                  "tri_cyc_per_round": round(float(tri_cyc[big].sum() / max(1, tris[big].sum())), 1),
                  "tri_wait_per_round": round(float(tri_wait[big].sum() / max(1, tris[big].sum())), 1),
                  "shade_cyc_per_trace": round(float(shade_cyc[big].sum() / max(1, ntrace[big].sum())), 1),
                  "share_node_tri_shade_other": [round(float(x / cyc[big].sum()), 3) for x in (
                      node_cyc[big].sum(), tri_cyc[big].sum(), shade_cyc[big].sum(),
                      cyc[big].sum() - node_cyc[big].sum() - tri_cyc[big].sum() - shade_cyc[big].sum())]},
              "slowest_tree": tree(k),
              "slowest_wave_groups": sorted((tree(j) for j in same), key=lambda d: -d["wall_us"])}
        report["launches"].append(L_)
    txt = json.dumps(report, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n")


def shade_report(ctx, abi, p, out):
    """k_shade per wave and iteration: cycles of part A (hit, attributes, normal, material, child
    directions), the allocation's first barrier + atomic issue, part B (environment / texel fetch,
    attenuation, R), the allocation's second barrier, the emit -- by level and by the wave's mix of
    ray kinds (verdict r5 #3: why a bounce-level ray costs more than a level-0 ray)."""
    L = ctx.L
    if not hasattr(L, "pgrt_diag_shade_profile"):
        sys.exit("this libpgrt.so is not the PGRT_STEP_PROFILE build")
    L.pgrt_diag_shade_profile.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.c_int]
    W, H, F, inflight = 1920, 1080, 8, 8
    fb = ctx.alloc(inflight * F * W * H * 16)
    ctx.set_frames_in_flight(inflight)
    frame = [0]

    def run(nframes):
        pend = []
        k = 0
        while nframes > 0:
            nf = min(F, nframes)
            pc = abi.RenderParams.from_buffer_copy(p)
            pc.jitter = abi.PGRT_JITTER_HASH
            pc.frame = frame[0]
            frame[0] += nf
            pend.append(ctx.render_frames_device_async(pc, nf, fb + (k % inflight) * F * W * H * 16))
            k += 1
            nframes -= nf
            if len(pend) >= inflight:
                ctx.render_wait(pend.pop(0))
        for t in pend:
            ctx.render_wait(t)

    n = C.c_int(0)
    run(inflight * F)
    run(5)
    ctx.synchronize()
    L.pgrt_diag_shade_profile(None, 0, C.byref(n), 1)
    run(20)
    ctx.synchronize()
    L.pgrt_diag_shade_profile(None, 0, C.byref(n), 0)
    cnt = min(n.value, 1 << 20)
    rec = np.zeros((cnt, 4), np.uint64)
    L.pgrt_diag_shade_profile(rec.ctypes.data, cnt, C.byref(n), 0)
    lo = lambda x: (x & np.uint64(0xFFFFFFFF)).astype(np.float64)
    hi = lambda x: (x >> np.uint64(32)).astype(np.float64)
    level = (rec[:, 0] & np.uint64(0xFF)).astype(np.int64)
    act = ((rec[:, 0] >> np.uint64(8)) & np.uint64(0xFF)).astype(np.int64)
    miss = ((rec[:, 0] >> np.uint64(16)) & np.uint64(0xFF)).astype(np.int64)
    diel = ((rec[:, 0] >> np.uint64(24)) & np.uint64(0xFF)).astype(np.int64)
    opq = ((rec[:, 0] >> np.uint64(32)) & np.uint64(0xFF)).astype(np.int64)
    ph = np.stack([lo(rec[:, 1]), hi(rec[:, 1]), lo(rec[:, 2]), hi(rec[:, 2]), lo(rec[:, 3])], 1)
    tot = hi(rec[:, 3])
    names = ["part_a", "alloc_begin", "part_b", "alloc_end", "emit"]
    rep = {"wave_iterations": int(cnt), "note": "shader-clock cycles per wave and shading iteration (diagnostics build; "
           "s_memtime stamps add ~10%)", "levels": []}
    for lv in sorted(set(level.tolist())):
        m = (level == lv) & (act > 0)
        if not m.any():
            continue
        kinds = (miss[m] > 0).astype(int) + 2 * (diel[m] > 0).astype(int) + 4 * (opq[m] > 0).astype(int)
        mix = {}
        for code, name in ((1, "miss only"), (2, "dielectric only"), (4, "opaque only"), (3, "miss+dielectric"),
                           (5, "miss+opaque"), (6, "dielectric+opaque"), (7, "all three")):
            sel = kinds == code
            if sel.any():
                mix[name] = {"waves": int(sel.sum()), "cycles_mean": round(float(tot[m][sel].mean()), 0),
                             "phase_mean": {nm: round(float(ph[m][sel][:, j].mean()), 0) for j, nm in enumerate(names)}}
        rep["levels"].append({
            "level": int(lv), "wave_iterations": int(m.sum()), "rays": int(act[m].sum()),
            "rays_miss_dielectric_opaque": [int(miss[m].sum()), int(diel[m].sum()), int(opq[m].sum())],
            "cycles_per_wave_iteration": round(float(tot[m].mean()), 0),
            "cycles_per_ray": round(float(tot[m].sum() / act[m].sum()), 1),
            "phase_share": {nm: round(float(ph[m][:, j].sum() / tot[m].sum()), 3) for j, nm in enumerate(names)},
            "by_wave_mix": mix})
    txt = json.dumps(rep, indent=1)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
