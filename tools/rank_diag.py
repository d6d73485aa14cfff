import os, sys
ROOT="/root/repo"; sys.path[:0]=[ROOT, ROOT+"/tools"]
import scenes
from pgi_raytracing_amd import abi
from pgi_raytracing_amd.raytracer import Context, load_obj
sc = load_obj(scenes.AVENGER_OBJ); sc.set_environment(os.path.join(ROOT,"assets","spherical_map_windows.jpg"))
ctx = Context(0); ctx.set_scene(sc); ctx.set_camera(abi.default_camera(1920,1080))
fb = ctx.alloc(1920*1080*16+(1<<24))
for world in (1, 8):
    p = abi.make_params(max_level=5, profile=1)
    for _ in range(5): st = ctx.render_tiles_device(p, 0, world, fb)
    acc = {}
    R=9
    import statistics
    rows=[]
    for _ in range(R):
        st = ctx.render_tiles_device(p, 0, world, fb)
        d = ctx.frame_diag()[:6]
        rows.append((st.ms_total, st.ms_raygen, st.ms_trace, st.ms_shade, st.ms_shadow, st.ms_combine, [(x["ms_trace"], x["ms_shade"], x["rays"]) for x in d] if isinstance(d[0], dict) else [(x.ms_trace,x.ms_shade,x.rays) for x in d]))
    rows.sort(key=lambda r:r[0]); r=rows[R//2]
    print(f"world={world} total {r[0]:.3f} raygen {r[1]:.3f} trace {r[2]:.3f} shade {r[3]:.3f} shadow {r[4]:.3f} combine+finish {r[5]:.3f}")
    for L,(a,b,n) in enumerate(r[6]): print(f"  L{L} rays {n} trace {a:.3f} shade {b:.3f}")
