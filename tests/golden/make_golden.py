"""Write the golden fixtures under tests/golden/ (run from the repo root; no GPU):

  reference_kats.json  -- the reference's own known-answer demos as data: inputs and the text the
                          reference prints (tutorial_1, tutorials.cpp:29-139; tutorial_2,
                          tutorials.cpp:170-178 on data/test4.png), and the PinHoleCamera basis of
                          raytrace_loop's pose (PinHoleCamera.cpp:5-29, tutorials.cpp:186-191) as
                          SURVEY.md §8 A3 lists it.  Hand-derived from the reference source; the
                          reference cannot run here.
  oracle_vectors.npz   -- regression vectors of the CPU restatement (oracle/, pinned by the KATs
                          above): texel lookups over test3.png / test4.png including the edge
                          bands, environment lookups on 4096 seeded directions, primary rays of
                          the default camera, mix_srgb / gamma on edge and random inputs, and two
                          48x36 avenger-proxy frames (Whitted d=5, path tracing d=5 S=2).  They
                          freeze the restatement: tests/test_golden.py checks the oracle and the
                          GPU against them.

usage: python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")):
    sys.path.insert(0, p)

import pyoracle  # noqa: E402
import scenes  # noqa: E402
from pgi_raytracing_amd import abi  # noqa: E402
from pgi_raytracing_amd.raytracer import load_obj  # noqa: E402
from pgi_raytracing_amd.scene import TextureData  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
ASSETS = os.path.join(ROOT, "assets")

KATS = {
    "tutorial_1": {
        "source": "APP/tutorials.cpp:29-139 (add_triangle :29-80, generate_and_trace_ray :83-139)",
        "triangle": [[0.0, 0.0, 0.0], [2.0, 0.0, 0.0], [0.0, 3.0, 0.0]],
        "normals": [[0.0, 0.0, 1.0]] * 3,
        "uvs": [[0.0, 1.0], [1.0, 1.0], [0.0, 0.0]],
        "ray": {"org": [0.1, 0.2, 2.0], "dir": [0.0, 0.0, -1.0], "tnear": "FLT_MIN", "tfar": "FLT_MAX"},
        "expect": {"t": 2.0, "u_print": "0.050", "v": 1.0 / 15.0, "geomID": 0, "primID": 0,
                   "printed": ["normal = (0.000, 0.000, 1.000)", "tex_coord = (0.050, 0.933)"]},
    },
    "tutorial_2": {
        "source": "APP/tutorials.cpp:170-178, APP/texture.cpp:56-130, data/test4.png (64x32 RGBA)",
        "texture": "test4.png",
        "uv": ["2.5/64 (float)", 0.0],
        "expect": {"printed": "(r = 1.000, g = 0.000, b = 0.500)"},
    },
    "camera_basis": {
        "source": "APP/PinHoleCamera.cpp:5-29 with raytrace_loop's pose (tutorials.cpp:186-191): "
                  "fov_y deg2rad(42.185), from (-140,-175,80), at (0,0,40), up (0,0,1); SURVEY.md §8 A3",
        "f_y": {"480": 622.217, "1080": 1399.988, "2160": 2799.977},
        "x_c": [0.78087, -0.62470, 0.0], "y_c": [0.10976, 0.13720, 0.98444], "z_c": [-0.61498, -0.76872, 0.17571],
        "atol": 1e-4,
    },
}


def texel_vectors(tex):
    w, h = tex.width, tex.height
    us = np.concatenate([np.arange(0, w + 1, 0.25) / w, np.array([-0.01, 1.0, 1.01, 0.5 / w, (w - 0.5) / w])])
    vs = np.concatenate([np.arange(0, h + 1, 0.25) / h, np.array([-0.01, 1.0, (h - 0.5) / h])])
    uv = np.array([(u, v) for u in us[::3] for v in vs[::2]], np.float32)
    out = np.array([pyoracle.get_texel(tex, float(u), float(v)) for u, v in uv], np.float32)
    return uv, out


def main():
    with open(os.path.join(OUT, "reference_kats.json"), "w") as fh:
        json.dump(KATS, fh, indent=1)
    vec = {}
    for name in ("test3.png", "test4.png"):
        uv, out = texel_vectors(TextureData.from_file(os.path.join(ASSETS, name)))
        vec[f"texel_{name[:-4]}_uv"], vec[f"texel_{name[:-4]}_out"] = uv, out
    env = TextureData.from_file(os.path.join(ASSETS, "spherical_map_windows.jpg"))
    rng = np.random.default_rng(2024)
    d = rng.normal(size=(4096, 3)).astype(np.float32)
    d[:8] = [[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1], [1, 1, 0], [0, -1, 1]]
    vec["env_dir"] = d
    vec["env_out"] = np.array([pyoracle.env_texel(env, *map(float, x)) for x in d], np.float32)
    cam = abi.default_camera(1920, 1080)
    xy = np.array([(x, y) for x in (0.0, 0.5, 959.25, 960.0, 1919.75) for y in (0.0, 539.5, 540.0, 1079.75)],
                  np.float32)
    vec["ray_xy"] = xy
    vec["ray_pinhole"] = np.array([pyoracle.generate_ray(cam, float(x), float(y)) for x, y in xy], np.float32)
    vec["ray_dof"] = np.array([pyoracle.generate_ray(cam, float(x), float(y), 1, 200.0, 5.0, 1.25, -2.0)
                               for x, y in xy], np.float32)
    c = rng.uniform(-0.2, 1.3, size=(256, 9)).astype(np.float32)
    c[:4, :8] = [[0, 0, 0, 1, 1, 1, 1, 1], [1, 0, 0.5, 1, 0, 1, 0.5, 1], [-1, 2, 0, 1, 0.3, 0.3, 0.3, 1],
                 [np.nan, 0, 0, 1, 0, 0, 0, 1]]
    vec["mix_in"] = c
    vec["mix_out"] = np.array([pyoracle.mix_srgb(x[0:4], x[4:8], float(x[8])) for x in c], np.float32)
    vec["gamma_out"] = np.array([pyoracle.gamma(x[0:4], 0.5) for x in c], np.float32)
    if not os.path.exists(scenes.AVENGER_OBJ):
        scenes.write_avenger_proxy()
    sc = load_obj(scenes.AVENGER_OBJ)
    sc.set_environment(os.path.join(ASSETS, "spherical_map_windows.jpg"))
    osc = pyoracle.OracleScene(sc)
    fcam = abi.default_camera(48, 36)
    vec["frame_whitted_d5"], _ = osc.render(fcam, abi.make_params(max_level=5))
    vec["frame_path_d5_s2"], _ = osc.render(fcam, abi.make_params(max_level=5, spp_side=2, mode=abi.PGRT_MODE_PATH,
                                                                  jitter=abi.PGRT_JITTER_HASH, seed=7))
    np.savez_compressed(os.path.join(OUT, "oracle_vectors.npz"), **vec)
    print("wrote", sorted(vec))


if __name__ == "__main__":
    main()
