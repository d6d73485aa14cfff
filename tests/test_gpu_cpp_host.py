"""The C++ host facade (include/pgrt_raytracer.hpp, examples/pg1_pgrt.cpp) on the GPU: the
reference's own entry points re-run through libpgrt and checked like the reference checks
them (printed tutorial_1 output) and against the oracle (raytrace_loop frame)."""
import os
import subprocess

import numpy as np
import pytest

import pyoracle
from conftest import ENV_MAP, ROOT, assert_frames_match
from pgi_raytracing_amd import abi

pytestmark = pytest.mark.gpu
EXE = os.path.join(ROOT, "build", "pg1_pgrt")


def test_tutorial_1_prints_reference_output():
    out = subprocess.run([EXE, "tutorial_1"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "normal = (0.000, 0.000, 1.000)" in out.stdout
    assert "tex_coord = (0.050, 0.933)" in out.stdout


def test_raytrace_loop_frame_matches_oracle(tmp_path, avenger_obj, avenger_scene):
    """raytrace_loop through the C++ facade alone: LoadOBJ in libpgrt, every texture decoded from
    the reference's own .jpg files by libpgrt_image (Texture::Texture, texture.cpp:5-54) -- no
    Python-written texture files anywhere -- and the frame equals the oracle's bit for bit."""
    import glob

    assert not glob.glob(os.path.join(ROOT, "assets", "**", "*.pgrttex"), recursive=True)
    raw = tmp_path / "frame.raw"
    W, H, S, d, dof = 160, 120, 2, 5, 1
    out = subprocess.run([EXE, "render", avenger_obj, ENV_MAP, str(raw), str(W), str(H), str(S), str(d), str(dof)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "Surfaces = 94" in out.stdout and "Materials = 5" in out.stdout
    img = np.fromfile(raw, np.float32).reshape(H, W, 4)
    cam = abi.default_camera(W, H)
    p = abi.make_params(spp_side=S, max_level=d, dof=dof, jitter=abi.PGRT_JITTER_HASH, seed=1234)
    ref, _ = pyoracle.OracleScene(avenger_scene).render(cam, p)
    _, exact = assert_frames_match(img, ref)
    assert exact == 1.0
    assert os.path.getsize(str(raw) + ".pfm") > W * H * 12


def test_raytrace_loop_single_process_multi_device(tmp_path, avenger_obj, avenger_scene):
    """The same C++ raytrace_loop with the facade's multi-device constructor (pgrt_create_devices,
    ranks 0,0,0 -- three ranks on this box's one GPU, gathered by device copies): the frame is
    the oracle's bit for bit."""
    raw = tmp_path / "frame_md.raw"
    W, H, S, d, dof = 200, 130, 2, 5, 1
    out = subprocess.run([EXE, "render", avenger_obj, ENV_MAP, str(raw), str(W), str(H), str(S), str(d), str(dof),
                          "0,0,0"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    img = np.fromfile(raw, np.float32).reshape(H, W, 4)
    cam = abi.default_camera(W, H)
    p = abi.make_params(spp_side=S, max_level=d, dof=dof, jitter=abi.PGRT_JITTER_HASH, seed=1234)
    ref, _ = pyoracle.OracleScene(avenger_scene).render(cam, p)
    _, exact = assert_frames_match(img, ref)
    assert exact == 1.0
