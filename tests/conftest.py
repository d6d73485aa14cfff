import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

ASSETS = os.path.join(ROOT, "assets")
ENV_MAP = os.path.join(ASSETS, "spherical_map_windows.jpg")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpgrt's HIP kernels)")


@pytest.fixture(scope="session")
def avenger_obj():
    import scenes

    if not os.path.exists(scenes.AVENGER_OBJ):
        scenes.write_avenger_proxy()
    return scenes.AVENGER_OBJ


@pytest.fixture(scope="session")
def geosphere_obj():
    import scenes

    if not os.path.exists(scenes.SPHERE_OBJ):
        scenes.write_geosphere()
    return scenes.SPHERE_OBJ


@pytest.fixture(scope="session")
def avenger_scene(avenger_obj):
    """Product-path scene: the C++ loader in libpgrt (no GPU needed) + PIL texture decode."""
    from pgi_raytracing_amd.raytracer import load_obj

    sc = load_obj(avenger_obj)
    sc.set_environment(ENV_MAP)
    return sc


@pytest.fixture(scope="session")
def geosphere_scene(geosphere_obj):
    from pgi_raytracing_amd.raytracer import load_obj

    sc = load_obj(geosphere_obj)
    sc.set_environment(ENV_MAP)
    return sc


@pytest.fixture(scope="session")
def gpu_ctx():
    from pgi_raytracing_amd.raytracer import Context, device_count

    if device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on an MI355X")
    return Context(0)


def assert_frames_match(gpu, ref, tol=1e-4):
    """Parity bar: |gpu - ref| <= tol after gamma, NaN at the same pixels/channels."""
    assert gpu.shape == ref.shape
    ng, nr = np.isnan(gpu), np.isnan(ref)
    assert (ng == nr).all(), f"NaN mismatch at {np.argwhere(ng != nr)[:5]}"
    d = np.abs(np.where(ng, 0, gpu) - np.where(nr, 0, ref))
    assert d.max() <= tol, f"max diff {d.max()} at {np.unravel_index(d.argmax(), d.shape)}"
    return float(d.max()), float((d == 0).mean())
