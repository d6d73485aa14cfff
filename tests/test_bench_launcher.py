"""bench.py --gpus N starts its own rank processes (no torch.distributed.run needed): CPU checks
of the launcher -- a clear error when fewer GPUs are visible, and N ranks with the launcher
environment (here they stop at pgrt_create: no GPU in this container, the failure propagates)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(env_extra, *args):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=120)


def test_too_few_gpus_is_an_error():
    r = _run({"HIP_VISIBLE_DEVICES": "0"}, "--gpus", "2")
    assert r.returncode == 2
    assert "needs 2 GPUs, 1 visible" in r.stderr


def test_ranks_are_started_with_the_launcher_environment():
    import pytest

    from pgi_raytracing_amd.raytracer import device_count

    if device_count() > 0:
        pytest.skip("GPU present: the ranks would run the bench")
    r = _run({"HIP_VISIBLE_DEVICES": "0,1"}, "--gpus", "2", "--steps", "2")
    assert r.returncode != 0
    # both ranks got their own process and device index (rank 1 -> LOCAL_RANK 1)
    assert "pgrt_create(device=1)" in r.stderr or "pgrt_create(device=0)" in r.stderr
    assert "WORLD_SIZE" not in r.stdout


def test_world_size_must_match_gpus():
    r = _run({"WORLD_SIZE": "1", "RANK": "0"}, "--gpus", "2")
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
