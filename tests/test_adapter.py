"""The pbrt-facing C++ host layer (cuda-raytrace_amd/adapter, mirroring
cudaapi.h:8-19 / cudarender.h:14-91) driven by its CLI.

CPU: host-side transform math self-test; a clean error (not a crash) when no
device is present. GPU: the C++ path (CudaRenderInit -> CreateCudaShape ->
CreateCudaRenderer -> Render -> Film::AddSample) renders the same image, bit
for bit, as the Python stage driver over the same C-ABI; an identity object
instance (ObjectBegin/ObjectInstance flattening) changes nothing."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "cuda-raytrace_amd", "lib", "pm_render_cli")

needs_cli = pytest.mark.skipif(not os.path.exists(CLI), reason="adapter CLI not built (make -C cuda-raytrace_amd)")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3)[::-1]


def camera_args(sc):
    _, eye, fwd, right, up, _, _ = sc.camera
    return [repr(float(v)) for vec in (eye, fwd, right, up) for v in vec]


@needs_cli
def test_adapter_selftest():
    r = subprocess.run([CLI, "--selftest"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "selftest: ok" in r.stdout


@needs_cli
@pytest.mark.skipif(_has_gpu(), reason="checks the no-device error path")
def test_adapter_reports_missing_device(tmp_path):
    from pmrender import scenes
    sc = scenes.cornell_box(16, 16)
    r = subprocess.run([CLI, "--scene", "cornell", "--camera", *camera_args(sc), "--out", str(tmp_path / "x.pfm")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert "no HIP device" in r.stderr


@needs_cli
@pytest.mark.gpu
@pytest.mark.parametrize("structure", ["grid", "kd"])
def test_adapter_matches_stage_driver(structure, tmp_path, hip_mod):
    from pmrender import scenes
    from pmrender.abi import PM_GATHER_GRID, PM_GATHER_KDTREE, RenderParams
    W, H, paths = 64, 48, 16384
    sc = scenes.cornell_box(W, H)
    out = tmp_path / "img.pfm"
    args = [CLI, "--scene", "cornell", "--width", str(W), "--height", str(H), "--paths", str(paths),
            "--structure", structure, "--camera", *camera_args(sc), "--out", str(out)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    img = read_pfm(out)

    ctx = sc.load_into(hip_mod.Context(0))
    p = RenderParams.defaults(paths_per_pass=paths,
                              gather_structure=PM_GATHER_KDTREE if structure == "kd" else PM_GATHER_GRID)
    ref, _ = ctx.render(p)
    ctx.close()
    assert img.shape == ref.shape
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), "adapter image differs from stage driver"

    r2 = subprocess.run(args[:-2] + ["--instanced", "--out", str(tmp_path / "inst.pfm")], capture_output=True,
                        text=True, timeout=300)
    assert r2.returncode == 0, r2.stderr
    assert np.array_equal(read_pfm(tmp_path / "inst.pfm").view(np.uint32), img.view(np.uint32))
