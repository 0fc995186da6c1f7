"""Multi-device context behind the C-ABI (pm_config::n_devices; SURVEY.md
§8e, north_star: photon batches and image tiles over the GPUs of one node
with an RCCL all-gather of the photon slots before the gather).

One process drives every device: paths are sharded by global id, the 40-B
slots all-gathered (ncclAllGather when the devices are distinct, peer copies
otherwise), every device builds the same map and gathers its interleaved
8-row bands. The test box has one GPU, so the group runs as [0] (RCCL, world
size 1) and as [0, 0] (two sub-contexts on one device, the peer-copy
exchange and the band split). Either way the image must equal one context
rendering all the paths, bit for bit (exact fixed-point gather sums, the
same valid photons in the map)."""
import os
import subprocess

import numpy as np
import pytest

from pmrender import scenes
from pmrender.abi import PM_GATHER_GRID, PM_GATHER_KDTREE, PM_ESTIMATOR_KNN, RenderParams

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _render(sc, hip_mod, devices, p):
    ctx = sc.load_into(hip_mod.Context(0, devices=devices))
    try:
        return ctx.render(p)
    finally:
        ctx.close()


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
@pytest.mark.parametrize("structure,paths,passes", [(PM_GATHER_GRID, 16384, 2), (PM_GATHER_GRID, 10001, 1),
                                                    (PM_GATHER_KDTREE, 8192, 1)])
def test_group_render_equals_one_context(devices, structure, paths, passes, hip_mod):
    """[0]: the RCCL all-gather at world size 1; [0, 0] / [0, 0, 0]: peer
    copies and bands over two / three sub-contexts; 10,001 paths leave the
    last shard short (padding slots must be invalid)."""
    sc = scenes.cornell_box(80, 56)
    p = RenderParams.defaults(paths_per_pass=paths, passes=passes, gather_structure=structure, initial_radius2=25.0)
    want, st_want = _render(sc, hip_mod, None, p)
    got, st = _render(sc, hip_mod, devices, p)
    assert (want > 0).any()
    assert st["photons_valid"] == st_want["photons_valid"] > 0
    assert st["paths_emitted"] == paths * passes
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"group {devices} image differs"


def test_group_host_rays_and_knn(hip_mod):
    """Host eye rays (pbrt's sample order, the plugin's mode) and the kNN
    estimator through the group's band gathers."""
    sc = scenes.cornell_box(48, 40)
    sc.camera = scenes.rays_from_pinhole(sc)
    for p in (RenderParams.defaults(paths_per_pass=16384, initial_radius2=25.0),
              RenderParams.defaults(paths_per_pass=16384, initial_radius2=100.0, estimator=PM_ESTIMATOR_KNN,
                                    knn_lookup=20)):
        want, _ = _render(sc, hip_mod, None, p)
        got, _ = _render(sc, hip_mod, [0, 0], p)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_group_rejects_stage_api(hip_mod):
    from pmrender.hip import PMError
    sc = scenes.cornell_box(32, 32)
    ctx = sc.load_into(hip_mod.Context(0, devices=[0, 0]))
    try:
        assert ctx.num_records() == 32 * 32
        with pytest.raises(PMError, match="multi-device"):
            ctx.eye_pass(RenderParams.defaults())
    finally:
        ctx.close()


def test_plugin_on_device_list(tmp_path, hip_mod):
    """The pbrt-facing layer with PM_DEVICES (the plugin's device list): the
    .pbrt render on a [0, 0] group equals the single-device render."""
    cli = os.path.join(ROOT, "cuda-raytrace_amd", "lib", "pm_render_cli")
    scene = os.path.join(ROOT, "cuda-raytrace_amd", "scenes", "cornell-box.pbrt")
    imgs = []
    for env in ({}, {"PM_DEVICES": "0,0"}):
        out = tmp_path / f"img{len(imgs)}.pfm"
        r = subprocess.run([cli, "--pbrt", scene, "--paths", "16384", "--passes", "2", "--out", str(out)],
                           capture_output=True, text=True, timeout=300, env={**os.environ, **env})
        assert r.returncode == 0, r.stderr
        imgs.append(out.read_bytes())
    assert imgs[0] == imgs[1]


def _n_gpus():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


@pytest.mark.skipif(_n_gpus() < 2, reason="needs two GPUs (the one-GPU boxes run the same-device branches above)")
@pytest.mark.parametrize("rccl", ["1", "0"])
def test_group_distinct_devices(rccl, hip_mod, monkeypatch):
    """The branches only a node with distinct devices takes: ncclCommInitAll
    over devices [0, 1] with the in-place all-gather, and (PM_GROUP_RCCL=0)
    hipMemcpyPeerAsync between them — the image equals one context's."""
    monkeypatch.setenv("PM_GROUP_RCCL", rccl)
    sc = scenes.cornell_box(80, 56)
    p = RenderParams.defaults(paths_per_pass=10001, passes=2, initial_radius2=25.0)
    want, st_want = _render(sc, hip_mod, None, p)
    got, st = _render(sc, hip_mod, [0, 1], p)
    assert st["photons_valid"] == st_want["photons_valid"] > 0
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
