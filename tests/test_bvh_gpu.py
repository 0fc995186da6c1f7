"""The scene BVH built on the device (csrc/pm_bvh_gpu.hip: PLOC over Morton-
sorted primitive boxes, collapsed to the quantized 4-wide nodes on the
device). The reference has OptiX build its acceleration structure on the GPU
at the first launch (cuda_render/cudarender.cpp:38-75, :118-119).

Parity has two layers:
  * the device tree equals its host restatement (pm_build.cpp build_ploc +
    ploc_to_bvh + collapse_bvh4 + bvh4_bfs_order + quantize_bvh4, selected
    with PM_BVH_BUILD=ploc-host PM_BVH4_BFS=1) bit for bit: the quantized
    nodes, the refs, and the triangle records in storage order;
  * closest hits do not depend on the tree (conservative culling, ties to the
    lowest primitive id), so rendering through the device tree equals
    rendering through the host binned-SAH tree bit for bit, and the oracle
    parity of the full C3 workload (test_gpu_configs.py::test_c3_full_workload)
    runs on the device tree, the default for scenes of >= 65,536 primitives."""
import numpy as np
import pytest

from pmrender import scenes
from pmrender.abi import PM_MATTE, RenderParams

pytestmark = pytest.mark.gpu

SECTIONS = ("refs", "tri_geo", "tri_shade", "tri_id", "tri_info", "bvh4")


def _soup(n, W=48, H=40, sphere=True):
    s = scenes.triangle_soup(n, W, H)
    if sphere:  # a sphere and the ceiling disk light: refs that are not triangles
        o2w, w2o = scenes.translate(300.0, 200.0, 260.0)
        s.spheres.append((np.float32(40.0), o2w, w2o, s.material(PM_MATTE, (0.6, 0.6, 0.6)), -1))
    return s


def _commit(sc, hip_mod, monkeypatch, env):
    for k in ("PM_BVH_BUILD", "PM_BVH4_BFS", "PM_PLOC_RADIUS", "PM_BVH_GPU_MIN"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    return sc.load_into(hip_mod.Context(0))


@pytest.mark.parametrize("n,radius", [(3000, "3"), (40000, "3"), (40000, "1"), (40000, "8"), (120000, "3")])
def test_device_tree_equals_host_restatement(n, radius, hip_mod, monkeypatch):
    sc = _soup(n)
    dev = _commit(sc, hip_mod, monkeypatch, {"PM_BVH_BUILD": "gpu", "PM_PLOC_RADIUS": radius})
    host = _commit(sc, hip_mod, monkeypatch, {"PM_BVH_BUILD": "ploc-host", "PM_BVH4_BFS": "1", "PM_PLOC_RADIUS": radius})
    try:
        di, hi = dev.scene_info(), host.scene_info()
        assert di["mode"] == hi["mode"] == "bvh-hbm"
        assert di["triangles"] == hi["triangles"] > n
        for name in SECTIONS:
            a, b = dev.scene_section(name), host.scene_section(name)
            assert a.size > 0 and a.shape == b.shape, name
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), f"{name} differs"
    finally:
        dev.close()
        host.close()


def test_device_tree_renders_as_the_sah_tree(hip_mod, monkeypatch):
    """Closest hits are tree-independent: photon slots and the image through
    the device PLOC tree equal those through the host binned-SAH tree."""
    sc = _soup(30000)
    p = RenderParams.defaults(paths_per_pass=8192, initial_radius2=100.0)
    out = []
    for env in ({"PM_BVH_BUILD": "gpu"}, {"PM_BVH_BUILD": "host"}):
        ctx = _commit(sc, hip_mod, monkeypatch, env)
        try:
            img, st = ctx.render(p)
            ctx.eye_pass(p)
            ctx.trace_photons(p, 0, 0, 8192)
            ctx.synchronize()
            out.append((img, st, ctx.download_slots(8192 * 4)))
        finally:
            ctx.close()
    (ig, sg, pg), (ih, sh, ph) = out
    assert sg["photons_valid"] == sh["photons_valid"] > 0
    assert np.array_equal(pg.view(np.uint8), ph.view(np.uint8))
    assert np.array_equal(ig.view(np.uint32), ih.view(np.uint32))


def test_auto_uses_device_build_for_large_scenes(hip_mod, monkeypatch):
    """Default (unset PM_BVH_BUILD): >= PM_BVH_GPU_MIN primitives take the
    device build (no binary tree: scene bytes well below the host blob)."""
    sc = _soup(70000, sphere=False)
    dev = _commit(sc, hip_mod, monkeypatch, {})
    host = _commit(sc, hip_mod, monkeypatch, {"PM_BVH_BUILD": "host"})
    try:
        assert dev.scene_info()["bytes"] < host.scene_info()["bytes"]
        assert dev.scene_section("bvh4").size > 0
    finally:
        dev.close()
        host.close()
