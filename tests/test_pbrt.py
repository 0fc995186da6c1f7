"""pbrt-v2 scene files through the pbrt-facing layer (adapter/pm_pbrt.h,
SURVEY.md §8f row 3): the parser issues the plugin calls pbrt-v2's api.cpp
would (CreateCudaShape / CudaObjectInstance / lights / camera).

CPU (`pm_render_cli --pbrt f --dump`, no device): the committed Cornell and
caustic scenes parse to exactly the scenes of pmrender/scenes.py, and pbrt-v2
semantics (post-multiplied CTM, Rotate / Scale / LookAt, AttributeBegin/End,
point light "from" + CTM, "scale", named materials, constant textures,
ObjectBegin/Instance, fallbacks) come out as pbrt defines them.
GPU: rendering the .pbrt file through the C++ layer gives the same image, bit
for bit, as the Python stage driver on the in-code scene — photon mapping and
the simple renderer — and matches the CPU oracle on that scene (simple
renderer bit for bit, photon mapping within RMSE 1e-3).
"""
import json
import math
import os
import subprocess

import numpy as np
import pytest

from pmrender import scenes
from pmrender.abi import PM_GATHER_GRID, RenderParams

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "cuda-raytrace_amd", "lib", "pm_render_cli")
SCENES = os.path.join(ROOT, "cuda-raytrace_amd", "scenes")

pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="adapter CLI not built (make -C cuda-raytrace_amd)")


def dump(path):
    r = subprocess.run([CLI, "--pbrt", str(path), "--dump"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout), r.stderr


def parse_text(tmp_path, text):
    f = tmp_path / "t.pbrt"
    f.write_text(text)
    return dump(f)


def f32(a):
    return np.asarray(a, np.float32)


def check_camera(d, cam):
    _, eye, fwd, right, up, W, H = cam
    c = d["camera"]
    assert (c["width"], c["height"]) == (W, H)
    for k, v in (("eye", eye), ("fwd", fwd), ("right", right), ("up", up)):
        np.testing.assert_array_equal(f32(c[k]), f32(v), err_msg=k)


def test_cornell_pbrt_is_the_c2_scene():
    d, err = dump(os.path.join(SCENES, "cornell-box.pbrt"))
    sc = scenes.cornell_box(256, 256)
    shapes = [c for c in d["calls"] if c["call"] == "shape"]
    meshes = [c for c in shapes if c["name"] == "trianglemesh"]
    assert len(meshes) == len(sc.meshes) == 5
    for got, want in zip(meshes, sc.meshes):
        np.testing.assert_array_equal(f32(got["P"]), want["P"].reshape(-1))
        np.testing.assert_array_equal(np.int32(got["indices"]), want["idx"].reshape(-1))
        np.testing.assert_array_equal(f32(got["k"]), sc.materials[want["material"]][1])
        assert got["light"] == -1
    disks = [c for c in shapes if c["name"] == "disk"]
    assert len(disks) == 1 and disks[0]["light"] == 0
    (L,) = d["lights"]
    assert L["kind"] == "disk" and L["nsamples"] == 1 and L["Le"] == [17, 17, 17]
    m = f32(L["o2w"]).reshape(4, 4)
    r, h = L["radius_height_inner_phimax"][0], L["radius_height_inner_phimax"][1]
    _, o, p1, p2, n, Le, area, ns = sc.lights[0]
    np.testing.assert_array_equal((m @ f32([0, 0, h, 1]))[:3], o)
    np.testing.assert_array_equal((m[:3, :3] @ f32([r, 0, 0])), p1)
    np.testing.assert_array_equal((m[:3, :3] @ f32([0, r, 0])), p2)
    assert np.float32(L["radius_height_inner_phimax"][3]) == np.float32(2 * math.pi)
    check_camera(d, sc.camera)
    assert d["renderer"] == "photonmapping" and d["paths"] == 262144 and d["passes"] == 1
    assert d["warnings"] == 0, err


def test_caustic_pbrt_is_the_c5_substitute():
    d, err = dump(os.path.join(SCENES, "caustic-glass.pbrt"))
    sc = scenes.caustic_scene(256, 256)
    spheres = [c for c in d["calls"] if c["name"] == "sphere"]
    assert len(spheres) == len(sc.spheres) == 2
    for got, (r, o2w, w2o, mat, light) in zip(spheres, sc.spheres):
        assert np.float32(got["radius_height_inner_phimax"][0]) == r
        np.testing.assert_array_equal(f32(got["o2w"]), o2w)
        np.testing.assert_array_equal(f32(got["w2o"]), w2o)
        assert got["material"] == {0: 0, 1: 1, 2: 2}[sc.materials[mat][0]]  # Matte/Mirror/Glass enum order
    check_camera(d, sc.camera)
    assert d["passes"] == 4 and d["warnings"] == 0, err


def test_killeroo_proxy_pbrt_is_the_figure_scene():
    """scenes/killeroo-proxy.pbrt (killeroo substitute): one figure mesh
    defined inside ObjectBegin and two ObjectInstance calls whose
    translations, applied as the adapter flattens instances, give exactly
    figure_scene()'s meshes."""
    d, err = dump(os.path.join(SCENES, "killeroo-proxy.pbrt"))
    sc = scenes.figure_scene(256, 256)
    calls = d["calls"]
    proto = [c for c in calls if c["call"] == "shape" and c.get("instance", -1) == 0]
    insts = [c for c in calls if c["call"] == "instance"]
    assert len(proto) == 1 and len(insts) == len(scenes.FIGURE_INSTANCES) == 2
    P, idx = scenes.figure_mesh()
    np.testing.assert_array_equal(f32(proto[0]["P"]), P.reshape(-1))
    np.testing.assert_array_equal(np.int32(proto[0]["indices"]), idx.reshape(-1))
    np.testing.assert_array_equal(f32(proto[0]["k"]), f32([0.5, 0.5, 0.8]))
    figs = [sc.flattened(k) for k in range(len(sc.instances))]
    for inst, want in zip(insts, figs):
        m = f32(inst["o2w"]).reshape(4, 4)
        assert np.array_equal(m[:3, :3], np.eye(3, dtype=np.float32))
        np.testing.assert_array_equal((P + m[:3, 3]).astype(np.float32), want["P"])
    assert sc.num_triangles == 10 + 2 * len(idx) and len(idx) == 5120
    check_camera(d, sc.camera)
    assert d["warnings"] == 0, err


def test_pbrt_transform_and_state_semantics(tmp_path):
    d, err = parse_text(tmp_path, """
        LookAt 0 0 0  0 0 1  0 1 0
        Camera "perspective" "float fov" [90]
        Film "image" "integer xresolution" [20] "integer yresolution" [10]
        WorldBegin
        Texture "kd" "color" "constant" "color value" [0.1 0.2 0.3]
        MakeNamedMaterial "shiny" "string type" ["mirror"]
        AttributeBegin
          Translate 1 2 3
          Rotate 90 0 0 1
          Scale 2 2 2
          LightSource "point" "rgb I" [10 20 30] "rgb scale" [2 2 2] "point from" [5 0 0]
          Material "matte" "texture Kd" "kd"
          Shape "sphere" "float radius" [0.5]
        AttributeEnd
        NamedMaterial "shiny"
        Shape "disk" "float radius" [2] "float innerradius" [1] "float phimax" [90] "float height" [0.25]
        Material "plastic" "rgb Kd" [1 1 1]
        Shape "trianglemesh" "integer indices" [0 1 2] "point P" [0 0 0 1 0 0 0 1 0] "normal N" [0 0 1 0 0 1 0 0 1]
          "float uv" [0 0 1 0 0 1]
        Shape "cylinder" "float radius" [1]
        ObjectBegin "pair"
          Shape "sphere" "float radius" [3]
        ObjectEnd
        AttributeBegin
          Translate 0 0 10
          ObjectInstance "pair"
        AttributeEnd
        WorldEnd
    """)
    calls = d["calls"]
    sph, disk, mesh, cyl, inst_sphere, inst = calls
    # CTM = T(1,2,3) * Rz(90) * S(2): the sphere's object-to-world maps (1,0,0) -> (1,4,3)
    m = f32(sph["o2w"]).reshape(4, 4)
    np.testing.assert_allclose((m @ f32([1, 0, 0, 1]))[:3], [1, 4, 3], atol=1e-6)
    np.testing.assert_allclose(f32(sph["w2o"]).reshape(4, 4) @ m, np.eye(4), atol=1e-6)
    assert sph["material"] == 0 and sph["k"] == pytest.approx([0.1, 0.2, 0.3])  # constant texture Kd
    # pbrt-v2 point light: Translate(from) * light2world applied to the origin
    (pl,) = d["lights"]
    np.testing.assert_allclose(pl["pos"], [1 + 5, 2, 3], atol=1e-6)
    assert pl["I"] == [20, 40, 60]
    # AttributeEnd restored the CTM and material; NamedMaterial -> mirror (default Kr 0.9)
    np.testing.assert_array_equal(f32(disk["o2w"]), np.eye(4, dtype=np.float32).reshape(-1))
    assert disk["material"] == 1 and disk["k"] == pytest.approx([0.9] * 3)
    r, h, inner, phimax = disk["radius_height_inner_phimax"]
    assert (r, h, inner) == (2, 0.25, 1) and phimax == pytest.approx(math.pi / 2)
    # unknown material -> reference fallback matte 0.5 (material kind 3 = Unknown)
    assert mesh["material"] == 3 and mesh["N"] == [0, 0, 1] * 3 and mesh["uv"] == [0, 0, 1, 0, 0, 1]
    # unsupported shapes are handed to CreateCudaShape (which warns and skips them)
    assert cyl["name"] == "cylinder"
    assert inst_sphere["instance"] == 0 and inst["call"] == "instance" and inst["instance"] == 0
    np.testing.assert_array_equal(f32(inst["o2w"]).reshape(4, 4)[:3, 3], [0, 0, 10])
    # camera: LookAt along +z, fov 90 spans the shorter (y) axis, 2:1 frame
    c = d["camera"]
    np.testing.assert_allclose(c["fwd"], [0, 0, 1], atol=1e-7)
    np.testing.assert_allclose(c["right"], [2, 0, 0], atol=1e-6)  # pbrt camera x = cross(up, dir) = +x
    np.testing.assert_allclose(c["up"], [0, 1, 0], atol=1e-6)
    assert d["warnings"] == 1  # "plastic"


def test_pbrt_mesh_vertices_in_world_space_normals_raw(tmp_path):
    """pbrt's TriangleMesh keeps P in world space and N as given
    (cudatrianglemesh.cpp:24-51 copies both)."""
    d, _ = parse_text(tmp_path, """
        Camera "perspective"
        WorldBegin
        Translate 10 0 0
        Shape "trianglemesh" "integer indices" [0 1 2] "point P" [0 0 0 1 0 0 0 1 0] "normal N" [1 0 0 1 0 0 1 0 0]
        WorldEnd
    """)
    (mesh,) = d["calls"]
    assert mesh["P"] == [10, 0, 0, 11, 0, 0, 10, 1, 0]
    assert mesh["N"] == [1, 0, 0] * 3


def test_pbrt_area_light_rules(tmp_path):
    """Only disks emit (cudalight.cpp:35-56): a sphere under an area light is
    a plain shape plus a warning; "scale" and "nsamples" reach the light."""
    d, err = parse_text(tmp_path, """
        Camera "perspective"
        WorldBegin
        AttributeBegin
          AreaLightSource "diffuse" "rgb L" [1 2 3] "rgb scale" [2 2 2] "integer nsamples" [4]
          Shape "sphere"
          Shape "disk" "float radius" [3]
        AttributeEnd
        Shape "disk"
        LightSource "spot"
        WorldEnd
    """)
    sph, disk, plain = d["calls"]
    assert sph["light"] == -1 and disk["light"] == 0 and plain["light"] == -1
    (L,) = d["lights"]
    assert L["Le"] == [2, 4, 6] and L["nsamples"] == 4
    assert d["warnings"] == 2 and "UnImplemented" in err


@pytest.mark.parametrize("text,msg", [
    ("WorldBegin Shape \"trianglemesh\" \"integer indices\" [0 1 5] \"point P\" [0 0 0 1 0 0 0 1 0] WorldEnd",
     "out of range"),
    ("WorldBegin AttributeEnd", "unmatched AttributeEnd"),
    ("Bogus 1 2 3", "unknown directive"),
    ("Camera \"orthographic\"", "perspective only"),
    ("WorldBegin ObjectInstance \"nope\"", "not defined"),
])
def test_pbrt_errors_name_file_and_line(tmp_path, text, msg):
    f = tmp_path / "bad.pbrt"
    f.write_text("# header\n" + text + "\n")
    r = subprocess.run([CLI, "--pbrt", str(f), "--dump"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert msg in r.stderr and "bad.pbrt:2" in r.stderr


# ---------------------------------------------------------------- GPU
def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), "<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3)[::-1]


@pytest.mark.gpu
@pytest.mark.parametrize("scene,renderer", [("cornell-box", "photonmapping"), ("cornell-box", "simple"),
                                            ("caustic-glass", "photonmapping"), ("caustic-glass", "simple"),
                                            ("killeroo-proxy", "photonmapping"), ("killeroo-proxy", "simple")])
def test_pbrt_render_matches_stage_driver(scene, renderer, tmp_path, hip_mod, oracle_mod):
    paths, passes = 16384, 2
    out = tmp_path / "img.pfm"
    r = subprocess.run([CLI, "--pbrt", os.path.join(SCENES, scene + ".pbrt"), "--renderer", renderer,
                        "--paths", str(paths), "--passes", str(passes), "--out", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    img = read_pfm(out)
    sc = {"cornell-box": scenes.cornell_box, "caustic-glass": scenes.caustic_scene,
          "killeroo-proxy": scenes.figure_scene}[scene](256, 256)
    ctx = sc.load_into(hip_mod.Context(0))
    orc = sc.load_into(oracle_mod.Oracle())
    if renderer == "simple":
        ref, _ = ctx.render_simple(RenderParams.simple_defaults())
        want = orc.render_simple(RenderParams.simple_defaults())
    else:
        p = RenderParams.defaults(paths_per_pass=paths, passes=passes, gather_structure=PM_GATHER_GRID)
        ref, _ = ctx.render(p)
        want, _ = orc.render(p)
    ctx.close()
    assert img.shape == ref.shape
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f"{scene}/{renderer}: .pbrt image differs"
    # the .pbrt render vs the CPU oracle of the same scene: the simple
    # renderer bit for bit, photon mapping (bucket gather) within RMSE 1e-3
    want = np.asarray(want, np.float32).reshape(img.shape)
    if renderer == "simple":
        assert np.array_equal(img.view(np.uint32), want.view(np.uint32)), f"{scene}/simple: differs from the oracle"
    else:
        err = float(np.sqrt(np.mean((img.astype(np.float64) - want) ** 2)))
        assert err < 1e-3, f"{scene}: .pbrt image vs oracle RMSE {err}"


@pytest.mark.gpu
def test_pbrt_instancing_two_level_equals_flattened(tmp_path):
    """killeroo-proxy.pbrt's ObjectInstance through the adapter: the two-level
    path (pm_add_object_mesh + pm_add_mesh_instance, the default) and the
    flattened one (PM_INSTANCING=0) render the same image bit for bit."""
    imgs = {}
    for inst in ("1", "0"):
        out = tmp_path / ("img%s.pfm" % inst)
        env = dict(os.environ, PM_INSTANCING=inst)
        r = subprocess.run([CLI, "--pbrt", os.path.join(SCENES, "killeroo-proxy.pbrt"), "--paths", "16384",
                            "--passes", "2", "--out", str(out)], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        imgs[inst] = read_pfm(out)
    assert np.array_equal(imgs["1"].view(np.uint32), imgs["0"].view(np.uint32))
