"""The `simple` renderer (SimpleRenderer, simple_render/simplerender.cpp:18-103
+ simplerender.cu): direct light only.

CPU: the oracle's restatement against analytic values (point light over a
matte quad: |ns.wi| * Kd/pi * I/d^2, no pdf division, no emission) and
against the photon mapper's direct-light term, which equals it for point
lights (pdf 1) on non-emitting diffuse hits at the same epsilon.
GPU: the HIP kernel (k_simple) bit-exact against the oracle in all three
traversal modes (brute / LDS / global BVH) and both eye-sample modes.
"""
import math

import numpy as np
import pytest

from pmrender import scenes
from pmrender.abi import PM_MATTE, PM_MIRROR, PM_REC_EXCEPTION, PM_REC_INVALID, PM_REC_MISS, RenderParams, \
    record_pixels


def plane_scene(W=16, H=16, I=(1000.0, 2000.0, 500.0), kd=(0.5, 0.25, 0.75), light=(0.0, 10.0, 0.0)):
    """A 200x200 matte quad at y=0 under a point light, camera looking down."""
    s = scenes.Scene()
    m = s.material(PM_MATTE, kd)
    s.add_quads([[(-100, 0, -100), (-100, 0, 100), (100, 0, 100), (100, 0, -100)]], m)
    s.lights.append(("point", np.float32(light), np.float32(I)))
    # pinhole straight down from y=50: fwd -y, right +x, up +z (narrow fov)
    s.camera = ("pinhole", np.float32([0, 50, 0]), np.float32([0, -1, 0]), np.float32([0.2, 0, 0]),
                np.float32([0, 0, 0.2]), W, H)
    return s


def test_simple_point_light_analytic(oracle_mod):
    s = plane_scene()
    orc = s.load_into(oracle_mod.Oracle(nthreads=2))
    img = orc.render_simple(RenderParams.simple_defaults())
    _, eye, f, r, u, W, H = s.camera
    kd = np.float32([0.5, 0.25, 0.75])
    I = np.float32([1000.0, 2000.0, 500.0])
    for py, px in [(0, 0), (7, 9), (15, 15), (3, 12)]:
        sx = 2.0 * (px + 0.5) / W - 1.0
        sy = 1.0 - 2.0 * (py + 0.5) / H
        d = f + sx * r + sy * u
        d = d / np.linalg.norm(d)
        t = 50.0 / -d[1]
        p = eye + t * d
        to_l = np.float32([0, 10, 0]) - p
        d2 = float(to_l @ to_l)
        cos = abs(to_l[1]) / math.sqrt(d2)
        want = cos * kd / math.pi * I / d2
        np.testing.assert_allclose(img[py, px], want, rtol=2e-5)


def test_simple_shadow_and_miss(oracle_mod):
    s = plane_scene()
    # an occluder between the light and the centre of the plane
    occ = s.material(PM_MATTE, (1, 1, 1))
    s.add_quads([[(-5, 5, -5), (5, 5, -5), (5, 5, 5), (-5, 5, 5)]], occ)
    orc = s.load_into(oracle_mod.Oracle(nthreads=2))
    img = orc.render_simple(RenderParams.simple_defaults())
    # the occluder faces the camera (hit), is lit from above only through its
    # back: |ns.wi| is two-sided in the reference, so it is lit
    assert img[8, 8].sum() > 0
    # plane points shadowed by the occluder: ring around the occluder's shadow
    s2 = plane_scene(light=(0.0, 10.0, 0.0))
    s2.camera = ("pinhole", np.float32([0, 50, 0]), np.float32([0, -1, 0]), np.float32([4.0, 0, 0]),
                 np.float32([0, 0, 4.0]), 8, 8)          # wide fov: corners miss the plane
    orc2 = s2.load_into(oracle_mod.Oracle(nthreads=2))
    img2 = orc2.render_simple(RenderParams.simple_defaults())
    assert np.all(img2[0, 0] == 0)                         # miss -> black (simplerender.cu:75-79)


def test_simple_equals_eye_direct_light_for_point_lights(oracle_mod):
    """For point lights (pdf 1, one sample) the photon mapper's direct light on
    a non-emitting diffuse hit is the simple renderer's sum."""
    s = scenes.cornell_box(40, 32)
    s.lights = [("point", np.float32([278, 500, 279.5]), np.float32([30000, 30000, 30000])),
                ("point", np.float32([100, 300, 100]), np.float32([5000, 8000, 3000]))]
    orc = s.load_into(oracle_mod.Oracle(nthreads=2))
    p = RenderParams.simple_defaults()
    img = orc.render_simple(p)
    recs = orc.eye_pass(p)
    pix = record_pixels(len(recs), 40, 32)
    ok = (pix >= 0) & ((recs["flags"] & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) == 0)
    flat = img.reshape(-1, 3)
    assert ok.sum() > 800
    np.testing.assert_array_equal(flat[pix[ok]].view(np.uint32), recs["dl"][ok].view(np.uint32))


def test_simple_specular_hit_is_black(oracle_mod):
    """f() is 0 for mirror / glass (cudamaterial.cu.h:23-32): no chain is followed."""
    s = plane_scene()
    s.materials[0] = (PM_MIRROR, np.float32([1, 1, 1]))
    orc = s.load_into(oracle_mod.Oracle(nthreads=2))
    img = orc.render_simple(RenderParams.simple_defaults())
    assert np.all(img == 0)


# ---------------------------------------------------------------- GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cornell", "feature", "caustic", "soup", "instanced", "cornell_rays", "feature_rays"])
def test_simple_gpu_bitexact(name, oracle_mod, hip_mod):
    if name.startswith("cornell"):
        s = scenes.cornell_box(64, 48)
    elif name.startswith("feature"):
        s = scenes.feature_scene()
    elif name == "caustic":
        s = scenes.caustic_scene(48, 40)
    elif name == "instanced":   # two-level trees (MODE_INST) on the GPU, flattened in the oracle
        s = scenes.instanced_scene(64, 48)
    else:
        s = scenes.triangle_soup(20000, 64, 40)
    if name.endswith("_rays"):
        s.camera = scenes.rays_from_pinhole(s)
    ctx = s.load_into(hip_mod.Context(0))
    orc = s.load_into(oracle_mod.Oracle())
    p = RenderParams.simple_defaults()
    img, st = ctx.render_simple(p)
    ref = orc.render_simple(p)
    assert img.shape == ref.shape
    assert (ref.reshape(-1, 3).sum(axis=1) > 0).mean() > 0.2
    np.testing.assert_array_equal(img.view(np.uint32), ref.view(np.uint32))
    ctx.close()
