"""Synthetic scenes of BASELINE.json's configurations.

A Scene is plain data (numpy float32 arrays) that `load_into` pushes through
the C-ABI calls of either the HIP renderer or the CPU oracle, so both see
bit-identical inputs.

* cornell_box: the classic 555-unit Cornell box (two blocks), ceiling disk
  area light r=65 at (278, 548.7, 279.5) facing -y, Lemit 17, pinhole
  camera at (278, 273, -800), fov 39.3 deg (C1, C2, C4).
* triangle_soup: Cornell enclosure + N random triangles, centres
  U[30,525]^3, edges U[-4,4]^3, Kd 0.5 (reference default matte,
  cudamaterial.cpp:40), numpy seed 1 (C3).
* caustic_scene: Cornell box + glass sphere r=100 (+ mirror sphere) (C5
  substitute; killeroo/caustic-glass .pbrt files are not in the container).
* figure_scene: Cornell enclosure + two instances of a procedural 5,120-
  triangle closed mesh (killeroo substitute, scenes/killeroo-proxy.pbrt).
"""
import math
from dataclasses import dataclass, field

import numpy as np

from .abi import PM_GLASS, PM_MATTE, PM_MIRROR

WHITE = (0.73, 0.73, 0.73)
RED = (0.63, 0.065, 0.05)
GREEN = (0.14, 0.45, 0.091)


@dataclass
class Scene:
    materials: list = field(default_factory=list)   # (type, rgb)
    meshes: list = field(default_factory=list)      # dict(P, idx, N, uv, material, light)
    spheres: list = field(default_factory=list)     # (r, o2w, w2o, material, light)
    disks: list = field(default_factory=list)       # (o, x, y, z, inner, phimax, material, light)
    lights: list = field(default_factory=list)      # ("point", pos, I) | ("disk", o, p1, p2, n, Le, area, ns)
    objects: list = field(default_factory=list)     # object meshes (as meshes), placed by `instances` only
    instances: list = field(default_factory=list)   # (object index, o2w 4x4, w2o 4x4), affine
    camera: tuple = None                            # ("pinhole", eye, fwd, right, up, W, H) | ("rays", rays, rand2d, n2d)

    def material(self, mtype, rgb):
        self.materials.append((mtype, np.asarray(rgb, np.float32)))
        return len(self.materials) - 1

    def add_quads(self, quads, material, light=-1):
        P, idx = [], []
        for q in quads:
            b = len(P)
            P.extend(q)
            idx.append((b, b + 1, b + 2))
            idx.append((b, b + 2, b + 3))
        self.meshes.append(dict(P=np.asarray(P, np.float32), idx=np.asarray(idx, np.int32), N=None, uv=None,
                                material=material, light=light))

    @property
    def num_triangles(self):
        """triangles rendered (an object mesh once per instance)"""
        return sum(len(m["idx"]) for m in self.meshes) + sum(len(self.objects[o]["idx"]) for o, _, _ in self.instances)

    def flattened(self, k):
        """Instance k as the world-space mesh pbrt's Transform gives (the
        adapter's flattening, pm_cudarender.cpp): points m[0]*x + m[1]*y +
        m[2]*z + m[3] per row, left to right, in float32; normals through the
        transpose of w2o."""
        o, m, mi = self.objects[self.instances[k][0]], *self.instances[k][1:]
        m = np.asarray(m, np.float32).reshape(4, 4)
        mi = np.asarray(mi, np.float32).reshape(4, 4)
        P = np.asarray(o["P"], np.float32).reshape(-1, 3)
        W = np.stack([((m[a, 0] * P[:, 0] + m[a, 1] * P[:, 1]) + m[a, 2] * P[:, 2]) + m[a, 3] for a in range(3)], 1)
        N = o.get("N")
        if N is not None:
            N = np.asarray(N, np.float32).reshape(-1, 3)
            N = np.stack([(mi[0, a] * N[:, 0] + mi[1, a] * N[:, 1]) + mi[2, a] * N[:, 2] for a in range(3)], 1)
        return dict(o, P=W.astype(np.float32), N=N)

    def load_into(self, api, instancing=True):
        """The scene through the C-ABI calls of `api`. Object instances go in
        as pm_add_object_mesh / pm_add_mesh_instance (two-level) when the api
        has them and `instancing`, else flattened (the CPU oracle; the A/B
        of the two-level trees) — after the meshes either way, so the global
        ids are the same."""
        for mtype, rgb in self.materials:
            api.add_material(mtype, rgb)
        for m in self.meshes:
            api.add_trimesh(m["P"], m["idx"], m.get("N"), m.get("uv"), m["material"], m["light"])
        if self.instances and instancing and hasattr(api, "add_mesh_instance"):
            ids = {}
            for k, (oi, o2w, w2o) in enumerate(self.instances):
                if oi not in ids:
                    o = self.objects[oi]
                    ids[oi] = api.add_object_mesh(o["P"], o["idx"], o.get("N"), o.get("uv"), o["material"], o["light"])
                api.add_mesh_instance(ids[oi], o2w, w2o)
        else:
            for k in range(len(self.instances)):
                m = self.flattened(k)
                api.add_trimesh(m["P"], m["idx"], m.get("N"), m.get("uv"), m["material"], m["light"])
        for r, o2w, w2o, mat, light in self.spheres:
            api.add_sphere(r, o2w, w2o, mat, light)
        for o, x, y, z, inner, phimax, mat, light in self.disks:
            api.add_disk(o, x, y, z, inner, phimax, mat, light)
        for L in self.lights:
            if L[0] == "point":
                api.add_light_point(L[1], L[2])
            else:
                api.add_light_disk(*L[1:])
        cam = self.camera
        if cam[0] == "pinhole":
            api.set_pinhole(*cam[1:])
        else:
            api.set_eye_rays(*cam[1:])
        api.commit()
        return api

    @property
    def width(self):
        return self.camera[5] if self.camera[0] == "pinhole" else len(self.camera[1])

    @property
    def height(self):
        return self.camera[6] if self.camera[0] == "pinhole" else 1


def pinhole(W, H, eye=(278.0, 273.0, -800.0), look=(278.0, 273.0, 0.0), up=(0.0, 1.0, 0.0), fov_deg=39.3):
    """pbrt-style perspective camera: fov spans the shorter image axis;
    image x grows towards -x world (red wall on the left, classic view)."""
    e = np.asarray(eye, np.float64)
    f = np.asarray(look, np.float64) - e
    f /= np.linalg.norm(f)
    u = np.asarray(up, np.float64)
    r = np.cross(f, u)          # right-handed: +z forward, +y up -> right = -x
    r /= np.linalg.norm(r)
    u = np.cross(r, f)
    t = math.tan(math.radians(fov_deg) / 2.0)
    sx, sy = (t * W / H, t) if W >= H else (t, t * H / W)
    return ("pinhole", np.float32(e), np.float32(f), np.float32(r * sx), np.float32(u * sy), int(W), int(H))


def _ceiling_light(scene, Le=17.0, radius=65.0, nsamples=1, material=None):
    """Disk area light facing -y (pbrt Disk under Rotate 90 about x)."""
    o = np.float32([278.0, 548.7, 279.5])
    x = np.float32([radius, 0.0, 0.0])
    y = np.float32([0.0, 0.0, radius])
    z = np.float32([0.0, -1.0, 0.0])
    n = np.float32([0.0, -1.0, 0.0])
    phimax = np.float32(2.0 * math.pi)
    area = np.float32(phimax * np.float32(0.5) * np.float32(radius * radius))  # pbrt Disk::Area
    if material is None:
        material = scene.material(PM_MATTE, (0.0, 0.0, 0.0))
    light_id = len(scene.lights)
    scene.lights.append(("disk", o, x, y, n, np.float32([Le, Le, Le]), area, nsamples))
    scene.disks.append((o, x, y, z, np.float32(0.0), phimax, material, light_id))
    return light_id


def _walls(scene):
    white = scene.material(PM_MATTE, WHITE)
    red = scene.material(PM_MATTE, RED)
    green = scene.material(PM_MATTE, GREEN)
    scene.add_quads([
        [(552.8, 0, 0), (0, 0, 0), (0, 0, 559.2), (549.6, 0, 559.2)],                      # floor
        [(556.0, 548.8, 0), (556.0, 548.8, 559.2), (0, 548.8, 559.2), (0, 548.8, 0)],      # ceiling
        [(549.6, 0, 559.2), (0, 0, 559.2), (0, 548.8, 559.2), (556.0, 548.8, 559.2)],      # back
    ], white)
    scene.add_quads([[(0, 0, 559.2), (0, 0, 0), (0, 548.8, 0), (0, 548.8, 559.2)]], green)              # right wall x=0
    scene.add_quads([[(552.8, 0, 0), (549.6, 0, 559.2), (556.0, 548.8, 559.2), (556.0, 548.8, 0)]], red)  # left wall
    return white


def cornell_box(W=256, H=256, blocks=True, nsamples=1):
    s = Scene()
    white = _walls(s)
    if blocks:
        s.add_quads([  # short block
            [(130, 165, 65), (82, 165, 225), (240, 165, 272), (290, 165, 114)],
            [(290, 0, 114), (290, 165, 114), (240, 165, 272), (240, 0, 272)],
            [(130, 0, 65), (130, 165, 65), (290, 165, 114), (290, 0, 114)],
            [(82, 0, 225), (82, 165, 225), (130, 165, 65), (130, 0, 65)],
            [(240, 0, 272), (240, 165, 272), (82, 165, 225), (82, 0, 225)],
        ], white)
        s.add_quads([  # tall block
            [(423, 330, 247), (265, 330, 296), (314, 330, 456), (472, 330, 406)],
            [(423, 0, 247), (423, 330, 247), (472, 330, 406), (472, 0, 406)],
            [(472, 0, 406), (472, 330, 406), (314, 330, 456), (314, 0, 456)],
            [(314, 0, 456), (314, 330, 456), (265, 330, 296), (265, 0, 296)],
            [(265, 0, 296), (265, 330, 296), (423, 330, 247), (423, 0, 247)],
        ], white)
    _ceiling_light(s, nsamples=nsamples)
    s.camera = pinhole(W, H)
    return s


def triangle_soup(n_tris=1_000_000, W=1920, H=1080, seed=1):
    s = Scene()
    _walls(s)
    grey = s.material(PM_MATTE, (0.5, 0.5, 0.5))
    rng = np.random.RandomState(seed)
    c = rng.uniform(30.0, 525.0, size=(n_tris, 3)).astype(np.float32)
    e1 = rng.uniform(-4.0, 4.0, size=(n_tris, 3)).astype(np.float32)
    e2 = rng.uniform(-4.0, 4.0, size=(n_tris, 3)).astype(np.float32)
    P = np.empty((n_tris * 3, 3), np.float32)
    P[0::3] = c
    P[1::3] = c + e1
    P[2::3] = c + e2
    idx = np.arange(n_tris * 3, dtype=np.int32).reshape(n_tris, 3)
    s.meshes.append(dict(P=P, idx=idx, N=None, uv=None, material=grey, light=-1))
    _ceiling_light(s)
    s.camera = pinhole(W, H)
    return s


def translate(tx, ty, tz):
    m = np.eye(4, dtype=np.float32)
    m[:3, 3] = (tx, ty, tz)
    inv = np.eye(4, dtype=np.float32)
    inv[:3, 3] = (-tx, -ty, -tz)
    return m.reshape(-1), inv.reshape(-1)


def affine(yaw_deg=0.0, pitch_deg=0.0, scale=(1.0, 1.0, 1.0), t=(0.0, 0.0, 0.0)):
    """o2w = T * Ry(yaw) * Rx(pitch) * S and its inverse (float64 math, float32 out)."""
    a, b = math.radians(yaw_deg), math.radians(pitch_deg)
    ry = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    rx = np.array([[1, 0, 0], [0, math.cos(b), -math.sin(b)], [0, math.sin(b), math.cos(b)]])
    m = np.eye(4)
    m[:3, :3] = ry @ rx @ np.diag(scale)
    m[:3, 3] = t
    return m.astype(np.float32).reshape(-1), np.linalg.inv(m).astype(np.float32).reshape(-1)


def instanced_scene(W=80, H=64, subdiv=2):
    """Two-level test scene: the figure mesh three times under rotations and
    non-uniform scales (one mirror object among them), plus a shading-normal
    + uv quad object (one degenerate-uv triangle) placed twice. Built for the
    two-level vs flattened A/B (tests/test_gpu_parity.py)."""
    s = cornell_box(W, H, blocks=False)
    blue = s.material(PM_MATTE, (0.5, 0.5, 0.8))
    mir = s.material(PM_MIRROR, (0.9, 0.9, 0.9))
    tan = s.material(PM_MATTE, (0.8, 0.6, 0.3))
    P, idx = figure_mesh(subdiv)
    s.objects.append(dict(P=P, idx=idx, N=None, uv=None, material=blue, light=-1))
    s.objects.append(dict(P=P, idx=idx, N=None, uv=None, material=mir, light=-1))
    Pq = np.float32([[-60, 0, 0], [60, 10, 20], [0, 120, -20], [70, 140, 30]])
    Nq = np.float32([[0, 0, -1], [0.2, 0, -1], [-0.2, 0.1, -1], [0, 0.3, -1]])
    uvq = np.float32([[0, 0], [1, 0], [0, 1], [0, 1]])
    s.objects.append(dict(P=Pq, idx=np.int32([[0, 1, 2], [0, 2, 3]]), N=Nq, uv=uvq, material=tan, light=-1))
    s.instances.append((0, *affine(30.0, 0.0, (1.2, 0.8, 1.0), (170.0, 0.0, 220.0))))
    s.instances.append((0, *affine(-75.0, 10.0, (0.7, 0.7, 0.9), (400.0, 40.0, 380.0))))
    s.instances.append((1, *affine(140.0, 0.0, (0.6, 0.9, 0.6), (300.0, 200.0, 150.0))))
    s.instances.append((2, *affine(20.0, -15.0, (1.0, 1.0, 1.0), (120.0, 300.0, 420.0))))
    s.instances.append((2, *affine(-160.0, 0.0, (0.8, 1.3, 0.8), (430.0, 250.0, 120.0))))
    return s


def caustic_scene(W=256, H=256, mirror=True):
    s = cornell_box(W, H, blocks=False)
    glass = s.material(PM_GLASS, (1.0, 1.0, 1.0))
    o2w, w2o = translate(370.0, 100.0, 250.0)
    s.spheres.append((np.float32(100.0), o2w, w2o, glass, -1))
    if mirror:
        mir = s.material(PM_MIRROR, (0.9, 0.9, 0.9))
        o2w, w2o = translate(150.0, 90.0, 380.0)
        s.spheres.append((np.float32(90.0), o2w, w2o, mir, -1))
    return s


FIGURE_INSTANCES = ((180.0, 0.0, 200.0), (370.0, 0.0, 340.0))


def figure_mesh(subdiv=4):
    """Killeroo substitute (the killeroo mesh is not in the container): a
    closed, smoothly bumped blob — an icosphere subdivided `subdiv` times
    (20 * 4^subdiv triangles), displaced radially and scaled to ~140 x 180 x
    110 units, resting above y = 0. Coordinates are multiples of 1/64, so the
    float32 values round-trip through a .pbrt file's decimal text exactly."""
    t = (1.0 + math.sqrt(5.0)) / 2.0
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    V = [np.asarray(v, np.float64) / np.linalg.norm(v) for v in V]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    for _ in range(subdiv):
        mid = {}

        def midpoint(a, b):
            k = (min(a, b), max(a, b))
            if k not in mid:
                m = V[a] + V[b]
                V.append(m / np.linalg.norm(m))
                mid[k] = len(V) - 1
            return mid[k]

        F2 = []
        for a, b, c in F:
            ab, bc, ca = midpoint(a, b), midpoint(b, c), midpoint(c, a)
            F2 += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        F = F2
    P = np.asarray(V)
    x, y, z = P[:, 0], P[:, 1], P[:, 2]
    r = 1.0 + 0.18 * np.sin(3.0 * x + 1.0) * np.cos(2.0 * y) + 0.12 * np.sin(4.0 * z) * np.sin(2.0 * x + y)
    P = P * r[:, None] * np.asarray([70.0, 90.0, 55.0])
    P[:, 1] -= P[:, 1].min() - 1.0
    P = np.round(P * 64.0) / 64.0
    return P.astype(np.float32), np.asarray(F, np.int32)


def figure_scene(W=256, H=256, subdiv=4):
    """killeroo-proxy.pbrt as an in-code scene: the Cornell enclosure and
    ceiling light with two instances of `figure_mesh` (pbrt ObjectInstance,
    flattened to world space like the adapter, translations only) in a
    bluish matte. The BVH exceeds the 16 KB LDS budget, so this is a global
    (4-wide BVH, pooled trace kernel) scene of moderate size."""
    s = cornell_box(W, H, blocks=False)
    blue = s.material(PM_MATTE, (0.5, 0.5, 0.8))
    P, idx = figure_mesh(subdiv)
    s.objects.append(dict(P=P, idx=idx, N=None, uv=None, material=blue, light=-1))
    for t in FIGURE_INSTANCES:
        o2w, w2o = translate(*t)
        s.instances.append((0, o2w, w2o))
    return s


def feature_scene(W=72, H=40):
    """Small scene exercising the less common paths: mesh with per-vertex
    normals and uvs, a degenerate-uv triangle, partial disk with an inner
    radius, point light + disk light with 2 shadow samples, W/H not multiples
    of 8 (padding records)."""
    s = Scene()
    _walls(s)
    shiny = s.material(PM_MATTE, (0.8, 0.6, 0.3))
    P = np.float32([[200, 50, 300], [350, 60, 320], [260, 220, 260], [330, 240, 330]])
    N = np.float32([[0, 0, -1], [0.2, 0, -1], [-0.2, 0.1, -1], [0, 0.3, -1]])
    uv = np.float32([[0, 0], [1, 0], [0, 1], [0, 1]])  # (0,2,3): uv2==uv3 -> degenerate determinant
    s.meshes.append(dict(P=P, idx=np.int32([[0, 1, 2], [0, 2, 3]]), N=N, uv=uv, material=shiny, light=-1))
    ring = s.material(PM_MATTE, (0.3, 0.7, 0.7))
    s.disks.append((np.float32([420, 120, 300]), np.float32([60, 0, 0]), np.float32([0, 60, 0]),
                    np.float32([0, 0, 1]), np.float32(0.3), np.float32(4.5), ring, -1))
    _ceiling_light(s, nsamples=2)
    s.lights.append(("point", np.float32([100, 400, 100]), np.float32([20000, 18000, 15000])))
    mir = s.material(PM_MIRROR, (1, 1, 1))
    o2w, w2o = translate(120.0, 60.0, 420.0)
    s.spheres.append((np.float32(60.0), o2w, w2o, mir, -1))
    s.camera = pinhole(W, H)
    return s


def rays_from_pinhole(scene, jitter_seed=5):
    """Host-generated eye rays in sampler order with per-ray 2D light samples
    (the PbrtCamera::preLaunch packing, pbrtcamera.cpp:57-122)."""
    _, eye, f, r, u, W, H = scene.camera
    rng = np.random.RandomState(jitter_seed)
    py, px = np.mgrid[0:H, 0:W]
    sx = (2.0 * (px + rng.uniform(0, 1, px.shape)) / W - 1.0)
    sy = 1.0 - 2.0 * (py + rng.uniform(0, 1, py.shape)) / H
    d = f[None, None, :] + sx[..., None] * r[None, None, :] + sy[..., None] * u[None, None, :]
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    rays = np.concatenate([np.broadcast_to(eye, d.shape), d], axis=-1).reshape(-1, 6).astype(np.float32)
    n2d = sum(L[7] for L in scene.lights if L[0] == "disk")
    rand2d = rng.uniform(0, 1, size=(rays.shape[0], max(n2d, 1), 2)).astype(np.float32)
    return ("rays", rays, rand2d, max(n2d, 1))
