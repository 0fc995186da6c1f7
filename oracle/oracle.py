"""ctypes binding of the CPU oracle (liborc.so) — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, and only as the checker. Parity status: unpinned (see the
header of pm_oracle.cpp and DESIGN.md §oracle).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "cuda-raytrace_amd"))
from pmrender.abi import PHOTON_DTYPE, RECORD_DTYPE, RenderParams, Stats, f32, fptr, iptr  # noqa: E402

LIB_PATH = os.path.join(_HERE, "liborc.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    vp, i64, c_int, c_float, c_double = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_double
    P_f, P_i, P_u = ctypes.POINTER(c_float), ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_uint32)
    RP = ctypes.POINTER(RenderParams)
    sig = {
        "orc_create": (vp, []),
        "orc_destroy": (None, [vp]),
        "orc_add_material": (c_int, [vp, c_int, P_f]),
        "orc_add_trimesh": (c_int, [vp, P_f, c_int, P_i, c_int, P_f, P_f, c_int, c_int]),
        "orc_add_sphere": (c_int, [vp, c_float, P_f, P_f, c_int, c_int]),
        "orc_add_disk": (c_int, [vp, P_f, P_f, P_f, P_f, c_float, c_float, c_int, c_int]),
        "orc_add_light_point": (c_int, [vp, P_f, P_f]),
        "orc_add_light_disk": (c_int, [vp, P_f, P_f, P_f, P_f, P_f, c_float, c_int]),
        "orc_set_pinhole": (c_int, [vp, P_f, P_f, P_f, P_f, c_int, c_int]),
        "orc_set_eye_rays": (c_int, [vp, P_f, i64, P_f, c_int]),
        "orc_commit": (c_int, [vp]),
        "orc_num_records": (i64, [vp]),
        "orc_eye_pass": (None, [vp, RP, vp, c_int]),
        "orc_halton_permutation": (None, [ctypes.c_uint32, P_u]),
        "orc_halton_sample": (None, [ctypes.c_uint32, P_u, P_f]),
        "orc_trace_photons": (None, [vp, RP, c_int, i64, i64, vp, c_int]),
        "orc_build_kdtree": (i64, [vp, i64, vp]),
        "orc_gather": (None, [vp, vp, i64, vp, i64, RP, ctypes.POINTER(i64), c_int]),
        "orc_gather_partial": (None, [vp, vp, i64, vp, i64, vp, c_int]),
        "orc_final": (None, [vp, vp, i64, c_double, P_f, c_int]),
        "orc_final_est": (None, [vp, vp, i64, c_double, c_int, P_f, c_int]),
        "orc_render": (c_int, [vp, RP, P_f, ctypes.POINTER(Stats), c_int]),
        "orc_render_simple": (None, [vp, RP, P_f, c_int]),
        "orc_concentric_sample_disk": (None, [c_float, c_float, P_f]),
        "orc_uniform_sample_sphere": (None, [c_float, c_float, P_f]),
        "orc_intersect_triangle": (c_int, [P_f, P_f, P_f, P_f, P_f, c_float, c_float, P_f]),
        "orc_intersect_disk": (c_int, [P_f, P_f, P_f, P_f, c_float, c_float, P_f, P_f, c_float, c_float, P_f]),
        "orc_intersect_sphere": (c_int, [c_float, P_f, P_f, P_f, P_f, c_float, c_float, P_f]),
        "orc_ppm_update": (None, [P_f, P_f, P_f, c_int, P_f, c_float]),
        "orc_philox": (None, [P_u, P_u, P_u]),
        "orc_sinf": (c_float, [c_float]),
        "orc_cosf": (c_float, [c_float]),
        "orc_atan2f": (c_float, [c_float, c_float]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def nthreads_default():
    return int(os.environ.get("PM_ORACLE_THREADS", min(16, os.cpu_count() or 1)))


class Oracle:
    """Scene + passes on the CPU; same Scene.load_into protocol as the HIP Context."""

    def __init__(self, nthreads=None):
        self.lib = load()
        self.h = self.lib.orc_create()
        self.nthreads = nthreads or nthreads_default()
        self.width = self.height = 0
        self.pinhole = False

    def __del__(self):
        try:
            if self.h:
                self.lib.orc_destroy(self.h)
                self.h = None
        except Exception:
            pass

    # scene
    def add_material(self, mtype, rgb):
        return self.lib.orc_add_material(self.h, int(mtype), fptr(f32(rgb, 3)))

    def add_trimesh(self, P, idx, N=None, uv=None, material=0, light=-1):
        P = f32(P)
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        N, uv = f32(N), f32(uv)
        self.lib.orc_add_trimesh(self.h, fptr(P), P.size // 3, iptr(idx), idx.size // 3, fptr(N), fptr(uv),
                                 int(material), int(light))

    def add_sphere(self, r, o2w, w2o, material, light=-1):
        self.lib.orc_add_sphere(self.h, float(r), fptr(f32(o2w, 16)), fptr(f32(w2o, 16)), int(material), int(light))

    def add_disk(self, o, x, y, z, inner, phimax, material, light=-1):
        self.lib.orc_add_disk(self.h, fptr(f32(o, 3)), fptr(f32(x, 3)), fptr(f32(y, 3)), fptr(f32(z, 3)),
                              float(inner), float(phimax), int(material), int(light))

    def add_light_point(self, pos, I):
        self.lib.orc_add_light_point(self.h, fptr(f32(pos, 3)), fptr(f32(I, 3)))

    def add_light_disk(self, o, p1, p2, n, Le, area, nsamples):
        self.lib.orc_add_light_disk(self.h, fptr(f32(o, 3)), fptr(f32(p1, 3)), fptr(f32(p2, 3)), fptr(f32(n, 3)),
                                    fptr(f32(Le, 3)), float(area), int(nsamples))

    def set_pinhole(self, eye, fwd, right, up, W, H):
        self.width, self.height, self.pinhole = int(W), int(H), True
        self.lib.orc_set_pinhole(self.h, fptr(f32(eye, 3)), fptr(f32(fwd, 3)), fptr(f32(right, 3)),
                                 fptr(f32(up, 3)), int(W), int(H))

    def set_eye_rays(self, rays, rand2d=None, n2d=0):
        rays, rand2d = f32(rays), f32(rand2d)
        self.width, self.height, self.pinhole = rays.size // 6, 1, False
        self.lib.orc_set_eye_rays(self.h, fptr(rays), rays.size // 6, fptr(rand2d), int(n2d))

    def commit(self):
        self.lib.orc_commit(self.h)

    # passes
    def num_records(self):
        return int(self.lib.orc_num_records(self.h))

    def eye_pass(self, params):
        recs = np.zeros(self.num_records(), dtype=RECORD_DTYPE)
        self.lib.orc_eye_pass(self.h, ctypes.byref(params), recs.ctypes.data, self.nthreads)
        return recs

    def trace_photons(self, params, pass_index=0, path_begin=0, path_count=None):
        if path_count is None:
            path_count = params.paths_per_pass
        slots = np.zeros(path_count * params.max_photon_count, dtype=PHOTON_DTYPE)
        self.lib.orc_trace_photons(self.h, ctypes.byref(params), int(pass_index), int(path_begin), int(path_count),
                                   slots.ctypes.data, self.nthreads)
        return slots

    @staticmethod
    def build_kdtree(slots):
        lib = load()
        slots = np.ascontiguousarray(slots, dtype=PHOTON_DTYPE)
        nodes = np.zeros(len(slots), dtype=PHOTON_DTYPE)
        n = lib.orc_build_kdtree(slots.ctypes.data, len(slots), nodes.ctypes.data)
        return nodes[:n]

    def gather(self, nodes, recs, params):
        """In-place kd-tree gather: range query + PPM update, or (params.estimator
        == PM_ESTIMATOR_KNN) pbrt's k-nearest lookup + LPhoton sum; returns
        (kd nodes visited, photons in radius / found)."""
        cnt = (ctypes.c_int64 * 2)()
        self.lib.orc_gather(self.h, nodes.ctypes.data, len(nodes), recs.ctypes.data, len(recs), ctypes.byref(params),
                            cnt, self.nthreads)
        return int(cnt[0]), int(cnt[1])

    def gather_partial(self, nodes, recs):
        """Per-record (M, L.rgb) without the PPM update (float32 [n,4])."""
        out = np.zeros((len(recs), 4), np.float32)
        self.lib.orc_gather_partial(self.h, nodes.ctypes.data, len(nodes), recs.ctypes.data, len(recs),
                                    out.ctypes.data, self.nthreads)
        return out

    def final(self, recs, emitted, estimator=0):
        n = self.width * self.height if self.pinhole else len(recs)
        out = np.zeros((n, 3), np.float32)
        self.lib.orc_final_est(self.h, recs.ctypes.data, len(recs), float(emitted), int(estimator), fptr(out),
                               self.nthreads)
        return out.reshape(self.height, self.width, 3) if self.pinhole else out

    def render(self, params):
        n = self.width * self.height if self.pinhole else self.num_records()
        out = np.zeros((n, 3), np.float32)
        st = Stats()
        rc = self.lib.orc_render(self.h, ctypes.byref(params), fptr(out), ctypes.byref(st), self.nthreads)
        if rc != 0:
            raise RuntimeError(f"oracle render failed ({rc})")
        if self.pinhole:
            out = out.reshape(self.height, self.width, 3)
        return out, st.as_dict()

    def render_simple(self, params):
        """SimpleRenderer (simplerender.cpp:18-103): direct light only."""
        n = self.width * self.height if self.pinhole else self.num_records()
        out = np.zeros((n, 3), np.float32)
        self.lib.orc_render_simple(self.h, ctypes.byref(params), fptr(out), self.nthreads)
        return out.reshape(self.height, self.width, 3) if self.pinhole else out


# ---- primitive KAT helpers ---------------------------------------------------
def philox(ctr, key):
    lib = load()
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib.orc_philox(c, k, o)
    return list(o)


def halton_permutation(seed):
    lib = load()
    out = (ctypes.c_uint32 * 28)()
    lib.orc_halton_permutation(seed, out)
    return np.frombuffer(out, dtype=np.uint32).copy()


def halton_sample(n, perm):
    lib = load()
    perm = np.ascontiguousarray(perm, dtype=np.uint32)
    out = np.zeros(4, np.float32)
    lib.orc_halton_sample(n, perm.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), fptr(out))
    return out
