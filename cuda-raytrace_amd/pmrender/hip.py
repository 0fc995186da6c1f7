"""ctypes binding of libpmhip.so — the MI355X photon-mapping renderer.

This is a thin host-side mirror of the C-ABI (include/pm_api.h); every
compute call goes to HIP kernels. If the library is missing the import of
`Context` fails loudly: there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

from .abi import (PHOTON_DTYPE, RECORD_DTYPE, PM_ERR_NO_PHOTONS, PMConfig, RenderParams, Stats, f32, fptr, iptr,
                  record_pixels)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libpmhip.so")
_lib = None


class PMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"pm error {code}: {msg}")
        self.code = code


class NoPhotonsError(PMError):
    pass


def load_library(path=None):
    """Load libpmhip.so (built by `make -C cuda-raytrace_amd`). Raises if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("PMHIP_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise ImportError(f"libpmhip.so not found at {p}: build it with `make -C cuda-raytrace_amd` "
                          f"(there is no CPU fallback)")
    lib = ctypes.CDLL(p)
    vp, i64, c_int, c_float, c_double = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_double
    P_f, P_i = ctypes.POINTER(c_float), ctypes.POINTER(c_int)
    sig = {
        "pm_default_params": (None, [ctypes.POINTER(RenderParams)]),
        "pm_create": (c_int, [ctypes.POINTER(vp), vp]),
        "pm_destroy": (None, [vp]),
        "pm_last_error": (ctypes.c_char_p, [vp]),
        "pm_version": (ctypes.c_char_p, []),
        "pm_add_material": (c_int, [vp, c_int, P_f, P_i]),
        "pm_add_trimesh": (c_int, [vp, P_f, c_int, P_i, c_int, P_f, P_f, c_int, c_int]),
        "pm_add_object_mesh": (c_int, [vp, P_f, c_int, P_i, c_int, P_f, P_f, c_int, c_int, P_i]),
        "pm_add_mesh_instance": (c_int, [vp, c_int, P_f, P_f]),
        "pm_add_sphere": (c_int, [vp, c_float, P_f, P_f, c_int, c_int]),
        "pm_add_disk": (c_int, [vp, P_f, P_f, P_f, P_f, c_float, c_float, c_int, c_int]),
        "pm_add_light_point": (c_int, [vp, P_f, P_f]),
        "pm_add_light_disk": (c_int, [vp, P_f, P_f, P_f, P_f, P_f, c_float, c_int]),
        "pm_set_pinhole": (c_int, [vp, P_f, P_f, P_f, P_f, c_int, c_int]),
        "pm_set_eye_rays": (c_int, [vp, P_f, i64, P_f, c_int]),
        "pm_commit": (c_int, [vp]),
        "pm_render": (c_int, [vp, ctypes.POINTER(RenderParams), P_f, ctypes.POINTER(Stats)]),
        "pm_render_simple": (c_int, [vp, ctypes.POINTER(RenderParams), P_f, ctypes.POINTER(Stats)]),
        "pm_simple_pass": (c_int, [vp, ctypes.POINTER(RenderParams), vp, vp]),
        "pm_eye_pass": (c_int, [vp, ctypes.POINTER(RenderParams), vp]),
        "pm_trace_photons": (c_int, [vp, ctypes.POINTER(RenderParams), c_int, i64, i64, i64, vp]),
        "pm_build_photon_map": (c_int, [vp, ctypes.POINTER(RenderParams), i64, vp]),
        "pm_gather": (c_int, [vp, ctypes.POINTER(RenderParams), vp]),
        "pm_gather_partial": (c_int, [vp, ctypes.POINTER(RenderParams), vp, vp]),
        "pm_gather_split": (c_int, [vp, ctypes.POINTER(RenderParams), vp, vp, vp]),
        "pm_ppm_update_split": (c_int, [vp, ctypes.POINTER(RenderParams), vp, vp, i64, i64, vp]),
        "pm_ppm_update_split_radius": (c_int, [vp, ctypes.POINTER(RenderParams), vp, vp, vp]),
        "pm_ppm_update_split_flux": (c_int, [vp, ctypes.POINTER(RenderParams), vp, vp, i64, i64, vp]),
        "pm_ppm_update": (c_int, [vp, ctypes.POINTER(RenderParams), vp, i64, i64, vp]),
        "pm_final": (c_int, [vp, c_double, i64, i64, vp, vp]),
        "pm_num_records": (i64, [vp]),
        "pm_record_pixel": (c_int, [vp, i64, ctypes.POINTER(i64)]),
        "pm_reserve_slots": (c_int, [vp, i64, ctypes.POINTER(vp)]),
        "pm_download_slots": (c_int, [vp, vp, i64]),
        "pm_upload_slots": (c_int, [vp, vp, i64]),
        "pm_download_records": (c_int, [vp, vp, i64]),
        "pm_upload_records": (c_int, [vp, vp, i64]),
        "pm_kdtree_nodes": (i64, [vp]),
        "pm_download_kdtree": (c_int, [vp, vp, i64]),
        "pm_gather_counters": (c_int, [vp, ctypes.POINTER(i64)]),
        "pm_trace_counters": (c_int, [vp, ctypes.POINTER(i64)]),
        "pm_scene_info": (c_int, [vp, ctypes.POINTER(i64)]),
        "pm_scene_section": (c_int, [vp, c_int, vp, i64, ctypes.POINTER(i64)]),
        "pm_map_info": (c_int, [vp, ctypes.POINTER(i64)]),
        "pm_trace_profile": (c_int, [vp, ctypes.POINTER(i64), c_int]),
        "pm_set_counting": (c_int, [vp, c_int]),
        "pm_set_stage_timing": (c_int, [vp, ctypes.c_char_p]),
        "pm_set_record_view": (c_int, [vp, c_int, ctypes.POINTER(i64)]),
        "pm_final_view": (c_int, [vp, c_double, i64, i64, vp, vp]),
        "pm_record_view_list": (c_int, [vp, vp, vp]),
        "pm_synchronize": (c_int, [vp]),
        "pm_last_kernel_ms": (c_int, [vp, ctypes.c_char_p, ctypes.POINTER(c_double)]),
        "pm_halton_permutation": (c_int, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
        "pm_kdtree_build_host": (i64, [vp, i64, vp]),
        "pm_timing_reset": (c_int, [vp]),
        "pm_gather_range": (c_int, [vp, ctypes.POINTER(RenderParams), i64, i64, vp]),
        "pm_set_slot_buffer": (c_int, [vp, vp, i64]),
        "pm_get_radius2": (c_int, [vp, i64, i64, vp, vp]),
        "pm_set_radius2": (c_int, [vp, vp, i64, i64, vp]),
        "pm_timing_total": (c_int, [vp, ctypes.c_char_p, ctypes.POINTER(i64), ctypes.POINTER(c_double)]),
        "pm_reset_records": (c_int, [vp, ctypes.POINTER(RenderParams), vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


def halton_permutation(seed):
    lib = load_library()
    out = (ctypes.c_uint32 * 28)()
    lib.pm_halton_permutation(seed, out)
    return np.frombuffer(out, dtype=np.uint32).copy()


def kdtree_build_host(slots):
    """Canonical pbrt-v2 kd-tree over the valid slots (host, reference layout)."""
    lib = load_library()
    slots = np.ascontiguousarray(slots, dtype=PHOTON_DTYPE)
    nodes = np.zeros(len(slots), dtype=PHOTON_DTYPE)
    n = lib.pm_kdtree_build_host(slots.ctypes.data, len(slots), nodes.ctypes.data)
    return nodes[:n]


class Context:
    """One renderer context on one HIP device (cudarender.cpp's gContext)."""

    def __init__(self, device=0, devices=None):
        """devices: a list of device ordinals -> one multi-device context
        (pm_config::n_devices: scene calls, render() and render_simple()
        only; photon shards + RCCL all-gather + 8-row bands per device)."""
        self.lib = load_library()
        h = ctypes.c_void_p()
        cfg = PMConfig(device=device)
        if devices is not None:
            self._devlist = (ctypes.c_int * len(devices))(*devices)
            cfg.n_devices = len(devices)
            cfg.devices = ctypes.cast(self._devlist, ctypes.POINTER(ctypes.c_int))
        rc = self.lib.pm_create(ctypes.byref(h), ctypes.byref(cfg))
        if rc != 0:
            raise PMError(rc, self.lib.pm_last_error(None).decode())
        self.h = h
        self.device = device
        self.devices = list(devices) if devices is not None else [device]
        self.width = self.height = 0
        self.pinhole = False

    def close(self):
        if getattr(self, "h", None):
            self.lib.pm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        if rc != 0:
            msg = self.lib.pm_last_error(self.h).decode()
            if rc == PM_ERR_NO_PHOTONS:
                raise NoPhotonsError(rc, msg)
            raise PMError(rc, msg)

    # ---- scene (Scene.load_into protocol) ---------------------------------
    def add_material(self, mtype, rgb):
        out = ctypes.c_int()
        self._chk(self.lib.pm_add_material(self.h, int(mtype), fptr(f32(rgb, 3)), ctypes.byref(out)))
        return out.value

    def add_trimesh(self, P, idx, N=None, uv=None, material=0, light=-1):
        P = f32(P)
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        N, uv = f32(N), f32(uv)
        self._chk(self.lib.pm_add_trimesh(self.h, fptr(P), P.size // 3, iptr(idx), idx.size // 3, fptr(N), fptr(uv),
                                          int(material), int(light)))

    def add_object_mesh(self, P, idx, N=None, uv=None, material=0, light=-1):
        """A mesh stored once in object space (pm_add_object_mesh); returns its object id."""
        P = f32(P)
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        N, uv = f32(N), f32(uv)
        out = ctypes.c_int()
        self._chk(self.lib.pm_add_object_mesh(self.h, fptr(P), P.size // 3, iptr(idx), idx.size // 3, fptr(N),
                                              fptr(uv), int(material), int(light), ctypes.byref(out)))
        return out.value

    def add_mesh_instance(self, obj, o2w, w2o):
        """One instance of an object mesh (pm_add_mesh_instance): affine row-major 4x4 and its inverse."""
        self._chk(self.lib.pm_add_mesh_instance(self.h, int(obj), fptr(f32(o2w, 16)), fptr(f32(w2o, 16))))

    def add_sphere(self, r, o2w, w2o, material, light=-1):
        self._chk(self.lib.pm_add_sphere(self.h, float(r), fptr(f32(o2w, 16)), fptr(f32(w2o, 16)), int(material),
                                         int(light)))

    def add_disk(self, o, x, y, z, inner, phimax, material, light=-1):
        self._chk(self.lib.pm_add_disk(self.h, fptr(f32(o, 3)), fptr(f32(x, 3)), fptr(f32(y, 3)), fptr(f32(z, 3)),
                                       float(inner), float(phimax), int(material), int(light)))

    def add_light_point(self, pos, I):
        self._chk(self.lib.pm_add_light_point(self.h, fptr(f32(pos, 3)), fptr(f32(I, 3))))

    def add_light_disk(self, o, p1, p2, n, Le, area, nsamples):
        self._chk(self.lib.pm_add_light_disk(self.h, fptr(f32(o, 3)), fptr(f32(p1, 3)), fptr(f32(p2, 3)),
                                             fptr(f32(n, 3)), fptr(f32(Le, 3)), float(area), int(nsamples)))

    def set_pinhole(self, eye, fwd, right, up, W, H):
        self.width, self.height, self.pinhole = int(W), int(H), True
        self._chk(self.lib.pm_set_pinhole(self.h, fptr(f32(eye, 3)), fptr(f32(fwd, 3)), fptr(f32(right, 3)),
                                          fptr(f32(up, 3)), int(W), int(H)))

    def set_eye_rays(self, rays, rand2d=None, n2d=0):
        rays = f32(rays)
        rand2d = f32(rand2d)
        self.width, self.height, self.pinhole = rays.size // 6, 1, False
        self._chk(self.lib.pm_set_eye_rays(self.h, fptr(rays), rays.size // 6, fptr(rand2d), int(n2d)))

    def commit(self):
        self._chk(self.lib.pm_commit(self.h))

    # ---- whole render --------------------------------------------------------
    def render(self, params=None):
        params = params or RenderParams.defaults()
        n = self.width * self.height if self.pinhole else self.num_records()
        out = np.zeros((n, 3), np.float32)
        st = Stats()
        self._chk(self.lib.pm_render(self.h, ctypes.byref(params), fptr(out), ctypes.byref(st)))
        if self.pinhole:
            out = out.reshape(self.height, self.width, 3)
        return out, st.as_dict()

    def render_simple(self, params=None):
        """SimpleRenderer (simplerender.cpp:18-103): direct light only."""
        params = params or RenderParams.simple_defaults()
        n = self.width * self.height if self.pinhole else self.num_records()
        out = np.zeros((n, 3), np.float32)
        st = Stats()
        self._chk(self.lib.pm_render_simple(self.h, ctypes.byref(params), fptr(out), ctypes.byref(st)))
        if self.pinhole:
            out = out.reshape(self.height, self.width, 3)
        return out, st.as_dict()

    def simple_pass(self, params, d_out, stream=None):
        self._chk(self.lib.pm_simple_pass(self.h, ctypes.byref(params), d_out, stream))

    # ---- stages ---------------------------------------------------------------
    def eye_pass(self, params, stream=None):
        self._chk(self.lib.pm_eye_pass(self.h, ctypes.byref(params), stream))

    def trace_photons(self, params, pass_index=0, path_begin=0, path_count=None, slot_path_base=0, stream=None):
        if path_count is None:
            path_count = params.paths_per_pass
        self._chk(self.lib.pm_trace_photons(self.h, ctypes.byref(params), int(pass_index), int(path_begin),
                                            int(path_count), int(slot_path_base), stream))

    def build_photon_map(self, params, n_slots=0, stream=None):
        self._chk(self.lib.pm_build_photon_map(self.h, ctypes.byref(params), int(n_slots), stream))

    def gather(self, params, stream=None):
        self._chk(self.lib.pm_gather(self.h, ctypes.byref(params), stream))

    def gather_range(self, params, rec_begin, rec_count, stream=None):
        self._chk(self.lib.pm_gather_range(self.h, ctypes.byref(params), int(rec_begin), int(rec_count), stream))

    def set_slot_buffer(self, d_ptr, n_slots):
        self._chk(self.lib.pm_set_slot_buffer(self.h, ctypes.c_void_p(d_ptr) if d_ptr else None, int(n_slots)))

    def gather_partial(self, params, d_partial, stream=None):
        self._chk(self.lib.pm_gather_partial(self.h, ctypes.byref(params), ctypes.c_void_p(d_partial), stream))

    def gather_split(self, params, d_count, d_flux, stream=None):
        self._chk(self.lib.pm_gather_split(self.h, ctypes.byref(params), d_count, d_flux, stream))

    def ppm_update_split(self, params, d_count, d_flux_chunk, v_begin, v_count, stream=None):
        self._chk(self.lib.pm_ppm_update_split(self.h, ctypes.byref(params), d_count, d_flux_chunk, int(v_begin),
                                               int(v_count), stream))

    def ppm_update_split_radius(self, params, d_count, d_ratio, stream=None):
        self._chk(self.lib.pm_ppm_update_split_radius(self.h, ctypes.byref(params), d_count, d_ratio, stream))

    def ppm_update_split_flux(self, params, d_ratio, d_flux_chunk, v_begin, v_count, stream=None):
        self._chk(self.lib.pm_ppm_update_split_flux(self.h, ctypes.byref(params), d_ratio, d_flux_chunk,
                                                    int(v_begin), int(v_count), stream))

    def ppm_update(self, params, d_partial, rec_begin, rec_count, stream=None):
        self._chk(self.lib.pm_ppm_update(self.h, ctypes.byref(params), ctypes.c_void_p(d_partial), int(rec_begin),
                                         int(rec_count), stream))

    def get_radius2(self, rec_begin, rec_count, d_out, stream=None):
        self._chk(self.lib.pm_get_radius2(self.h, int(rec_begin), int(rec_count), ctypes.c_void_p(d_out), stream))

    def set_radius2(self, d_in, rec_begin, rec_count, stream=None):
        self._chk(self.lib.pm_set_radius2(self.h, ctypes.c_void_p(d_in), int(rec_begin), int(rec_count), stream))

    def final(self, emitted, rec_begin, rec_count, d_out, stream=None):
        self._chk(self.lib.pm_final(self.h, float(emitted), int(rec_begin), int(rec_count), ctypes.c_void_p(d_out),
                                    stream))

    def final_image(self, emitted):
        """pm_final over all records into a torch device buffer, returned on the
        host in the oracle's layout: (H, W, 3) raster for pinhole, else per ray."""
        import torch
        n = self.num_records()
        d = torch.empty((n, 3), dtype=torch.float32, device=f"cuda:{self.device}")
        torch.cuda.synchronize()
        self.final(emitted, 0, n, d.data_ptr())
        self.synchronize()
        out = d.cpu().numpy()
        if not self.pinhole:
            return out
        img = np.zeros((self.height * self.width, 3), np.float32)
        pix = self.record_pixels()
        ok = pix >= 0
        img[pix[ok]] = out[ok]
        return img.reshape(self.height, self.width, 3)

    # ---- buffers ----------------------------------------------------------------
    def num_records(self):
        return int(self.lib.pm_num_records(self.h))

    def record_pixels(self):
        n = self.num_records()
        if not self.pinhole:
            return np.arange(n, dtype=np.int64)
        return record_pixels(n, self.width, self.height)

    def reserve_slots(self, n):
        p = ctypes.c_void_p()
        self._chk(self.lib.pm_reserve_slots(self.h, int(n), ctypes.byref(p)))
        return p.value

    def download_slots(self, n):
        out = np.zeros(n, dtype=PHOTON_DTYPE)
        self._chk(self.lib.pm_download_slots(self.h, out.ctypes.data, n))
        return out

    def upload_slots(self, slots):
        slots = np.ascontiguousarray(slots, dtype=PHOTON_DTYPE)
        self._chk(self.lib.pm_upload_slots(self.h, slots.ctypes.data, len(slots)))

    def download_records(self):
        n = self.num_records()
        out = np.zeros(n, dtype=RECORD_DTYPE)
        self._chk(self.lib.pm_download_records(self.h, out.ctypes.data, n))
        return out

    def upload_records(self, recs):
        recs = np.ascontiguousarray(recs, dtype=RECORD_DTYPE)
        self._chk(self.lib.pm_upload_records(self.h, recs.ctypes.data, len(recs)))

    def download_kdtree(self):
        n = int(self.lib.pm_kdtree_nodes(self.h))
        out = np.zeros(max(n, 0), dtype=PHOTON_DTYPE)
        if n > 0:
            self._chk(self.lib.pm_download_kdtree(self.h, out.ctypes.data, n))
        return out

    def set_record_view(self, active_only=True):
        """Index record-range calls by active records only (compacted); returns the view size."""
        n = ctypes.c_int64()
        self._chk(self.lib.pm_set_record_view(self.h, int(bool(active_only)), ctypes.byref(n)))
        return int(n.value)

    def final_view(self, emitted, v_begin, v_count, d_out, stream=None):
        self._chk(self.lib.pm_final_view(self.h, float(emitted), int(v_begin), int(v_count), ctypes.c_void_p(d_out),
                                         stream))

    def record_view_list(self, d_out, stream=None):
        self._chk(self.lib.pm_record_view_list(self.h, ctypes.c_void_p(d_out), stream))

    def set_stage_timing(self, stages="all"):
        """Stages that record HIP events: "all", "" (none) or e.g. "gather"."""
        self._chk(self.lib.pm_set_stage_timing(self.h, (stages or "").encode()))

    def set_counting(self, enabled=True):
        self._chk(self.lib.pm_set_counting(self.h, int(bool(enabled))))

    def gather_counters(self, full=False):
        """(visited, in_radius) or, with full=True, (visited, in_radius, bucket_rows, active_records)."""
        out = (ctypes.c_int64 * 4)()
        self._chk(self.lib.pm_gather_counters(self.h, out))
        vals = tuple(int(v) for v in out)
        return vals if full else vals[:2]

    def trace_counters(self):
        """(rays traced, BVH nodes entered, primitive tests, photons deposited) of the last
        trace_photons launched with counting on."""
        out = (ctypes.c_int64 * 4)()
        self._chk(self.lib.pm_trace_counters(self.h, out))
        return tuple(int(v) for v in out)

    def scene_info(self):
        """dict: triangles, disks, spheres, bvh_nodes, bvh_depth, mode ("bvh-hbm" | "bvh-lds" | "brute"), bytes."""
        out = (ctypes.c_int64 * 7)()
        self._chk(self.lib.pm_scene_info(self.h, out))
        v = [int(x) for x in out]
        return {"triangles": v[0], "disks": v[1], "spheres": v[2], "bvh_nodes": v[3], "bvh_depth": v[4],
                "mode": ("bvh-hbm", "bvh-lds", "brute", "bvh-instanced")[v[5]], "bytes": v[6]}

    SCENE_SECTIONS = {"refs": (0, np.uint32), "tri_geo": (1, np.float32), "tri_shade": (2, np.float32),
                      "tri_id": (3, np.uint32), "tri_info": (4, np.int32), "bvh4": (5, np.uint32),
                      "instances": (6, np.float32), "obj_tris": (7, np.float32)}

    def scene_section(self, name):
        """One section of the committed scene blob as the kernels read it (pm_scene_section)."""
        sec, dt = self.SCENE_SECTIONS[name]
        n = ctypes.c_int64()
        self._chk(self.lib.pm_scene_section(self.h, sec, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value // 4, dtype=dt)
        if n.value:
            self._chk(self.lib.pm_scene_section(self.h, sec, out.ctypes.data, n.value, ctypes.byref(n)))
        return out

    def map_info(self):
        """dict: structure (PM_GATHER_*, -1 none), valid photons, slots, grid cells of the current photon map."""
        out = (ctypes.c_int64 * 4)()
        self._chk(self.lib.pm_map_info(self.h, out))
        v = [int(x) for x in out]
        return {"structure": v[0], "valid": v[1], "slots": v[2], "cells": v[3]}

    def trace_profile(self, reset=False):
        """k_trace phase cycles (profiling builds, lib/libpmhip_prof.so): dict of summed cycles."""
        out = (ctypes.c_int64 * 8)()
        self._chk(self.lib.pm_trace_profile(self.h, out, int(bool(reset))))
        keys = ("emit", "traverse", "shade", "compact_barrier", "exchange", "unused", "lifetime", "waves")
        return dict(zip(keys, (int(v) for v in out)))

    def synchronize(self):
        self._chk(self.lib.pm_synchronize(self.h))

    def timing_reset(self):
        self._chk(self.lib.pm_timing_reset(self.h))

    def timing_total(self, name):
        n, ms = ctypes.c_int64(), ctypes.c_double()
        self._chk(self.lib.pm_timing_total(self.h, name.encode(), ctypes.byref(n), ctypes.byref(ms)))
        return int(n.value), ms.value

    def reset_records(self, params, stream=None):
        self._chk(self.lib.pm_reset_records(self.h, ctypes.byref(params), stream))

    def last_ms(self, name):
        ms = ctypes.c_double()
        self._chk(self.lib.pm_last_kernel_ms(self.h, name.encode(), ctypes.byref(ms)))
        return ms.value
