"""ctypes mirrors of the POD types in include/pm_api.h (shared by the HIP
binding in hip.py and by the oracle binding in oracle/oracle.py)."""
import ctypes

import numpy as np

PM_OK = 0
PM_ERR_INVALID = 1
PM_ERR_HIP = 2
PM_ERR_NO_PHOTONS = 3
PM_ERR_NOMEM = 4

PM_MATTE, PM_MIRROR, PM_GLASS = 0, 1, 2
PM_LIGHT_POINT, PM_LIGHT_AREA_DISK = 1, 3
PM_REC_EXCEPTION, PM_REC_MISS, PM_REC_INVALID, PM_REC_BACKFACE = 0x1, 0x2, 0x4, 0x8
PM_REC_INACTIVE = PM_REC_EXCEPTION | PM_REC_MISS | PM_REC_INVALID
PM_GATHER_GRID, PM_GATHER_KDTREE = 0, 1
PM_ESTIMATOR_PPM, PM_ESTIMATOR_KNN = 0, 1
PM_KNN_MAX = 64
PM_PHOTON_MAX_RIGHT_CHILD = (1 << 29) - 1

# pm_photon == reference CudaPhoton (photon_mapping/photonmapping.h:32-41), 40 B
PHOTON_DTYPE = np.dtype([("bits", "<u4"), ("p", "<f4", 3), ("alpha", "<f4", 3), ("wi", "<f4", 3)])
assert PHOTON_DTYPE.itemsize == 40
# pm_record (subset of RayTracingRecord, photonmapping.h:7-24), 64 B
RECORD_DTYPE = np.dtype([
    ("pos", "<f4", 3), ("flags", "<u4"), ("ns", "<f4", 3), ("material", "<i4"),
    ("flux", "<f4", 3), ("radius2", "<f4"), ("dl", "<f4", 3), ("photon_count", "<f4"),
])
assert RECORD_DTYPE.itemsize == 64


class PMConfig(ctypes.Structure):
    """include/pm_api.h pm_config (32 B)."""
    _fields_ = [
        ("device", ctypes.c_int),
        ("n_devices", ctypes.c_int),
        ("devices", ctypes.POINTER(ctypes.c_int)),
        ("reserved", ctypes.c_int * 4),
    ]


class RenderParams(ctypes.Structure):
    """pm_render_params; defaults are the reference's hard-coded constants."""
    _fields_ = [
        ("scene_epsilon", ctypes.c_float),
        ("initial_radius2", ctypes.c_float),
        ("ppm_alpha", ctypes.c_float),
        ("max_photon_count", ctypes.c_int),
        ("paths_per_pass", ctypes.c_int64),
        ("passes", ctypes.c_int),
        ("light_source_index", ctypes.c_int),
        ("max_specular_depth", ctypes.c_int),
        ("rng_seed", ctypes.c_uint32),
        ("light_rng_seed", ctypes.c_uint32),
        ("gather_structure", ctypes.c_int),
        ("estimator", ctypes.c_int),
        ("knn_lookup", ctypes.c_int),
        ("reserved", ctypes.c_int * 4),
    ]

    @classmethod
    def defaults(cls, **kw):
        p = cls()
        p.scene_epsilon = 0.1        # photonmappingrenderer.cpp:52
        p.initial_radius2 = 4.0      # raytracing.cu:123
        p.ppm_alpha = 0.7            # gathering.cu:115
        p.max_photon_count = 4       # photonmappingrenderer.cpp:183
        p.paths_per_pass = 512 * 512  # photonmappingrenderer.cpp:184-185
        p.passes = 1                 # photonmappingrenderer.cpp:38
        p.light_source_index = 0     # photonmappingrenderer.cpp:211
        p.max_specular_depth = 10    # raytracing.cu:98
        p.rng_seed = 777             # cudarandom.h:15
        p.light_rng_seed = 2047
        p.gather_structure = PM_GATHER_GRID
        p.estimator = PM_ESTIMATOR_PPM
        p.knn_lookup = 50            # pbrt-v2 PhotonIntegrator "nused"
        return p._apply(kw)

    @classmethod
    def simple_defaults(cls, **kw):
        """the SimpleRenderer's constants: scene_epsilon 0.01 (simplerender.cpp:23)"""
        p = cls.defaults()
        p.scene_epsilon = 0.01
        return p._apply(kw)

    def _apply(self, kw):
        p = self
        for k, v in kw.items():
            if not hasattr(p, k):
                raise AttributeError(f"unknown render parameter {k!r}")
            setattr(p, k, v)
        return p


class Stats(ctypes.Structure):
    _fields_ = [
        ("paths_emitted", ctypes.c_int64),
        ("photons_valid", ctypes.c_int64),
        ("gather_points", ctypes.c_int64),
        ("nodes_visited", ctypes.c_int64),
        ("photons_in_radius", ctypes.c_int64),
        ("ms_eye", ctypes.c_double),
        ("ms_trace", ctypes.c_double),
        ("ms_build", ctypes.c_double),
        ("ms_gather", ctypes.c_double),
        ("ms_final", ctypes.c_double),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


def fptr(a):
    """float32 ndarray -> POINTER(c_float) (None passes NULL)."""
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def iptr(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def f32(a, n=None):
    if a is None:
        return None
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} floats, got {a.size}")
    return a


def record_pixels(n_records, width, height):
    """Pixel index of each record in the 8x8-tile order used by the pinhole
    camera (-1 for padding records). Mirrors rec_to_pixel in pm_device.h."""
    r = np.arange(n_records, dtype=np.int64)
    tile, lane = r >> 6, r & 63
    tiles_x = (width + 7) // 8
    px = (tile % tiles_x) * 8 + (lane & 7)
    py = (tile // tiles_x) * 8 + (lane >> 3)
    pix = py * width + px
    pix[(px >= width) | (py >= height)] = -1
    return pix
