"""Helpers shared by the parity tests (GPU vs CPU oracle)."""
import numpy as np


def u32(a):
    """Bit pattern view of a structured/float array for bit-exact checks."""
    a = np.ascontiguousarray(a)
    return a.view(np.uint32).reshape(len(a), -1) if a.dtype.names else a.view(np.uint32)


def assert_bitexact(a, b, what):
    ua, ub = u32(a), u32(b)
    assert ua.shape == ub.shape, f"{what}: shape {ua.shape} vs {ub.shape}"
    bad = np.nonzero((ua != ub).reshape(len(ua), -1).any(axis=1))[0]
    assert bad.size == 0, f"{what}: {bad.size} of {len(ua)} entries differ, first at {bad[:8].tolist()}:\n" \
                          f"gpu={a[bad[0]]}\noracle={b[bad[0]]}"


def rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


def compare_gathered_records(gpu, ref, flux_rtol=2e-5):
    """Integer/PPM outputs exact; flux within fp32 summation-order tolerance."""
    assert np.array_equal(gpu["flags"], ref["flags"])
    assert np.array_equal(gpu["photon_count"], ref["photon_count"]), "per-record photon count N' differs"
    assert np.array_equal(u32(gpu["radius2"]), u32(ref["radius2"])), "radius2 differs"
    scale = np.maximum(np.abs(ref["flux"]), 1e-30)
    rel = np.abs(gpu["flux"] - ref["flux"]) / scale
    assert rel.max() <= flux_rtol, f"flux rel err {rel.max():.3g}"
