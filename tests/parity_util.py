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


def knn_reference(recs, photons, K, maxd2):
    """Brute-force statement of pbrt-v2's kNN photon lookup + LPhoton diffuse
    sum (integrators/photonmap.cpp; see oracle knn_estimate) for records whose
    material is matte: per record (photons found, r_k^2, S) with S the sum
    over found photons with Dot(Faceforward(ns, wo), wi) > 0 of
    3/pi (1 - d^2/r_k^2)^2 / r_k^2 * alpha (float64 accumulate). d^2 in
    float32 with the kernels' operation order."""
    from pmrender.abi import PM_REC_BACKFACE
    n = len(recs)
    found = np.zeros(n, np.int64)
    r2 = np.full(n, np.float32(maxd2), np.float32)
    S = np.zeros((n, 3), np.float64)
    for i in range(n):
        diff = recs["pos"][i][None, :] - photons["p"]
        d2 = (diff[:, 0] * diff[:, 0] + diff[:, 1] * diff[:, 1]) + diff[:, 2] * diff[:, 2]
        idx = np.nonzero(d2 < np.float32(maxd2))[0]
        idx = idx[np.argsort(d2[idx], kind="stable")][:K]
        found[i] = len(idx)
        if len(idx) == K:
            r2[i] = d2[idx[-1]]
        ns = recs["ns"][i].astype(np.float64)
        if recs["flags"][i] & PM_REC_BACKFACE:
            ns = -ns
        md2 = np.float64(r2[i])
        for j in idx:
            if float(photons["wi"][j].astype(np.float64) @ ns) > 0:
                if md2 == 0.0:   # K photons at distance 0: pbrt's kernel() is 0/0
                    S[i] = np.nan
                    continue
                s = 1.0 - float(d2[j]) / md2
                S[i] += 3.0 / np.pi * s * s / md2 * photons["alpha"][j].astype(np.float64)
    return found, r2, S


def knn_fixed_unit(scene, r2, max_photon_count=4):
    """The kNN gathers' fixed-point unit per record (1 / sc): sc = the power of
    two below knn_fx * r_k^2 (pm_gather.hip knn_scale), knn_fx = 2^24 / amax,
    amax = 4 emit_max kd_max^mpc (pm_api.cpp gather setup; emit_max over the
    lights: Le * area * 2 pi for a disk, I * 4 pi for a point; kd_max >= 1
    over the matte materials). Every term is rounded to this unit."""
    from pmrender.abi import PM_MATTE
    em = 0.0
    for L in scene.lights:
        if L[0] == "point":
            em = max(em, float(np.abs(np.float32(L[2])).max()) * 4.0 * np.pi)
        else:
            em = max(em, float(np.abs(np.float32(L[5])).max()) * float(np.float32(L[6])) * 2.0 * np.pi)
    kd = 1.0
    for mtype, rgb in scene.materials:
        if mtype == PM_MATTE:
            kd = max(kd, float(np.max(rgb)))
    amax = max(em, 1e-30) * kd ** max_photon_count * 4.0
    fx = np.float32(2.0 ** 24 / amax)
    prod = (fx * np.asarray(r2, np.float32)).astype(np.float32)
    sc = (prod.view(np.uint32) & np.uint32(0xff800000)).view(np.float32).astype(np.float64)
    sc[np.asarray(r2) == 0] = 1.0
    return 1.0 / sc


def knn_term_floor(scene, found, r2, max_photon_count=4):
    """Per-record absolute flux floor of one pass: one fixed-point unit per
    photon found (each term is rounded to the unit, <= 1/2 unit off)."""
    return np.asarray(found, np.float64) * knn_fixed_unit(scene, r2, max_photon_count)


def compare_knn_records(got, found, r2, flux, flux_rtol=1e-4, floor=None):
    """kNN records: photons found and r_k^2 exact; flux per record within
    flux_rtol of that record's own flux plus `floor` (per record, absolute:
    knn_term_floor summed over the passes — the fixed point's rounding), so a
    dim record is held to its own scale, not to the brightest record's."""
    assert np.array_equal(got["photon_count"].astype(np.int64), found), "kNN photons found differ"
    assert np.array_equal(u32(got["radius2"]), u32(np.asarray(r2, np.float32))), "kNN r_k^2 differs"
    flux = np.asarray(flux, np.float64)
    g = np.asarray(got["flux"], np.float64)
    if flux.ndim == 1:
        flux = np.broadcast_to(flux[:, None], g.shape) if g.ndim == 2 else flux
    assert np.array_equal(np.isnan(g), np.isnan(flux)), "kNN NaN records differ"
    fl = np.zeros(len(g)) if floor is None else np.asarray(floor, np.float64)
    fl = fl.reshape((len(g),) + (1,) * (g.ndim - 1))
    tol = flux_rtol * np.abs(flux) + fl
    bad = (np.abs(g - flux) > tol) & ~np.isnan(flux)
    rows = bad.reshape(len(g), -1).any(axis=1)
    if rows.any():
        i = int(np.nonzero(rows)[0][0])
        raise AssertionError(f"kNN flux: {int(rows.sum())} of {len(g)} records outside {flux_rtol:g} relative "
                             f"+ floor; first {i}: gpu {g[i]} vs {flux[i]} (found {found[i]}, floor {fl[i]})")
