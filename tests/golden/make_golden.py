#!/usr/bin/env python3
"""Generates tests/golden/golden_v2.npz — regression fixtures for the photon
mapper, produced by the CPU oracle (oracle/pm_oracle.cpp).

The reference ships no tests, fixtures or golden vectors and cannot be built
or run here, so these vectors are NOT reference outputs: they
freeze the oracle's restatement (parity unpinned) so that any
drift of the oracle or of the HIP path shows up as a byte difference.
tests/test_golden.py checks the oracle (CPU) and the HIP path (GPU) against
them. Arrays are raw bytes of the C-ABI structs (pm_record 64 B, pm_photon
40 B) or plain numeric arrays; no pickled objects.

    python tests/golden/make_golden.py        # rewrites golden_v2.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "cuda-raytrace_amd"), os.path.join(ROOT, "oracle")]

OUT = os.path.join(HERE, "golden_v2.npz")

CASES = {
    # name: (scene builder args, paths per pass, passes, initial r^2)
    "cornell": dict(scene="cornell", W=32, H=24, paths=1024, passes=2, r2=900.0),
    "feature": dict(scene="feature", W=72, H=40, paths=1024, passes=1, r2=900.0),
    "caustic": dict(scene="caustic", W=32, H=24, paths=1024, passes=1, r2=900.0),
}


def build_scene(case):
    from pmrender import scenes
    if case["scene"] == "cornell":
        return scenes.cornell_box(case["W"], case["H"])
    if case["scene"] == "feature":
        return scenes.feature_scene(case["W"], case["H"])
    return scenes.caustic_scene(case["W"], case["H"])


def params_for(case):
    from pmrender.abi import PM_GATHER_KDTREE, RenderParams
    return RenderParams.defaults(paths_per_pass=case["paths"], passes=case["passes"],
                                 initial_radius2=case["r2"], gather_structure=PM_GATHER_KDTREE)


def run_case(api_factory, case):
    """Stage-by-stage run on an oracle-like API; returns {key: bytes array}."""
    import oracle
    sc = build_scene(case)
    orc = sc.load_into(api_factory())
    p = params_for(case)
    out = {}
    recs = orc.eye_pass(p)
    out["eye_records"] = recs.view(np.uint8).copy()
    for pass_index in range(case["passes"]):
        slots = orc.trace_photons(p, pass_index, 0, case["paths"])
        nodes = oracle.Oracle.build_kdtree(slots)
        orc.gather(nodes, recs, p)
        out[f"slots_p{pass_index}"] = slots.view(np.uint8).copy()
        out[f"kdnodes_p{pass_index}"] = nodes.view(np.uint8).copy()
        out[f"records_p{pass_index}"] = recs.view(np.uint8).copy()
    img = orc.final(recs, float(case["paths"] * case["passes"]))
    out["image"] = np.ascontiguousarray(img, np.float32)
    return out


def generate():
    import oracle
    oracle.load()
    data = {}
    for name, case in CASES.items():
        for k, v in run_case(lambda: oracle.Oracle(nthreads=4), case).items():
            data[f"{name}/{k}"] = v
    # primitive vectors
    ctrs = [(0, 0, 0, 0), (1, 0, 0, 0), (4 * 262143 + 3, 7, 0, 0), (0xffffffff, 0xffffffff, 0, 0)]
    data["philox/ctr"] = np.asarray(ctrs, np.uint32)
    data["philox/out"] = np.asarray([oracle.philox(c, (777, 0)) for c in ctrs], np.uint32)
    data["halton/perm"] = np.stack([oracle.halton_permutation(s) for s in range(4)])
    ns = np.asarray([0, 1, 2, 3, 7, 8, 100, 4095, 65536, 1048572, 12582911, 16777212], np.uint32)
    data["halton/n"] = ns
    data["halton/sample_p0"] = np.stack([oracle.halton_sample(int(n), data["halton/perm"][0]) for n in ns])
    data["meta"] = np.frombuffer(json.dumps(CASES, sort_keys=True).encode(), np.uint8)
    return data


def main():
    data = generate()
    np.savez_compressed(OUT, **data)
    print(f"wrote {OUT}: {len(data)} arrays, {os.path.getsize(OUT)} bytes")


if __name__ == "__main__":
    main()
