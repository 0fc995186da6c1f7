"""Committed golden fixtures (tests/golden/golden_v2.npz, made by
tests/golden/make_golden.py from the CPU oracle). The reference has no
golden vectors of its own, so these freeze the oracle's
restatement: the oracle must reproduce them on the CPU, and the HIP path must
reproduce them byte for byte through the C-ABI on the GPU."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden  # noqa: E402

GOLDEN = np.load(os.path.join(HERE, "golden", "golden_v2.npz"), allow_pickle=False)


def test_fixture_metadata_matches_generator():
    assert json.loads(GOLDEN["meta"].tobytes()) == json.loads(json.dumps(make_golden.CASES, sort_keys=True))


def test_fixtures_are_informative():
    from pmrender.abi import PHOTON_DTYPE, RECORD_DTYPE
    for name, case in make_golden.CASES.items():
        slots = GOLDEN[f"{name}/slots_p0"].view(PHOTON_DTYPE)
        assert (slots["bits"] & 1).sum() > 0.2 * len(slots), name
        recs = GOLDEN[f"{name}/records_p{case['passes'] - 1}"].view(RECORD_DTYPE)
        assert (recs["photon_count"] > 0).sum() > 0.2 * len(recs), name
        assert np.isfinite(GOLDEN[f"{name}/image"]).all()


@pytest.mark.parametrize("name", list(make_golden.CASES))
def test_oracle_reproduces_golden(name, oracle_mod):
    got = make_golden.run_case(lambda: oracle_mod.Oracle(nthreads=4), make_golden.CASES[name])
    for k, v in got.items():
        ref = GOLDEN[f"{name}/{k}"]
        assert v.shape == ref.shape, k
        assert np.array_equal(v.view(np.uint8), ref.view(np.uint8)), f"{name}/{k} drifted"


def test_oracle_primitives_reproduce_golden(oracle_mod):
    for c, o in zip(GOLDEN["philox/ctr"], GOLDEN["philox/out"]):
        assert oracle_mod.philox(tuple(int(x) for x in c), (777, 0)) == [int(x) for x in o]
    for s in range(4):
        assert np.array_equal(oracle_mod.halton_permutation(s), GOLDEN["halton/perm"][s])
    for n, ref in zip(GOLDEN["halton/n"], GOLDEN["halton/sample_p0"]):
        got = oracle_mod.halton_sample(int(n), GOLDEN["halton/perm"][0])
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), n


def test_host_halton_permutation_matches_golden(hip_mod):
    """libpmhip's host-side permutation (no device needed) == fixture."""
    for s in range(4):
        assert np.array_equal(hip_mod.halton_permutation(s), GOLDEN["halton/perm"][s])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(make_golden.CASES))
def test_hip_reproduces_golden(name, hip_mod):
    """HIP kernels through the C-ABI, stage by stage, == the fixture bytes:
    eye records, photon slots, reference-layout kd-tree, gathered records and
    the final image (kd-tree gather is bit-exact by construction)."""
    from pmrender.abi import PHOTON_DTYPE, RECORD_DTYPE
    case = make_golden.CASES[name]
    sc = make_golden.build_scene(case)
    ctx = sc.load_into(hip_mod.Context(0))
    p = make_golden.params_for(case)
    try:
        ctx.eye_pass(p)
        recs = ctx.download_records()
        assert np.array_equal(recs.view(np.uint8), GOLDEN[f"{name}/eye_records"]), "eye records"
        for pass_index in range(case["passes"]):
            ctx.trace_photons(p, pass_index, 0, case["paths"])
            slots = ctx.download_slots(case["paths"] * p.max_photon_count)
            assert np.array_equal(slots.view(np.uint8), GOLDEN[f"{name}/slots_p{pass_index}"]), f"slots p{pass_index}"
            ctx.build_photon_map(p, case["paths"] * p.max_photon_count)
            nodes = ctx.download_kdtree()
            assert np.array_equal(nodes.view(np.uint8), GOLDEN[f"{name}/kdnodes_p{pass_index}"]), f"kd p{pass_index}"
            ctx.gather(p)
            recs = ctx.download_records()
            assert np.array_equal(recs.view(np.uint8), GOLDEN[f"{name}/records_p{pass_index}"]), f"records p{pass_index}"
        img = ctx.final_image(float(case["paths"] * case["passes"]))
        assert np.array_equal(img.view(np.uint32), GOLDEN[f"{name}/image"].view(np.uint32)), "image"
    finally:
        ctx.close()
    del PHOTON_DTYPE, RECORD_DTYPE
