"""BASELINE.json configurations and index ranges beyond the small parity
cases, HIP path vs the CPU oracle (oracle/pm_oracle.cpp, parity unpinned —
see DESIGN.md §4):

* Halton index ranges of C4/C5 (photontracing.cu:19-31): path ranges whose
  pm_index = 4 * path crosses 2^20, 12,582,912 (where the reference's
  `n *= invBase` quirk stops equalling n / base) and 2^24 (where base 2
  leaves its closed form), traced with global path ids exactly as a rank of
  a multi-GPU run traces them — slots bit-exact;
* point-light photon emission (cudalight.cu.h:78-88) as light 0;
* C1 (256x256, 25,000 paths), C2 per-record PPM state at full size, C3 (1M
  triangles, 1,048,576 paths, 1080p) and C5 (caustic scene, 4 progressive
  passes of 1,048,576 paths at 1080p) at full size: slots / photon counts /
  N' / r^2 exact, flux within fp32 summation order, radiance RMSE < 1e-3,
  plus determinism and conservation properties of the full workloads."""
import numpy as np
import pytest

from parity_util import assert_bitexact, compare_gathered_records, rmse
from pmrender import scenes
from pmrender.abi import PM_GATHER_GRID, PM_GATHER_KDTREE, RenderParams

pytestmark = pytest.mark.gpu


def make_pair(scene, oracle_mod, hip_mod, threads=None):
    return scene.load_into(hip_mod.Context(0)), scene.load_into(oracle_mod.Oracle(nthreads=threads))


@pytest.fixture(scope="module")
def cornell_small(oracle_mod, hip_mod):
    ctx, orc = make_pair(scenes.cornell_box(32, 32), oracle_mod, hip_mod)
    yield ctx, orc
    ctx.close()


@pytest.mark.parametrize("path_begin", [262_100, 3_145_700, 4_194_270, 8_388_000])
@pytest.mark.parametrize("pass_index", [0, 3])
def test_halton_index_ranges(cornell_small, path_begin, pass_index):
    """pm_index = 4 * path across 2^20 (262,144), 12,582,912 (3,145,728),
    2^24 (4,194,304) and C5's last paths (8,388,607): GPU slots of the range
    == oracle slots of the same global paths."""
    ctx, orc = cornell_small
    n = 4096
    p = RenderParams.defaults(paths_per_pass=n)
    ctx.trace_photons(p, pass_index, path_begin, n, slot_path_base=path_begin)
    got = ctx.download_slots(n * 4)
    ref = orc.trace_photons(p, pass_index, path_begin, n)
    assert (ref["bits"] & 1).sum() > n // 2
    assert_bitexact(got, ref, f"slots of paths [{path_begin}, {path_begin + n}) pass {pass_index}")


def point_light_scene(W, H):
    """The Cornell box lit by a point light (light 0) instead of the disk."""
    s = scenes.cornell_box(W, H)
    s.lights = [("point", np.float32([278.0, 500.0, 279.5]), np.float32([150000.0, 150000.0, 150000.0]))]
    s.disks = []
    return s


@pytest.mark.parametrize("structure", [PM_GATHER_KDTREE, PM_GATHER_GRID])
def test_point_light_emission(structure, oracle_mod, hip_mod):
    sc = point_light_scene(64, 48)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        p = RenderParams.defaults(paths_per_pass=16384, gather_structure=structure, initial_radius2=25.0)
        img, st = ctx.render(p)
        slots = ctx.download_slots(16384 * 4)
        ref_slots = orc.trace_photons(p, 0, 0, 16384)
        assert (ref_slots["bits"] & 1).sum() > 10000
        assert_bitexact(slots, ref_slots, "point-light slots")
        ref, st_ref = orc.render(p)
        assert st["photons_valid"] == st_ref["photons_valid"]
        assert rmse(img, ref) < 1e-3
        if structure == PM_GATHER_KDTREE:
            assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    finally:
        ctx.close()


def stage_records(ctx, orc, p, passes=1):
    """Per-record PPM state after `passes` passes: GPU stage API (grid) vs the
    oracle's pbrt kd-tree passes."""
    ctx.eye_pass(p)
    recs = orc.eye_pass(p)
    for k in range(passes):
        ctx.trace_photons(p, k, 0, p.paths_per_pass)
        ctx.build_photon_map(p, p.paths_per_pass * 4)
        ctx.gather(p)
        slots = orc.trace_photons(p, k, 0, p.paths_per_pass)
        orc.gather(orc.build_kdtree(slots), recs, p)
    return ctx.download_records(), recs


def test_c1_full(oracle_mod, hip_mod):
    """C1: Cornell 256x256, 100,000 slots (25,000 paths)."""
    sc = scenes.cornell_box(256, 256)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        p = RenderParams.defaults(paths_per_pass=25_000)
        got, ref = stage_records(ctx, orc, p)
        compare_gathered_records(got, ref)
        img, st = ctx.render(p)
        ref_img, st_ref = orc.render(p)
        assert st["photons_valid"] == st_ref["photons_valid"] > 50_000
        assert rmse(img, ref_img) < 1e-3
        pk = RenderParams.defaults(paths_per_pass=25_000, gather_structure=PM_GATHER_KDTREE)
        img_kd, _ = ctx.render(pk)
        ref_kd, _ = orc.render(pk)
        assert np.array_equal(img_kd.view(np.uint32), ref_kd.view(np.uint32))
    finally:
        ctx.close()


def test_c2_full_records(oracle_mod, hip_mod):
    """C2 at full size: per-record M -> N', r^2 exact, flux <= 2e-5 relative."""
    sc = scenes.cornell_box(1920, 1080)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        p = RenderParams.defaults()
        got, ref = stage_records(ctx, orc, p)
        active = (ref["photon_count"] > 0).sum()
        assert active > 500_000
        compare_gathered_records(got, ref)
    finally:
        ctx.close()


def test_c2_bench_step_twice(oracle_mod, hip_mod):
    """C2 at full size, bench.py's step run twice in one context: reset ->
    trace -> build -> gather. The first full-range gather of a context runs
    the cost-recording tile instance over the unsorted tile list; the second
    is the timed instance (k_gather_tile over the cost-sorted list, counts
    fused into the trace) — compared here with the oracle: M -> N', r^2
    exact, flux <= 2e-5 (gathering.cu:104-126); and equal to the first
    gather bit for bit (exact fixed-point sums)."""
    sc = scenes.cornell_box(1920, 1080)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        p = RenderParams.defaults()
        n = p.paths_per_pass
        ctx.eye_pass(p)
        recs = orc.eye_pass(p)
        first = None
        for step in range(2):
            ctx.reset_records(p)
            ctx.trace_photons(p, 0, 0, n)
            ctx.build_photon_map(p, n * 4)
            ctx.gather(p)
            if step == 0:
                first = ctx.download_records()
        got = ctx.download_records()
    finally:
        ctx.close()
    slots = orc.trace_photons(p, 0, 0, n)
    orc.gather(orc.build_kdtree(slots), recs, p)
    assert (recs["photon_count"] > 0).sum() > 500_000
    compare_gathered_records(got, recs)
    assert_bitexact(got, first, "C2 second (sorted-list) gather vs the first (unsorted, cost-recording)")


def shard_records(ctx, orc, p, path_begin):
    """One rank's photon shard at its global path ids (slots of paths
    [path_begin, path_begin + paths_per_pass)), gathered over all records:
    GPU stage API (grid) vs the oracle's pbrt kd-tree pass over the same
    global paths."""
    n = p.paths_per_pass
    ctx.eye_pass(p)
    recs = orc.eye_pass(p)
    ctx.trace_photons(p, 0, path_begin, n, slot_path_base=path_begin)
    ctx.build_photon_map(p, n * 4)
    ctx.gather(p)
    slots = orc.trace_photons(p, 0, path_begin, n)
    orc.gather(orc.build_kdtree(slots), recs, p)
    return ctx.download_records(), recs, ctx.download_slots(n * 4), slots


@pytest.mark.parametrize("rank", [0, 7])
def test_c4_share(rank, oracle_mod, hip_mod):
    """C4 per-GPU share at full size (the bench's --config c4 line): Cornell
    3840x2160 (8,294,400 gather points), 524,288 paths = 2,097,152 slots of
    rank `rank` of 8 (global paths [rank * 524,288, ...): rank 7's pm_index
    runs to 16,777,212, past the 12,582,912 limit of the Halton quirk).
    Slots bit-exact; per-record M -> N', r^2 exact and flux <= 2e-5 relative
    vs the oracle (photontracing.cu:80-103, gathering.cu:104-126)."""
    sc = scenes.cornell_box(3840, 2160)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        paths = 524_288
        p = RenderParams.defaults(paths_per_pass=paths)
        got, ref, slots, ref_slots = shard_records(ctx, orc, p, rank * paths)
        assert_bitexact(slots, ref_slots, f"C4 rank {rank} slots")
        assert len(got) == 3840 * 2160
        assert (ref["photon_count"] > 0).sum() > 2_000_000
        compare_gathered_records(got, ref)
    finally:
        ctx.close()


def test_c4_allgather_map(oracle_mod, hip_mod):
    """C4 in north_star's all-gather form: after the RCCL
    all-gather of the 8 ranks' slots every GPU holds all 4,194,304 paths'
    16,777,216 slots, builds ONE photon map over them and gathers its own
    interleaved 8-row bands of the 3840x2160 records (pmrender.dist._bands).
    Here one context holds what every rank holds after the exchange (the 8
    shards traced at their global path ids are the one 4,194,304-path trace,
    slot for slot) and gathers the bands of ranks 0 and 7:
      * slots bit-exact vs the oracle, map photons == valid slots;
      * the bands' records vs the oracle's kd-tree gather over the same
        slots (gathering.cu:104-126): M -> N', r^2 exact, flux <= 2e-5;
        records outside the two ranks' bands untouched;
      * the same bands after the reduce exchange's form — the 8 shards'
        2,097,152-slot maps gathered one by one into per-record partial sums
        (int32 M, int64 fixed-point flux), summed, then one split update —
        are the full map's records bit for bit (exact fixed-point sums)."""
    _allgather_map(scenes.cornell_box(3840, 2160), 3840, 2160, 524_288, 8_000_000, 500_000,
                   oracle_mod, hip_mod)


def test_c5_allgather_map(oracle_mod, hip_mod):
    """C5's photon budget in its 8-GPU all-gather form: the caustic scene at
    1080p, 8 ranks x 1,048,576 paths = 8,388,608 paths = 33,554,432 slots
    all-gathered into one map (twice C4's), the bands of ranks 0 and 7
    gathered against it vs the oracle's kd-tree gather (M -> N', r^2 exact,
    flux <= 2e-5), slots bit-exact, and the 8 reduce-mode shares summed equal
    to the full map bit for bit — as test_c4_allgather_map."""
    _allgather_map(scenes.caustic_scene(1920, 1080), 1920, 1080, 1_048_576, 5_000_000, 100_000,
                   oracle_mod, hip_mod)


def _allgather_map(sc, W, H, per, min_valid, min_lit, oracle_mod, hip_mod):
    """one context holds what every rank of 8 holds after the slot all-gather
    (the 8 shards traced at their global path ids are one trace of all the
    paths, slot for slot) and gathers the bands of ranks 0 and 7"""
    import torch
    from pmrender.dist import _bands
    world = 8
    total = world * per
    p = RenderParams.defaults(paths_per_pass=total)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        ctx.eye_pass(p)
        ctx.trace_photons(p, 0, 0, total)
        ctx.build_photon_map(p, total * 4)
        n = ctx.num_records()
        bands = _bands(n, ((W + 7) // 8) * 64, world)
        mine = [bands[0], bands[world - 1]]
        for runs in mine:
            for b, c in runs:
                ctx.gather_range(p, b, c)
        info = ctx.map_info()
        got = ctx.download_records()
        slots = ctx.download_slots(total * 4)
    finally:
        ctx.close()
    ref_slots = orc.trace_photons(p, 0, 0, total)
    assert_bitexact(slots, ref_slots, f"all-gathered slots ({total * 4:,})")
    del slots
    nvalid = int((ref_slots["bits"] & 1).sum())
    assert info["valid"] == nvalid > min_valid, (info, nvalid)
    recs = orc.eye_pass(p)
    idx = np.concatenate([np.arange(b, b + c) for runs in mine for b, c in runs])
    assert len(idx) > 0.9 * 2 * W * H / world  # two ranks' bands, less the bands short of a whole run
    sub = recs[idx].copy()
    orc.gather(orc.build_kdtree(ref_slots), sub, p)
    del ref_slots
    assert (sub["photon_count"] > 0).sum() > min_lit
    compare_gathered_records(got[idx], sub)
    rest = np.ones(n, bool)
    rest[idx] = False
    assert_bitexact(got[rest], recs[rest], "records outside ranks 0 and 7's bands")
    del recs, sub

    # the reduce exchange's form over the same paths: 8 shard maps, summed partials
    ps = RenderParams.defaults(paths_per_pass=per)
    ctx = sc.load_into(hip_mod.Context(0))
    try:
        ctx.eye_pass(ps)
        nv = ctx.set_record_view(True)
        dev = torch.device("cuda", 0)
        cnt = torch.zeros(nv, dtype=torch.int32, device=dev)
        flux = torch.zeros((nv, 3), dtype=torch.int64, device=dev)
        cnt_sum, flux_sum = torch.zeros_like(cnt), torch.zeros_like(flux)
        for r in range(world):
            ctx.trace_photons(ps, 0, r * per, per, slot_path_base=r * per)
            ctx.build_photon_map(ps, per * 4)
            torch.cuda.synchronize()
            ctx.gather_split(ps, cnt.data_ptr(), flux.data_ptr())
            ctx.synchronize()
            cnt_sum += cnt
            flux_sum += flux
        torch.cuda.synchronize()
        ctx.ppm_update_split(ps, cnt_sum.data_ptr(), flux_sum.data_ptr(), 0, nv)
        ctx.synchronize()
        red = ctx.download_records()
    finally:
        ctx.close()
    assert_bitexact(red[idx], got[idx], "bands: sum of the 8 reduce-mode shares vs the all-gathered map")


def test_c3_full_workload(oracle_mod, hip_mod):
    """C3: Cornell enclosure + 1M-triangle soup, 1,048,576 paths, 1080p.
    Oracle: eye records and every photon slot bit-exact, per-record PPM
    state after the gather; properties: two runs bit-identical, valid slots
    == photons in the map == cell_start[ncells]."""
    sc = scenes.triangle_soup(1_000_000, 1920, 1080)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        assert ctx.scene_info()["mode"] == "bvh-hbm"
        paths = 1_048_576
        p = RenderParams.defaults(paths_per_pass=paths)
        got, ref = stage_records(ctx, orc, p)
        compare_gathered_records(got, ref)
        slots = ctx.download_slots(paths * 4)
        ref_slots = orc.trace_photons(p, 0, 0, paths)
        assert_bitexact(slots, ref_slots, "C3 slots")
        nvalid = int((slots["bits"] & 1).sum())
        assert nvalid > 3_000_000
        assert ctx.map_info()["valid"] == nvalid
        img1, st1 = ctx.render(p)
        img2, st2 = ctx.render(p)
        assert st1["photons_valid"] == st2["photons_valid"] == nvalid
        assert np.array_equal(img1.view(np.uint32), img2.view(np.uint32)), "C3 render not deterministic"
    finally:
        ctx.close()


def test_c5_progressive(oracle_mod, hip_mod):
    """C5 substitute at its full photon budget: caustic scene (glass + mirror
    spheres), 1080p, 8 progressive passes of 1,048,576 paths = 8,388,608
    paths = 33,554,432 slots (shrinking radii, PPM state
    carried, later passes on the cost-sorted tile list and the radius
    histogram's grid): per-record N', r^2 exact after the passes, flux within
    tolerance, image RMSE < 1e-3."""
    sc = scenes.caustic_scene(1920, 1080)
    ctx, orc = make_pair(sc, oracle_mod, hip_mod)
    try:
        paths, passes = 1_048_576, 8
        p = RenderParams.defaults(paths_per_pass=paths)
        got, ref = stage_records(ctx, orc, p, passes=passes)
        compare_gathered_records(got, ref, flux_rtol=5e-5)
        assert (ref["photon_count"] > 0).sum() > 500_000
        pp = RenderParams.defaults(paths_per_pass=paths, passes=passes)
        img, st = ctx.render(pp)
        ref_img = orc.final(ref, float(paths * passes))
        assert rmse(img, ref_img) < 1e-3
    finally:
        ctx.close()


def test_c2_full_knn(oracle_mod, hip_mod, monkeypatch):
    """The kNN estimator at C2 size (1080p, 262,144 paths, K = 50, r^2 = 100,
    the bench's kNN line): the tile kernel equals the per-lane heap kernel
    bit for bit, and both match the oracle's pbrt kd-tree lookup (found
    count and r_k^2 exact, flux to fp32 summation order)."""
    from parity_util import compare_knn_records, knn_term_floor
    from pmrender.abi import PM_ESTIMATOR_KNN
    sc = scenes.cornell_box(1920, 1080)
    orc = sc.load_into(oracle_mod.Oracle())
    p = RenderParams.defaults(paths_per_pass=262_144, initial_radius2=100.0, estimator=PM_ESTIMATOR_KNN,
                              knn_lookup=50)
    recs = orc.eye_pass(p)
    slots = orc.trace_photons(p, 0, 0, 262_144)
    outs = {}
    for name in ("lane", "tile", "ss"):
        monkeypatch.setenv("PM_GATHER_KERNEL", "lane" if name == "lane" else "tile")
        monkeypatch.setenv("PM_KNN_SS", "1" if name == "ss" else "0")
        ctx = sc.load_into(hip_mod.Context(0))
        try:
            ctx.upload_records(recs)
            ctx.upload_slots(slots)
            ctx.build_photon_map(p, len(slots))
            ctx.gather(p)
            outs[name] = ctx.download_records()
        finally:
            ctx.close()
    assert_bitexact(outs["tile"], outs["lane"], "C2 kNN tile vs per-lane")
    assert_bitexact(outs["ss"], outs["lane"], "C2 kNN scalar-stream vs per-lane")
    ref = recs.copy()
    orc.gather(orc.build_kdtree(slots), ref, p)
    act = (ref["flags"] & 7) == 0
    assert act.sum() > 1_000_000 and (ref["photon_count"][act] == 50).mean() > 0.2
    compare_knn_records(outs["tile"], ref["photon_count"].astype(np.int64), ref["radius2"], ref["flux"],
                        floor=knn_term_floor(sc, ref["photon_count"], ref["radius2"]))
