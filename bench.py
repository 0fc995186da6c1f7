#!/usr/bin/env python3
"""bench.py — BASELINE.json metric on MI355X: "Mphotons/s traced +
Mgather-samples/s, Cornell box 1M photons @1080p" (configs[1] = C2).

A step is one photon-mapping pass over the C2 workload from the initial PPM
state (the reference's default single pass), inputs (scene, BVH, eye-pass
records) already resident in HBM:
    reset PPM state (deferred: the gather starts from the initial state) ->
    emit + trace 262,144 paths (1,048,576 photon slots) per GPU, counting the
    bucket cells of the deposits -> scan + fill the photon buckets -> range
    query + PPM update over the 2,073,600 gather points (+ the reduce-scatter
    of (M, L) and all-gather of radii for N > 1).
`value` = emitted photon paths over all ranks / step time (whole job,
Mphotons/s); `mgather_samples_per_s` = gather points / step time.

Single GPU: `python bench.py`. N GPUs (one process per GPU):
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N`.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))

METRIC = "Mphotons/s traced + Mgather-samples/s, Cornell box 1M photons @1080p"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c2", "c3"])
    ap.add_argument("--structure", default="grid", choices=["grid", "kd"])
    ap.add_argument("--exchange", default="reduce", choices=["reduce", "allgather"])
    ap.add_argument("--paths", type=int, default=512 * 512, help="photon paths per GPU per pass")
    ap.add_argument("--estimator", default="ppm", choices=["ppm", "knn"],
                    help="ppm: the reference's fixed-radius PPM gather (headline); knn: pbrt-v2 LPhoton kNN")
    ap.add_argument("--knn-k", type=int, default=50, help="kNN photons per lookup (pbrt 'nused')")
    ap.add_argument("--radius2", type=float, default=None,
                    help="initial / maximum search radius^2 (default: 4 for ppm = raytracing.cu:123, 100 for knn)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-census", action="store_true")
    return ap.parse_args()


def build_scene(cfg):
    from pmrender import scenes
    if cfg == "c2":
        return scenes.cornell_box(1920, 1080), "C2: Cornell box, 1,048,576 photon slots (262,144 paths) per GPU, 1920x1080 gather points"
    return scenes.triangle_soup(1_000_000, 1920, 1080), "C3: Cornell enclosure + 1M-triangle soup, 1920x1080 gather points"


def load_pmc_traffic(kernel_prefix):
    """Per-launch HBM bytes of the gather kernel from the committed PMC
    profile (tools/pmc_traffic.py writes it from a separate rocprofv3 --pmc
    pass); None if absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    k = d.get("kernels", {}).get(kernel_prefix)
    return (k.get("hbm_bytes_per_launch") if k else None), os.path.relpath(path, ROOT)


def cpu_baseline(scene, params, threads):
    """Oracle (CPU restatement of the reference, test infrastructure) timed on
    this host: one full pass of the same workload (trace 262,144 paths +
    pbrt kd-tree build + range query/PPM update over all gather points)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    orc = scene.load_into(oracle.Oracle(nthreads=threads))
    recs0 = orc.eye_pass(params)                     # setup (the GPU eye pass is outside the step too)
    # repeat whole passes (fresh PPM state each, like the GPU step) until the
    # sample holds >= 12 s of CPU work (wall x threads), at most 20 passes
    passes, dt, nodes = 0, 0.0, []
    while passes < 20 and (passes == 0 or dt * threads < 12.0):
        recs = recs0.copy()
        t0 = time.perf_counter()
        slots = orc.trace_photons(params, passes, 0, params.paths_per_pass)
        nodes = orc.build_kdtree(slots)
        orc.gather(nodes, recs, params)
        dt += time.perf_counter() - t0
        passes += 1
    return {
        "value": round(params.paths_per_pass * passes / dt / 1e6, 4),
        "unit": "Mphotons/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{passes} full C2 passes on the host (each: trace {params.paths_per_pass} paths + pbrt kd-tree "
                  f"build over ~{len(nodes)} photons + gather/PPM over {len(recs0)} records); {dt:.2f} s wall, "
                  f"{dt * threads:.1f} thread-s",
        "mgather_samples_per_s": round(len(recs0) * passes / dt / 1e6, 4),
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        if world == 1 and args.gpus > 1:
            sys.exit("bench.py --gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
        args.gpus = world

    import torch  # first: the renderer then shares torch's HIP runtime (one runtime per process)
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from pmrender import hip
    from pmrender.abi import PM_ESTIMATOR_KNN, PM_ESTIMATOR_PPM, PM_GATHER_GRID, PM_GATHER_KDTREE, \
        PM_REC_EXCEPTION, PM_REC_INVALID, PM_REC_MISS, RenderParams
    from pmrender.dist import HipEngine, PassRunner

    scene, workload = build_scene(args.config)
    t_setup = time.perf_counter()
    ctx = scene.load_into(hip.Context(local))
    structure = PM_GATHER_KDTREE if args.structure == "kd" else PM_GATHER_GRID
    knn = args.estimator == "knn"
    if knn and world > 1:
        args.exchange = "allgather"        # the kNN estimate is not a sum over photon shards
    radius2 = args.radius2 if args.radius2 is not None else (100.0 if knn else 4.0)
    est = dict(estimator=PM_ESTIMATOR_KNN if knn else PM_ESTIMATOR_PPM, knn_lookup=args.knn_k, initial_radius2=radius2)
    p = RenderParams.defaults(paths_per_pass=args.paths, gather_structure=structure, **est)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        eng = HipEngine(ctx)
        ctx.eye_pass(p, eng._s())
        runner = PassRunner(eng, p, rank, world, args.exchange)
        for _ in range(args.warmup):
            runner.step(0, reset=True)
        runner.flush()
        torch.cuda.synchronize()
        setup_s = time.perf_counter() - t_setup
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ctx.timing_reset()
        # events only on the roofline kernel's stage inside the timed region:
        # every timed stage boundary costs a few us of idle GPU
        ctx.set_stage_timing("gather")
        t0 = time.perf_counter()
        for _ in range(args.steps):
            runner.step(0, reset=True)
        runner.flush()                 # the last pass's exchange is part of the timed work
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
            t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        gather_launches, gather_ms_total = ctx.timing_total("gather")
        gather_ms = gather_ms_total / max(gather_launches, 1)
        # per-stage split: a few more passes after the timed region, every stage timed
        ctx.set_stage_timing("all")
        ctx.timing_reset()
        for _ in range(min(args.steps, 10)):
            runner.step(0, reset=True)
        runner.flush()
        torch.cuda.synchronize()
        stages = {}
        for name in ("reset", "trace", "build", "gather", "update"):
            n, ms = ctx.timing_total(name)
            if n:
                stages[name] = round(ms / n, 5)

        census = canonical = tcensus = None
        if not args.no_census:
            # untimed counting launch of the same step: algorithmic-byte units
            ctx.set_counting(True)
            runner.step(0, reset=True)
            runner.flush()
            torch.cuda.synchronize()
            census = ctx.gather_counters(full=True)
            tcensus = ctx.trace_counters()
            ctx.set_counting(False)
            if rank == 0 and world == 1 and structure == PM_GATHER_GRID and not knn:
                # SURVEY.md §8d's per-unit figure counts V on the canonical pbrt kd-tree
                pk = RenderParams.defaults(paths_per_pass=args.paths, gather_structure=PM_GATHER_KDTREE)
                ctx.set_counting(True)
                ctx.reset_records(pk, eng._s())
                ctx.trace_photons(pk, 0, 0, args.paths, 0, eng._s())
                ctx.build_photon_map(pk, args.paths * 4, eng._s())
                ctx.gather(pk, eng._s())
                torch.cuda.synchronize()
                canonical = ctx.gather_counters(full=True)
                ctx.set_counting(False)

    n_rec = ctx.num_records()
    recs = ctx.download_records()
    active = int(((recs["flags"] & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) == 0).sum())
    g_points = scene.width * scene.height
    paths_total = args.paths * world
    ms_per_step = elapsed / args.steps * 1e3
    value = paths_total * args.steps / elapsed / 1e6

    roofline = None
    if census is not None:
        vis, hits, rows, act = census
        inactive = n_rec - act
        if knn:
            # records as below; 8 B per bucket row; 16 B per photon tested; per
            # photon found: its slot id (4 B, ph_b) + alpha and wi from the slot (24 B)
            bytes_launch = 72 * act + 16 * inactive + 8 * rows + 16 * vis + 28 * hits
            formula = "72*G_act + 16*G_inactive + 8*bucket_rows + 16*photons_tested + 28*photons_found"
        elif structure == PM_GATHER_GRID:
            # records: pos 16 + nrm 16 + state 16 + N 4 read, state 16 + N 4 written (active);
            # pos 16 read (inactive); 8 B of bucket bounds per row; 16 B per photon tested;
            # 20 B (alpha + wi.y, wi.z) per photon inside the radius
            bytes_launch = 72 * act + 16 * inactive + 8 * rows + 16 * vis + 20 * hits
            formula = "72*G_act + 16*G_inactive + 8*bucket_rows + 16*photons_tested + 20*photons_in_radius"
        else:
            bytes_launch = 72 * act + 16 * inactive + 16 * vis + 24 * hits
            formula = "72*G_act + 16*G_inactive + 16*kd_nodes_visited + 24*photons_in_radius"
        achieved = bytes_launch / (gather_ms * 1e-3) / 1e9
        traffic, traffic_src = load_pmc_traffic(
            "k_gather_knn" if knn else "k_gather_grid" if structure == PM_GATHER_GRID else "k_gather_kd")
        roofline = {
            "bound": "hbm",
            "kernel": "k_gather_knn<0> (pbrt LPhoton kNN, fused record update)" if knn
            else "k_gather_grid<0,0> (fused range query + PPM update)" if structure == PM_GATHER_GRID
            else "k_gather_kd<0,0>",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": int(bytes_launch),
            "formula": formula,
            "units": {"G_act": act, "G_inactive": inactive, "bucket_rows": rows, "photons_tested": vis,
                      "photons_found" if knn else "photons_in_radius": hits},
            "avg_launch_ms": round(gather_ms, 5),
            "launches_timed": gather_launches,
        }
        if traffic_src:
            roofline["traffic_source"] = traffic_src
        if canonical is not None:
            cv, ch, _, cact = canonical
            survey_bytes = 92 * cact + 16 * cv + 24 * ch
            roofline["survey_8d_equivalent"] = {
                "formula": "92*G_act + 16*V_kd + 24*H (SURVEY.md §8d, V on the canonical pbrt kd-tree)",
                "bytes_per_launch": int(survey_bytes), "V_kd": cv, "H": ch,
                "GBs_at_measured_time": round(survey_bytes / (gather_ms * 1e-3) / 1e9, 1)}

    trace_roofline = None
    if tcensus is not None and "trace" in stages and ctx.scene_info()["mode"] == "brute":
        # brute-force scene (C2's Cornell box: 30 triangles + 1 disk, no BVH):
        # the triangles are read through the scalar cache, so the kernel's
        # algorithmic work is arithmetic — ~41 FP32 operations per primitive
        # test (OptiX test: dot 5, exact reciprocal 5, e2 6, cross 9, three
        # dots 15, beta+gamma 1) against the VALU FP32 peak
        rays, nodes, prims, deposits = tcensus
        tflop = 41.0 * prims / (stages["trace"] * 1e-3) / 1e12
        trace_roofline = {
            "bound": "valu", "kernel": "k_trace_lane<0,MODE_BRUTE>", "achieved": round(tflop, 2),
            "peak": VALU_FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(tflop / VALU_FP32_PEAK_TFLOPS, 4),
            "flops_per_launch": int(41 * prims), "formula": "41 * prim_tests",
            "units": {"rays": rays, "prim_tests": prims, "deposits": deposits},
            "avg_launch_ms": stages["trace"],
            "note": "bounded by its slowest waves (avg wave lifetime ~0.7 of the kernel), not by VALU throughput"}
    elif tcensus is not None and "trace" in stages:
        rays, nodes, prims, deposits = tcensus
        # SURVEY.md §8d (reported, not graded): 40 B per deposit + 32 B per BVH
        # node entered + 36 B per primitive test (RNG is inline Philox: 0 B)
        tbytes = 40 * deposits + 32 * nodes + 36 * prims
        tach = tbytes / (stages["trace"] * 1e-3) / 1e9
        trace_roofline = {
            "bound": "hbm", "kernel": "k_trace_lane<0,MODE_GLOBAL|MODE_LDS>", "achieved": round(tach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(tach / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": int(tbytes),
            "formula": "40*deposits + 32*bvh_nodes + 36*prim_tests (SURVEY.md §8d B_trace)",
            "units": {"rays": rays, "bvh_nodes": nodes, "prim_tests": prims, "deposits": deposits},
            "avg_launch_ms": stages["trace"],
            "note": "VALU-bound: the BVH and scene of C2 stay in L2/MALL, so B_trace is mostly cache traffic"}

    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mphotons/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: Cornell box built in code (pmrender/scenes.py), BASELINE.json configs[1]",
        "config": {
            "workload": workload,
            "photon_slots_per_gpu": args.paths * int(p.max_photon_count),
            "paths_per_gpu": args.paths,
            "gather_points": g_points,
            "active_gather_points": active,
            "structure": args.structure,
            "estimator": args.estimator + (f" (k={args.knn_k})" if knn else ""),
            "radius2": radius2,
            "exchange": args.exchange if world > 1 else "none",
            "parallelism": f"photon-shard x{world}" if world > 1 else "single",
        },
        "mgather_samples_per_s": round(g_points * args.steps / elapsed / 1e6, 3),
        "kernel_rates": {
            "trace_mphotons_per_s": round(args.paths / (stages["trace"] * 1e-3) / 1e6, 2) if "trace" in stages else None,
            "gather_msamples_per_s": round(g_points / (gather_ms * 1e-3) / 1e6, 2) if gather_ms > 0 else None,
        },
        "stages_ms": stages,
        "setup_s": round(setup_s, 3),
        "roofline": roofline,
        "trace_roofline": trace_roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(scene, RenderParams.defaults(paths_per_pass=args.paths, **est),
                                               args.cpu_threads)
        except Exception as exc:  # the baseline is reported, never required for the GPU number
            out["cpu_baseline"] = {"error": repr(exc)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
