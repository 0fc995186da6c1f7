"""k_gather_tile (or with argument knn: k_gather_knn_ss, PM_KNN_SS=0: k_gather_knn_tile) event counts at C2 (PM_TILE_STATS variant build):
   make -C cuda-raytrace_amd variant NAME=tstats VFLAGS=-DPM_TILE_STATS
   PMHIP_LIB=cuda-raytrace_amd/lib/variants/libpmhip_tstats.so python tools/tile_stats.py"""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "cuda-raytrace_amd"))
import torch  # noqa: F401
from pmrender import hip, scenes
from pmrender.abi import RenderParams
C5 = "c5" in sys.argv[1:]
C3 = "c3" in sys.argv[1:]
sc = (scenes.caustic_scene(1920, 1080) if C5 else
      scenes.triangle_soup(1_000_000, 1920, 1080) if C3 else scenes.cornell_box(1920, 1080))
ctx = sc.load_into(hip.Context(0))
KNN = "knn" in sys.argv[1:]
PATHS = 1_048_576 if (C5 or C3) else 262144
if KNN:
    from pmrender.abi import PM_ESTIMATOR_KNN
    p = RenderParams.defaults(paths_per_pass=PATHS, initial_radius2=100.0, estimator=PM_ESTIMATOR_KNN, knn_lookup=50)
else:
    p = RenderParams.defaults(paths_per_pass=PATHS)
# passes=N: progressive passes 0..N-1 first, then pass N is counted
NP = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("passes=")), 0)
ctx.eye_pass(p)
for k in range(NP):
    ctx.trace_photons(p, k, 0, PATHS)
    ctx.build_photon_map(p, PATHS * 4)
    ctx.gather(p)
ctx.trace_photons(p, NP, 0, PATHS)
ctx.build_photon_map(p, PATHS * 4)
ctx.synchronize()
ctx.trace_profile(reset=True)
ctx.gather(p)
ctx.synchronize()
v = list(ctx.trace_profile().values())
names = ["tile_waves", "windows", "test_pairs", "hit_iters", "direct_lanes", "chunks", "wide_waves", "staged"]
if KNN and os.environ.get("PM_KNN_SS", "1") != "0":  # k_gather_knn_ss (the default kNN kernel)
    names = ["tile_waves", "passes", "hist_passes", "rows", "hist_pairs", "collect_pairs", "sum_pairs", "sum_pairs_hit"]
elif KNN:  # k_gather_knn_tile: per-wave sums
    names = ["groups", "passes", "windows", "staged", "hit_iters", "direct_lanes", "min_lane_passes", "rebin_lane_passes"]
if os.environ.get("PM_COOP_STATS_NAMES"):
    names = ["waves_direct", "sum_cand", "sum_tot", "max_tot", "sum_direct", "waves_cand16", "tot_cand16", "max_cand"]
    print("map", ctx.map_info())
for k, x in zip(names, v):
    print(f"{k:14s} {x:12d}  per tile wave {x / max(v[0], 1):8.2f}")
