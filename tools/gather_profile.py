"""k_gather_tile (argument knn: k_gather_knn_ss, PM_KNN_SS=0: k_gather_knn_tile) phase clocks (PM_GATHER_PROFILE variant build) at C2 / C3 / C5:
   make -C cuda-raytrace_amd variant NAME=gprof VFLAGS=-DPM_GATHER_PROFILE
   PMHIP_LIB=cuda-raytrace_amd/lib/variants/libpmhip_gprof.so python tools/gather_profile.py [c3|c5]
Prints the summed wave clock per phase (record load, group forming + row
bounds, LDS staging, distance tests, hit sums, per-lane scans, store) as a
share of all waves' lifetime and per wave; the run is launched twice and the
second launch is reported (warm caches, like the bench's timed passes)."""
import os
import sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "cuda-raytrace_amd"))
import torch  # noqa: F401
from pmrender import hip, scenes
from pmrender.abi import RenderParams
C5, C3, KNN = "c5" in sys.argv[1:], "c3" in sys.argv[1:], "knn" in sys.argv[1:]
sc = (scenes.caustic_scene(1920, 1080) if C5 else
      scenes.triangle_soup(1_000_000, 1920, 1080) if C3 else scenes.cornell_box(1920, 1080))
ctx = sc.load_into(hip.Context(0))
PATHS = 1_048_576 if (C5 or C3) else 262144
if KNN:  # k_gather_knn_tile (BASELINE C2 kNN line: K = 50, maxD^2 = 100)
    from pmrender.abi import PM_ESTIMATOR_KNN
    p = RenderParams.defaults(paths_per_pass=PATHS, initial_radius2=100.0, estimator=PM_ESTIMATOR_KNN, knn_lookup=50)
else:
    p = RenderParams.defaults(paths_per_pass=PATHS)
# passes=N: progressive passes 0..N-1 first (radii shrink, the adaptive grid
# follows them), then pass N is the one profiled (the bench's timed state)
NP = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("passes=")), 0)
ctx.eye_pass(p)
for k in range(NP):
    ctx.trace_photons(p, k, 0, PATHS)
    ctx.build_photon_map(p, PATHS * 4)
    ctx.gather(p)
ctx.trace_photons(p, NP, 0, PATHS)
ctx.build_photon_map(p, PATHS * 4)
for rep in range(1 if NP else 2):
    if not NP:
        ctx.reset_records(p)
    ctx.synchronize()
    ctx.trace_profile(reset=True)
    ctx.gather(p)
    ctx.synchronize()
v = list(ctx.trace_profile().values())
names = (["record+groups", "pass_setup", "hist", "collect", "sum", "pass_end", "store"]
         if KNN and os.environ.get("PM_KNN_SS", "1") != "0" else
         ["record", "pass_setup", "stage", "test", "hits", "pass_end", "direct+store"] if KNN else
         ["record", "group", "stage", "test", "hits", "direct", "store"])
tot = sum(v[:7])
waves = max(v[7], 1)
print(f"{'c5' if C5 else 'c3' if C3 else 'c2'}{' knn' if KNN else ''}: {waves} waves, {tot / waves:.0f} clocks per wave")
for k, x in zip(names, v[:7]):
    print(f"  {k:8s} {100.0 * x / max(tot, 1):6.1f} %  {x / waves:9.0f} per wave")
