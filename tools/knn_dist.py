"""C2 kNN (K = 50, maxD^2 = 100): the distribution of r_k^2 / maxD^2 over the
live records after one gather, and the grid (what bounds a kNN pass needs).
   python tools/knn_dist.py"""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "cuda-raytrace_amd"))
import torch  # noqa: F401
from pmrender import hip, scenes
from pmrender.abi import RenderParams, PM_ESTIMATOR_KNN
sc = scenes.cornell_box(1920, 1080)
ctx = sc.load_into(hip.Context(0))
PATHS = 262144
p = RenderParams.defaults(paths_per_pass=PATHS, initial_radius2=100.0, estimator=PM_ESTIMATOR_KNN, knn_lookup=50)
ctx.eye_pass(p)
ctx.trace_photons(p, 0, 0, PATHS)
ctx.build_photon_map(p, PATHS * 4)
ctx.gather(p)
ctx.synchronize()
print("map", ctx.map_info())
rec = ctx.download_records()
live = rec["photon_count"] > 0
t = rec["radius2"][live] / 100.0
print("live records", int(live.sum()), "of", len(rec))
qs = [0.01, 0.1, 0.25, 0.5, 0.75, 0.9, 0.99]
print("r_k^2/maxD^2 quantiles", dict(zip(qs, np.round(np.quantile(t, qs), 4).tolist())))
print("full (cnt == K)", float((rec["photon_count"][live] == 50).mean()))
h, e = np.histogram(np.log2(np.maximum(t, 1e-9)), bins=[-30, -8, -6, -5, -4, -3, -2, -1.5, -1, -0.5, 0, 0.01])
for a, b, c in zip(e[:-1], e[1:], h):
    print(f"  log2 t in [{a:6.2f},{b:6.2f}): {c}")
