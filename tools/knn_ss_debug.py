"""Debug aid for k_gather_knn_ss: C2 kNN (1080p Cornell, 262,144 paths,
K = 50, r^2 = 100) gathered by the scalar-stream kernel and by the per-lane
heap kernel on the same photon map; prints the records that differ and the
kernel's PM_KNN_SS_DEBUG report (run with PMHIP_LIB=<variant built with
-DPM_KNN_SS_DBG> for the per-lane diagnostics)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))
from pmrender import hip, scenes  # noqa: E402
from pmrender.abi import PM_ESTIMATOR_KNN, RenderParams  # noqa: E402

W, H = (int(v) for v in os.environ.get("KD_SIZE", "1920x1080").split("x"))
sc = scenes.cornell_box(W, H)
p = RenderParams.defaults(paths_per_pass=262_144, initial_radius2=float(os.environ.get("KD_R2", "100")),
                          estimator=PM_ESTIMATOR_KNN, knn_lookup=int(os.environ.get("KD_K", "50")))
outs = {}
for name in ("lane", "ss"):
    os.environ["PM_GATHER_KERNEL"] = "lane" if name == "lane" else "tile"
    os.environ["PM_KNN_SS_DEBUG"] = "1"
    ctx = sc.load_into(hip.Context(0))
    ctx.eye_pass(p)
    ctx.trace_photons(p, 0, 0, 262_144)
    ctx.build_photon_map(p, 262_144 * 4)
    ctx.gather(p)
    outs[name] = ctx.download_records()
    ctx.close()
a, b = outs["ss"], outs["lane"]
ua = np.ascontiguousarray(a).view(np.uint32).reshape(len(a), -1)
ub = np.ascontiguousarray(b).view(np.uint32).reshape(len(b), -1)
bad = np.nonzero((ua != ub).any(axis=1))[0]
print(f"{bad.size} of {len(a)} records differ", flush=True)
for i in bad[:12]:
    print(i, i // 64, i % 64, a[i], b[i])
tiles = np.unique(bad // 64)
print("tiles", tiles.size, tiles[:20])
