"""Debug: compare k_gather_tile vs k_gather_grid partials per record (GPU)."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "cuda-raytrace_amd")); sys.path.insert(0, os.path.join(R, "oracle"))
import torch
import oracle
from pmrender import hip, scenes
from pmrender.abi import PM_GATHER_GRID, RenderParams
W, H, paths, r2 = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
sc = scenes.cornell_box(W, H)
orc = sc.load_into(oracle.Oracle())
p = RenderParams.defaults(paths_per_pass=paths, initial_radius2=r2)
recs = orc.eye_pass(p); slots = orc.trace_photons(p, 0, 0, paths)
p.gather_structure = PM_GATHER_GRID
outs = {}
for k in ("lane", "tile"):
    os.environ["PM_GATHER_KERNEL"] = k
    ctx = sc.load_into(hip.Context(0))
    ctx.upload_records(recs); ctx.upload_slots(slots); ctx.build_photon_map(p, len(slots))
    part = torch.zeros((len(recs), 4), dtype=torch.int64, device="cuda"); torch.cuda.synchronize()
    ctx.gather_partial(p, part.data_ptr()); ctx.synchronize()
    outs[k] = part.cpu().numpy(); ctx.close()
a, b = outs["lane"], outs["tile"]
bad = np.where((a != b).any(1))[0]
print("records", len(recs), "bad", len(bad), "tiles bad", len(np.unique(bad // 64)))
for i in bad[:20]:
    print(i, i // 64, i % 64, a[i], b[i])
