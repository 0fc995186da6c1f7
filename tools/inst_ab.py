"""Two-level instance trees vs the flattened mesh, same scene, same box:
stage times of full renders (trace / eye dominated by traversal) and the
committed scene bytes. usage: python tools/inst_ab.py [W H paths subdiv]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuda-raytrace_amd"))
import numpy as np  # noqa: E402

from pmrender import hip, scenes  # noqa: E402
from pmrender.abi import RenderParams  # noqa: E402

W, H, paths, subdiv = (int(a) for a in (sys.argv[1:] + ["1920", "1080", "262144", "6"])[:4])
sc = scenes.figure_scene(W, H, subdiv)
res = {}
for name, inst in (("two-level", True), ("flattened", False), ("two-level", True), ("flattened", False)):
    ctx = sc.load_into(hip.Context(0), instancing=inst)
    ctx.set_stage_timing("all")
    p = RenderParams.defaults(paths_per_pass=paths)
    img, _ = ctx.render(p)
    tr = []
    for _ in range(5):
        img, st = ctx.render(p)
        tr.append(st["ms_trace"])
    info = ctx.scene_info()
    res.setdefault(name, []).append(min(tr))
    print(f"{name:10s} mode={info['mode']:14s} tris={info['triangles']} bytes={info['bytes']} "
          f"trace_ms={min(tr):.4f} img_sum={float(np.float64(img).sum()):.6e}", flush=True)
    ctx.close()
