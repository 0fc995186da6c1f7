"""C3 trace cost vs scene size: pooled trace of 1M paths through triangle soups
of 30K..1M triangles (same density box), per-ray node visits (census) and
time per node visit — how much of the C3 trace is cache locality."""
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "cuda-raytrace_amd"))
import torch  # noqa: F401,E402
from pmrender import hip, scenes  # noqa: E402
from pmrender.abi import RenderParams  # noqa: E402

PATHS = 1 << 20
for n in [int(x) for x in (sys.argv[1:] or ["30000", "100000", "300000", "1000000"])]:
    sc = scenes.triangle_soup(n, 64, 64)
    ctx = sc.load_into(hip.Context(0))
    p = RenderParams.defaults(paths_per_pass=PATHS)
    ctx.set_stage_timing("all")
    ctx.eye_pass(p)
    for _ in range(2):
        ctx.trace_photons(p, 0, 0, PATHS)
    ctx.synchronize()
    ctx.timing_reset()
    for _ in range(5):
        ctx.trace_photons(p, 0, 0, PATHS)
    ctx.synchronize()
    k, ms = ctx.timing_total("trace")
    ctx.set_counting(True)
    ctx.trace_photons(p, 0, 0, PATHS)
    ctx.synchronize()
    rays, nodes, prims, dep = ctx.trace_counters()
    ctx.set_counting(False)
    info = ctx.scene_info()
    t = ms / k
    print(f"tris {n:8d} scene {info['bytes'] / 1e6:7.1f} MB  trace {t:7.3f} ms  rays {rays}  nodes/ray {nodes / rays:6.2f}  "
          f"prims/ray {prims / rays:5.2f}  ns per node visit {t * 1e6 / max(nodes, 1) * 1e3:8.4f} ps", flush=True)
    ctx.close()
