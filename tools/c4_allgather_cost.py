#!/usr/bin/env python3
"""Per-rank work of the all-gather exchange at C4, measured on
one GPU with one context: the full 8-rank photon map (4,194,304 paths = 8 x
524,288; what every rank holds after the slot all-gather) is built, and rank
0's 8-row bands (pmrender/dist.py _bands, 1/8 of the 4K records) are
gathered. Stage times from the context's HIP events. The reduce mode's
per-rank work is `bench.py --config c4` (all records against the rank's
own 524,288 paths)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))
import torch  # noqa: F401,E402  (one HIP runtime per process)
from pmrender import hip, scenes  # noqa: E402
from pmrender.abi import RenderParams  # noqa: E402
from pmrender.dist import _bands  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sc = scenes.cornell_box(3840, 2160)
ctx = sc.load_into(hip.Context(0))
paths = 524_288 * world
p = RenderParams.defaults(paths_per_pass=paths, initial_radius2=4.0)     # bench.py c4
ctx.set_stage_timing("all")
ctx.eye_pass(p)
bands = _bands(ctx.num_records(), ((3840 + 7) // 8) * 64, world)[0]
out = []
for it in range(6):
    ctx.timing_reset()
    ctx.reset_records(p)
    ctx.trace_photons(p, 0, 0, paths)
    ctx.build_photon_map(p, paths * 4)
    for b, c in bands:
        ctx.gather_range(p, b, c)
    ctx.synchronize()
    if it >= 2:
        out.append({k: round(ctx.timing_total(k)[1], 4) for k in ("trace", "build", "gather")})
info = ctx.map_info()
ctx.close()
print(json.dumps({"what": f"C4 all-gather mode, one rank of {world}: build of the full map + gather of its bands",
                  "paths_in_map": paths, "photons_valid": info["valid"], "bands": len(bands),
                  "records_gathered": sum(c for _, c in bands), "runs_ms": out}))
