#!/usr/bin/env python3
"""Per-rank cost of the all-gather exchange at C4, measured on
one GPU: a multi-device context of 8 sub-contexts on device 0 renders C4
(Cornell 3840x2160, 4,194,304 paths = 8 x 524,288) exactly as 8 GPUs would
(shards, slot all-gather by peer copies, full map on every device, 1/8 of
the records per device as 8-row bands); pm_stats' stage times are device 0's
— one rank's trace / build / gather in the all-gather mode. Compare with
the reduce mode's per-rank work, `bench.py --config c4` (gather of all
records against the rank's own photons)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))
import torch  # noqa: F401,E402  (one HIP runtime per process)
from pmrender import hip, scenes  # noqa: E402
from pmrender.abi import RenderParams  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sc = scenes.cornell_box(3840, 2160)
ctx = sc.load_into(hip.Context(0, devices=[0] * world))
p = RenderParams.defaults(paths_per_pass=524_288 * world)
ctx.render(p)  # warm-up (allocations, module load)
runs = []
for _ in range(3):
    t0 = time.perf_counter()
    img, st = ctx.render(p)
    runs.append({"wall_s": round(time.perf_counter() - t0, 4), "rank0_trace_ms": round(st["ms_trace"], 4),
                 "rank0_build_ms": round(st["ms_build"], 4), "rank0_gather_ms": round(st["ms_gather"], 4),
                 "photons_valid": st["photons_valid"]})
ctx.close()
print(json.dumps({"what": f"C4 all-gather exchange, {world} sub-contexts on one GPU: one rank's stage times",
                  "paths_total": 524_288 * world, "runs": runs}))
