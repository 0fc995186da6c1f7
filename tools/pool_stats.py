"""Lane occupancy of k_trace_pool's steps at C3 (PM_POOL_STATS variant):
   make -C cuda-raytrace_amd variant NAME=pstats VFLAGS=-DPM_POOL_STATS
   PMHIP_LIB=.../libpmhip_pstats.so python tools/pool_stats.py"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "cuda-raytrace_amd"))
import torch  # noqa: F401,E402
from pmrender import hip, scenes  # noqa: E402
from pmrender.abi import RenderParams  # noqa: E402

PATHS = 1 << 20
sc = scenes.triangle_soup(1_000_000, 64, 64)
ctx = sc.load_into(hip.Context(0))
p = RenderParams.defaults(paths_per_pass=PATHS)
ctx.eye_pass(p)
ctx.trace_photons(p, 0, 0, PATHS)
ctx.synchronize()
ctx.trace_profile(reset=True)
ctx.trace_photons(p, 0, 0, PATHS)
ctx.synchronize()
v = list(ctx.trace_profile().values())
steps, node_lanes, leaf_lanes, shades, shade_lanes, refill_lanes = v[:6]
waves = 4096
print(f"per wave: trav steps {steps / waves:.0f}, shade rounds {shades / waves:.0f}")
print(f"lanes per trav step: node {node_lanes / max(steps, 1):.1f}, leaf {leaf_lanes / max(steps, 1):.1f}, "
      f"idle {64 - (node_lanes + leaf_lanes) / max(steps, 1):.1f}")
print(f"lanes per shade round: shading {shade_lanes / max(shades, 1):.1f}, refilled {refill_lanes / max(shades, 1):.1f}")
