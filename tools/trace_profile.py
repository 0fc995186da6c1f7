#!/usr/bin/env python3
"""Phase anatomy of k_trace from the profiling build.

    make -C cuda-raytrace_amd prof
    PMHIP_LIB=cuda-raytrace_amd/lib/libpmhip_prof.so python tools/trace_profile.py [--config c2|c3]

Prints, per wave and as a share of the wave lifetime, the shader-clock cycles
spent in emission, BVH traversal, shading/bounce, the compaction barrier and
the state exchange (pm_trace_profile)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytrace_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c2", "c3"])
    ap.add_argument("--paths", type=int, default=512 * 512)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime per process)
    from pmrender import hip, scenes
    from pmrender.abi import RenderParams
    sc = scenes.cornell_box(1920, 1080) if args.config == "c2" else scenes.triangle_soup(1_000_000, 1920, 1080)
    ctx = sc.load_into(hip.Context(0))
    p = RenderParams.defaults(paths_per_pass=args.paths)
    ctx.trace_photons(p, 0, 0, args.paths)  # warm
    ctx.synchronize()
    ctx.trace_profile(reset=True)
    ctx.timing_reset()
    for _ in range(args.reps):
        ctx.trace_photons(p, 0, 0, args.paths)
    ctx.synchronize()
    prof = ctx.trace_profile()
    n, ms = ctx.timing_total("trace")
    waves = max(prof["waves"], 1)
    life = max(prof["lifetime"], 1)
    out = {"config": args.config, "trace_ms": ms / max(n, 1), "waves_per_launch": waves / args.reps,
           "cycles_per_wave": {k: round(v / waves) for k, v in prof.items() if k not in ("waves",)},
           "share_of_lifetime": {k: round(v / life, 4) for k, v in prof.items() if k not in ("waves", "lifetime")}}
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
