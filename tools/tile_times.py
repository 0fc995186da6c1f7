"""Wave timeline of the C2 tile gather (PM_TILE_TIMES variant build):
   make -C cuda-raytrace_amd variant NAME=ttimes VFLAGS=-DPM_TILE_TIMES
   PMHIP_LIB=cuda-raytrace_amd/lib/variants/libpmhip_ttimes.so python tools/tile_times.py [c3|c5] [out.txt]
Each launched wave records s_memrealtime (100 MHz, chip-wide) at its start and
end and its XCC_ID / HW_ID. Reports, for the last of several warm launches: the
launch span, the wave lifetime distribution, how many waves are resident over
time (against the occupancy limit), the dispatch ramp and the drain tail."""
import os
import sys
import tempfile

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "cuda-raytrace_amd"))
import torch  # noqa: F401,E402
from pmrender import hip, scenes  # noqa: E402
from pmrender.abi import RenderParams  # noqa: E402

C5, C3, KNN = "c5" in sys.argv[1:], "c3" in sys.argv[1:], "knn" in sys.argv[1:]
name = ("c5" if C5 else "c3" if C3 else "c2") + ("_knn" if KNN else "")
sc = (scenes.caustic_scene(1920, 1080) if C5 else
      scenes.triangle_soup(1_000_000, 1920, 1080) if C3 else scenes.cornell_box(1920, 1080))
path = os.path.join(tempfile.mkdtemp(), "tt.bin")
os.environ["PM_TILE_TIMES"] = path
ctx = sc.load_into(hip.Context(0))
PATHS = 1_048_576 if (C5 or C3) else 262144
if KNN:  # BASELINE C2 kNN line: K = 50, maxD^2 = 100 (k_gather_knn_ss)
    from pmrender.abi import PM_ESTIMATOR_KNN
    p = RenderParams.defaults(paths_per_pass=PATHS, initial_radius2=100.0, estimator=PM_ESTIMATOR_KNN, knn_lookup=50)
else:
    p = RenderParams.defaults(paths_per_pass=PATHS)
ctx.eye_pass(p)
for rep in range(4):
    ctx.reset_records(p)
    ctx.trace_photons(p, 0, 0, PATHS)
    ctx.build_photon_map(p, PATHS * 4)
    ctx.gather(p)
    ctx.synchronize()
raw = np.fromfile(path, dtype=np.uint64)
# records: header (all-ones, n) then n x 4 words; the last launch
i, last = 0, None
while i < len(raw):
    n = int(raw[i + 1])
    last = raw[i + 4: i + 4 + 8 * n].reshape(n, 8)
    i += 4 + 8 * n
rec = last[last[:, 1] > 0].astype(np.int64)
t0, t1 = rec[:, 0], rec[:, 1]
base = t0.min()
s, e = (t0 - base) * 0.01, (t1 - base) * 0.01         # us (100 MHz)
life = e - s
span = e.max()
out = []
out.append(f"{name}: {len(rec)} waves, launch span {span:.1f} us (first start -> last end)")
q = np.percentile(life, [50, 90, 99])
out.append(f"  wave lifetime: mean {life.mean():.2f} us, p50 {q[0]:.2f}, p90 {q[1]:.2f}, p99 {q[2]:.2f}, max {life.max():.2f}")
out.append(f"  sum of lifetimes / span = {life.sum() / span:.0f} waves resident on average "
           f"(limit {(6 if KNN else 5) * 4 * 256} at {6 if KNN else 5} waves/SIMD)")
grid = np.arange(0, span + 1.0, 1.0)
res = np.array([((s <= t) & (e > t)).sum() for t in grid])
out.append("  resident waves per 1-us step: " + " ".join(str(int(x)) for x in res))
ss = np.sort(s)
for k in (1024, 2560, 5120, len(ss) - 1):
    if k < len(ss):
        out.append(f"  wave #{k} started at {ss[k]:.2f} us")
es = np.sort(e)
for f in (0.5, 0.9, 0.95, 0.99):
    out.append(f"  {int(f * 100)} % of waves done at {es[int(f * (len(es) - 1))]:.2f} us")
xcc = rec[:, 2] & 0xf
for x in range(8):
    m = xcc == x
    if m.any():
        out.append(f"  XCC {x}: {m.sum()} waves, start {s[m].min():.2f} end {e[m].max():.2f} us, "
                   f"mean life {life[m].mean():.2f}")
# lifetime vs. dispatch order: the slowest tiles
order = np.argsort(-life)[:10]
blk = np.nonzero(last[:, 1] > 0)[0]
lo32 = lambda v: v & 0xffffffff  # noqa: E731
hi32 = lambda v: v >> 32  # noqa: E731
if KNN:
    st = {"passes": lo32(rec[:, 4]), "hist_passes": hi32(rec[:, 4]), "hist_pairs": lo32(rec[:, 5]),
          "collect_pairs": hi32(rec[:, 5]), "sum_pairs": lo32(rec[:, 6]), "rows": hi32(rec[:, 6]),
          "hit_batches": lo32(rec[:, 7])}
else:
    st = {"groups": lo32(rec[:, 4]), "windows": hi32(rec[:, 4]), "pairs": lo32(rec[:, 5]), "hit_iters": hi32(rec[:, 5]),
          "direct": lo32(rec[:, 6]), "chunks": hi32(rec[:, 6]), "staged": lo32(rec[:, 7])}
tile = hi32(rec[:, 7]) // 64
out.append("  per-wave means: " + ", ".join(f"{k} {v.mean():.2f}" for k, v in st.items()))
out.append("  slowest waves: block start life | tile (row, col of 240) | " + " ".join(st))
for j in order:
    out.append(f"    {int(blk[j]):6d} {s[j]:6.1f} {life[j]:6.1f} | {int(tile[j]):6d} ({int(tile[j]) // 240}, {int(tile[j]) % 240}) | " +
               " ".join(f"{int(v[j])}" for v in st.values()))
# lifetime against each count (which one explains the slow waves)
for k, v in st.items():
    if v.std() > 0:
        out.append(f"  corr(life, {k}) = {np.corrcoef(life, v)[0, 1]:+.2f}")
slow = life > np.percentile(life, 99)
out.append("  top-1% waves mean: " + ", ".join(f"{k} {v[slow].mean():.1f}" for k, v in st.items()))
if os.environ.get("PM_TT_DUMP"):  # raw per-wave records of the last launch (block order), for offline replay
    np.save(os.environ["PM_TT_DUMP"] + f"_{name}.npy", last)
txt = "\n".join(out)
print(txt)
if len(sys.argv) > 1 and sys.argv[-1].endswith(".txt"):
    with open(sys.argv[-1], "a") as f:
        f.write(txt + "\n")
