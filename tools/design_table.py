"""Prints DESIGN.md §6 table rows from bench JSON lines (default profiles/r02)."""
import json
import os
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02"
NAMES = [("c1", "C1 Cornell 25K paths, 256²"), ("c2", "**C2 Cornell 262K paths, 1080p**"),
         ("c2_knn", "C2, kNN estimator (K = 50, r² = 100)"), ("c3", "C3 1M-triangle soup, 1M paths, 1080p"),
         ("c4", "C4 share: Cornell 524K paths, 4K"), ("c5", "C5 caustic, 1M paths / progressive pass, 1080p")]
for key, name in NAMES:
    f = os.path.join(D, "bench_%s.json" % key)
    if not os.path.exists(f):
        continue
    d = json.load(open(f))
    st, rf, cb = d["stages_ms"], d["roofline"], d["cpu_baseline"]
    tr = rf.get("traffic")
    fr = "%.2f" % rf["frac"] + (" (HBM traffic %.0f MB = %.2f × compulsory)" % (tr / 1e6, tr / rf["algorithmic_bytes_per_launch"]) if tr else "")
    print("| %s | %s | %s | %.3f | %.3f | %.3f | %.3f | %s | %.2f Mphotons/s |" % (
        name, format(round(d["value"], 1), ",.1f"), format(round(d["mgather_samples_per_s"]), ","), d["ms_per_step"],
        st["trace"], st["build"], st["gather"], fr, cb["value"]))
