"""Kernel timeline of a rocprofv3 --kernel-trace CSV: every dispatch from the
first one whose name contains FROM, with its duration and the idle gap before
it (host stalls show as gaps).
usage: python tools/kt_timeline.py run_kernel_trace.csv [FROM] [N]"""
import csv
import sys

path = sys.argv[1]
frm = sys.argv[2] if len(sys.argv) > 2 else "k_trace"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 80
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
first = next(i for i, r in enumerate(rows) if frm in r["Kernel_Name"])
prev = None
for r in rows[first:first + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev is not None else 0.0
    prev = e
    print(f"{(s - t0) / 1000:10.1f} us  dur {(e - s) / 1000:8.1f}  gap {gap:7.1f}  {r['Kernel_Name'][:72]}")
