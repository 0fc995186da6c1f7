#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs,
MI355X_MICROARCH.md §rocprofv3 PMC slots) into per-launch HBM bytes per kernel
and write profiles/pmc_traffic.json.

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE reads 1/2 of the bytes of wide coalesced reads -> doubled here
(flagged: uncalibrated for the gather's 16-B random reads).

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [CONFIG]
(the JSON records the hash of the HIP sources it was measured on: bench.py
uses it as `traffic` only for the same sources)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                vals[name].append(float(row["Counter_Value"]))
    return vals


def short(name):
    for k in ("k_gather_tile", "k_gather_grid", "k_gather_knn_ss", "k_knn_pack", "k_gather_knn", "k_gather_kd", "k_trace", "k_eye", "k_bucket_fill",
              "k_scan_down", "k_scan_reduce", "k_reset_records", "k_ppm_update", "k_final"):
        if k in name:
            return k
    return None


def main():
    fetch, write = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_src_sha
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)",
           "kernel_src_sha": kernel_src_sha(), "config": sys.argv[4] if len(sys.argv) > 4 else "c2",
           "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
           "kernels": {}}
    agg = defaultdict(lambda: {"fetch_kib": [], "write_kib": []})
    for name, v in fetch.items():
        k = short(name) or name[:60]
        agg[k]["fetch_kib"] += v
    for name, v in write.items():
        k = short(name) or name[:60]
        agg[k]["write_kib"] += v
    for k, d in agg.items():
        f = sum(d["fetch_kib"]) / max(len(d["fetch_kib"]), 1)
        w = sum(d["write_kib"]) / max(len(d["write_kib"]), 1)
        out["kernels"][k] = {"launches": len(d["fetch_kib"]), "fetch_kib_per_launch": round(f, 1),
                             "write_kib_per_launch": round(w, 1),
                             "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024),
                             "hbm_bytes_uncorrected": int(f * 1024 + w * 1024)}
    with open(sys.argv[3], "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
