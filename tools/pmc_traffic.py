"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv \
        --kernel k_poly_step --out profiles/r01_pmc_traffic.json [--label "..."]

Corrections, as MI355X_MICROARCH.md §HBM and cdna_hip_programming.md §7 prescribe:
  * FETCH_SIZE and WRITE_SIZE are in KiB (hbm_bytes = (FETCH + WRITE) * 1024);
  * on gfx950 FETCH_SIZE reads exactly 1/2 of the bytes of a wide coalesced
    streaming read (16 B/lane).  Every row access of k_poly_step is a 16 B/lane
    float4 load (V = 4 whenever d % 4 == 0), so the read side is doubled;
  * WRITE_SIZE is exact for 16 B/lane streaming stores (k_poly_step's stores).
FETCH_SIZE counts Infinity-Cache hits as fabric reads (guide §HBM), so on a
cache-resident workload this is "bytes that left L2", an upper bound on DRAM.
FETCH_SIZE (3 TCC slots) and WRITE_SIZE (2) do not fit one pass: two runs.
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict


def per_kernel(path, counter):
    """{kernel name: [value per dispatch]} for one counter (summed over
    dimension rows of the same dispatch)."""
    acc = defaultdict(float)
    names = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r.get("Counter_Name") != counter:
                continue
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            acc[did] += float(r["Counter_Value"])
            names[did] = r["Kernel_Name"]
    out = defaultdict(list)
    for did, v in acc.items():
        out[names[did]].append(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", action="append", default=None,
                    help="substring of the kernel name (repeatable); default: all")
    ap.add_argument("--out", required=True)
    ap.add_argument("--label", default="")
    args = ap.parse_args()
    fetch = per_kernel(args.fetch_csv, "FETCH_SIZE")
    write = per_kernel(args.write_csv, "WRITE_SIZE")
    res = {"label": args.label, "fetch_correction": 2.0,
           "units": "bytes per launch (FETCH_SIZE*1024*2 + WRITE_SIZE*1024)", "kernels": {}}
    groups = defaultdict(lambda: {"fetch": [], "write": []})
    for name in set(fetch) | set(write):
        keys = args.kernel or [name]
        for k in keys:
            if k in name:
                groups[k]["fetch"] += fetch.get(name, [])
                groups[k]["write"] += write.get(name, [])
    for k, g in sorted(groups.items()):
        nf, nw = len(g["fetch"]), len(g["write"])
        fb = 2.0 * 1024.0 * sum(g["fetch"]) / max(nf, 1)
        wb = 1024.0 * sum(g["write"]) / max(nw, 1)
        res["kernels"][k] = {"launches_fetch_pass": nf, "launches_write_pass": nw,
                             "fetch_bytes": round(fb), "write_bytes": round(wb),
                             "traffic_bytes": round(fb + wb)}
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
