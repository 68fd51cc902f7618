"""Median per-dispatch PMC values per kernel from rocprofv3 --pmc csv files.

    python tools/pmc_kernel.py a_counter_collection.csv [b_counter_collection.csv ...] [--match k_proj]
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    args = ap.parse_args()
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch]
    for path in args.csv:
        acc = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(path)):
            if args.match not in r["Kernel_Name"]:
                continue
            acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
            names[r["Dispatch_Id"]] = m.group(1) if m else r["Kernel_Name"][:60]
        for d, cs in acc.items():
            for c, v in cs.items():
                per[names[d]][c].append(v)
    for k, cs in per.items():
        print(k)
        for c, vs in sorted(cs.items()):
            print(f"   {c:28s} {statistics.median(vs):14.0f}  (n={len(vs)})")


if __name__ == "__main__":
    main()
