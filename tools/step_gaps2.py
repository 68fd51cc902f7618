"""Per-queue gap analysis of one replayed bench step (rocprofv3 kernel trace):
for each hardware queue, busy time, idle gaps between consecutive kernels
(histogram), and how much of each gap overlaps work on the other queue."""
import csv
import sys
from collections import defaultdict


def main(path, step=-5):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "FusedOptimizer" in r["Kernel_Name"]]
    st = rows[idx[step - 1] + 1: idx[step] + 1]
    t0 = int(st[0]["Start_Timestamp"])
    span = (int(st[-1]["End_Timestamp"]) - t0) / 1e3
    byq = defaultdict(list)
    for r in st:
        byq[r["Queue_Id"]].append(((int(r["Start_Timestamp"]) - t0) / 1e3,
                                   (int(r["End_Timestamp"]) - t0) / 1e3, r["Kernel_Name"][:60]))
    print(f"span {span:.1f} us, {len(st)} dispatches")
    for q, ks in sorted(byq.items()):
        ks.sort()
        busy = sum(e - s for s, e, _ in ks)
        gaps = [ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1)]
        hist = defaultdict(int)
        for g in gaps:
            b = "<0" if g < 0 else ("<1" if g < 1 else ("<2" if g < 2 else ("<4" if g < 4 else (
                "<8" if g < 8 else ("<16" if g < 16 else ">=16")))))
            hist[b] += 1
        print(f"queue {q}: {len(ks)} kernels, busy {busy:.0f} us, gaps total "
              f"{sum(g for g in gaps if g > 0):.0f} us, median gap "
              f"{sorted(gaps)[len(gaps) // 2]:.2f} us, hist {dict(hist)}")


if __name__ == "__main__":
    main(sys.argv[1])
