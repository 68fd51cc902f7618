"""Dump the per-queue timeline of replayed cfg2 steps from a rocprofv3
--kernel-trace csv of `bench.py --replay-probe` (steps delimited by the Adam
kernel), and summarise where each hardware queue waits.

    python tools/replay_timeline.py TRACE.csv --out timeline.csv   # on the box
    python tools/replay_timeline.py --load timeline.csv             # analysis

Per queue: busy time, the gaps before each kernel, and for each gap whether the
other queue was busy during it (a cross-queue wait: the kernel waited for the
other chain) or idle too (launch / dependency latency with nothing running).
"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    return n[:40]


def load_trace(path, nsteps):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k_adam_flat" in r["Kernel_Name"]]
    out = []
    for s, (a, b) in enumerate(zip(marks[-nsteps - 1:-1], marks[-nsteps:])):
        st = rows[a + 1:b + 1]
        t0 = int(st[0]["Start_Timestamp"])
        for r in st:
            out.append((s, r["Queue_Id"], (int(r["Start_Timestamp"]) - t0) / 1e3,
                        (int(r["End_Timestamp"]) - t0) / 1e3, short(r["Kernel_Name"])))
    return out


def busy_at(iv, s, e):
    """Length of [s, e] covered by the intervals iv (sorted, may overlap)."""
    tot, cur = 0.0, s
    for a, b in iv:
        if b <= cur:
            continue
        if a >= e:
            break
        lo, hi = max(a, cur), min(b, e)
        if hi > lo:
            tot += hi - lo
            cur = hi
    return tot


def analyse(rows):
    steps = sorted({r[0] for r in rows})
    for s in steps:
        st = [r for r in rows if r[0] == s]
        span = max(r[3] for r in st) - min(r[2] for r in st)
        byq = defaultdict(list)
        for r in st:
            byq[r[1]].append(r)
        print(f"step {s}: {len(st)} dispatches, span {span:.1f} us")
        for q, ks in sorted(byq.items()):
            ks.sort(key=lambda r: r[2])
            other = sorted((r[2], r[3]) for r in st if r[1] != q)
            busy = sum(r[3] - r[2] for r in ks)
            waits = []
            for prev, k in zip(ks, ks[1:]):
                g = k[2] - prev[3]
                if g > 0:
                    ob = busy_at(other, prev[3], k[2])
                    waits.append((g, ob, prev[4], k[4], k[2]))
            tot = sum(w[0] for w in waits)
            cross = sum(w[1] for w in waits)
            print(f"  queue {q}: {len(ks)} kernels, busy {busy:.0f} us, waiting {tot:.0f} us "
                  f"(other queue busy {cross:.0f} us of it), first start {ks[0][2]:.0f}, "
                  f"last end {ks[-1][3]:.0f}")
            for g, ob, a, b, t in sorted(waits, reverse=True)[:12]:
                print(f"    {g:7.1f} us at {t:7.1f} (other busy {ob:5.1f})  {a} -> {b}")
        # order of the step, compressed: queue, start, end, name
        print("  timeline:")
        for r in sorted(st, key=lambda r: r[2]):
            print(f"    q{r[1]} {r[2]:8.1f} {r[3]:8.1f} {r[3] - r[2]:6.1f}  {r[4]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="?")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--out", default="")
    ap.add_argument("--load", default="")
    args = ap.parse_args()
    if args.load:
        rows = [(int(r[0]), r[1], float(r[2]), float(r[3]), r[4])
                for r in csv.reader(open(args.load))]
    else:
        rows = load_trace(args.trace, args.steps)
    if args.out:
        with open(args.out, "w", newline="") as f:
            csv.writer(f).writerows(rows)
        return
    analyse(rows)


if __name__ == "__main__":
    main()
