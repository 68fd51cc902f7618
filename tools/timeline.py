"""GPU busy fraction from a rocprofv3 --kernel-trace csv.

    python tools/timeline.py run_kernel_trace.csv [--window-ms 50] [--skip-ms 0]

Takes the densest window of `window-ms` (the timed region of bench.py is the
longest stretch of back-to-back kernels) and reports the union of kernel
intervals (busy), the span, and the idle gaps between kernels.
"""
from __future__ import annotations

import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window-ms", type=float, default=40.0)
    args = ap.parse_args()
    iv = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    iv.sort()
    W = int(args.window_ms * 1e6)
    # best window = max number of dispatches inside [t, t+W)
    j = 0
    best = (0, 0)
    for i in range(len(iv)):
        while j < len(iv) and iv[j][0] < iv[i][0] + W:
            j += 1
        if j - i > best[0]:
            best = (j - i, i)
    cnt, i0 = best
    sel = iv[i0:i0 + cnt]
    busy = 0
    cur_s, cur_e = sel[0][0], sel[0][1]
    gaps = []
    for s, e, _ in sel[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = sel[-1][1] - sel[0][0]
    gaps.sort()
    print(f"window: {cnt} dispatches over {span/1e6:.3f} ms; busy {busy/1e6:.3f} ms "
          f"({100*busy/span:.1f} %); idle gaps: {len(gaps)}, total {sum(gaps)/1e6:.3f} ms, "
          f"median {gaps[len(gaps)//2]/1e3 if gaps else 0:.2f} us, "
          f"p90 {gaps[int(len(gaps)*0.9)]/1e3 if gaps else 0:.2f} us")


if __name__ == "__main__":
    main()
