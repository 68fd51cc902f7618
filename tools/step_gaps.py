"""Idle gaps inside one replayed training step (rocprofv3 --kernel-trace csv).

    python tools/step_gaps.py run_kernel_trace.csv [--step -3] [--top 20]

Steps are delimited by the fused Adam kernel (as tools/step_kernels.py).
Prints the step span, the union of kernel intervals (GPU busy), the time with
exactly one / two queues busy, and the largest all-idle gaps with the kernels
that end / start them: the dependency stalls of the step.
"""
import argparse
import csv
import re


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"at::native::", "", n)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-3)
    ap.add_argument("--top", type=int, default=20)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", r.get("Stream_Id", "0"))))
    rows.sort()
    adam = [i for i, r in enumerate(rows) if "FusedAdam" in r[2] or "Adam" in r[2]]
    a, b = adam[args.step - 1], adam[args.step]
    st = rows[a + 1:b + 1]
    t0, t1 = st[0][0], max(r[1] for r in st)
    ev = []
    for s, e, n, q in st:
        ev += [(s, 1), (e, -1)]
    ev.sort()
    level, last, busy, one, two = 0, t0, 0, 0, 0
    for t, d in ev:
        if level >= 1:
            busy += t - last
        if level == 1:
            one += t - last
        if level >= 2:
            two += t - last
        level += d
        last = t
    print(f"step: {len(st)} dispatches, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"1 queue {one / 1e3:.1f} us, >=2 queues {two / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
    gaps = []
    end_max, prev = st[0][1], st[0]
    for r in st[1:]:
        if r[0] > end_max:
            gaps.append((r[0] - end_max, prev, r))
        if r[1] > end_max:
            end_max, prev = r[1], r
    gaps.sort(key=lambda g: -g[0])
    print(f"{len(gaps)} all-idle gaps, total {sum(g[0] for g in gaps) / 1e3:.1f} us; largest:")
    for g, p, n in gaps[:args.top]:
        print(f"  {g / 1e3:7.2f} us  after {short(p[2])}  ->  {short(n[2])}")


if __name__ == "__main__":
    main()
