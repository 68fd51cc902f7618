"""Per-step kernel census from a rocprofv3 --kernel-trace csv of bench.py.

    python tools/step_kernels.py run_kernel_trace.csv [--step -5]

Steps are delimited by the Adam kernel (k_adam_flat, or torch's fused Adam); prints the dispatches of one
replayed step grouped by kernel name (count, total and mean duration) and the
busy time per hardware queue.
"""
import argparse
import csv
import re
from collections import Counter, defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"at::native::", "", n)
    return n[:78]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-5)
    ap.add_argument("--dump", default="", help="write the step's dispatches (start, us, queue, "
                                               "grid, workgroup, name) to this csv")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows)
           if "FusedOptimizer" in r["Kernel_Name"] or "k_adam_flat" in r["Kernel_Name"]]
    a, b = idx[args.step - 1], idx[args.step]
    st = rows[a + 1:b + 1]
    span = (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3
    if args.dump:
        t0 = int(st[0]["Start_Timestamp"])
        gk = next((k for k in ("Grid_Size", "Grid_Size_X") if k in st[0]), None)
        wk = next((k for k in ("Workgroup_Size", "Workgroup_Size_X") if k in st[0]), None)
        with open(args.dump, "w") as f:
            f.write("start_us,dur_us,queue,grid,wg,lds,name\n")
            for r in st:
                f.write(f"{(int(r['Start_Timestamp']) - t0) / 1e3:.1f},"
                        f"{(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.1f},"
                        f"{r['Queue_Id']},{r.get(gk, '')},{r.get(wk, '')},"
                        f"{r.get('LDS_Block_Size', r.get('Lds_Size', ''))},"
                        f"\"{short(r['Kernel_Name'])}\"\n")
    q = defaultdict(float)
    c, t = Counter(), defaultdict(float)
    for r in st:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        q[r["Queue_Id"]] += d
        c[short(r["Kernel_Name"])] += 1
        t[short(r["Kernel_Name"])] += d
    print(f"step: {len(st)} dispatches, span {span:.1f} us, busy per queue "
          + ", ".join(f"q{k}: {v:.0f} us" for k, v in sorted(q.items())))
    for n in sorted(c, key=lambda n: -t[n]):
        print(f"{c[n]:4d} {t[n]:8.1f} {t[n] / c[n]:6.1f}  {n}")


if __name__ == "__main__":
    main()
