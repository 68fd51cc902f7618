"""Per-launch durations and grid sizes of one replayed step, grouped by
kernel name (rocprofv3 --kernel-trace csv).

    python tools/launch_shapes.py run_kernel_trace.csv [--step -3] [--match proj_bwd]
"""
import argparse
import csv
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-3)
    ap.add_argument("--match", default="")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "k_adam_flat" in r["Kernel_Name"]]
    a, b = idx[args.step - 1], idx[args.step]
    t0 = int(rows[a + 1]["Start_Timestamp"])
    for r in rows[a + 1:b + 1]:
        n = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        if args.match and args.match not in n:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']} wg={grid // max(wg, 1):6d} "
              f"lds={r['LDS_Block_Size']:>6} vgpr={r['VGPR_Count']:>4} {n[:70]}")


if __name__ == "__main__":
    main()
