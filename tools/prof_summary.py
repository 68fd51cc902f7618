"""Summarise a rocprofv3 --stats kernel_stats.csv into markdown (top kernels)."""
import csv
import sys


def main(path, out, title, top=40):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {title}", "", f"source: `{path}`  total kernel time {tot/1e6:.2f} ms", "",
             "| total ms | % | calls | avg us | min us | max us | kernel |", "|---|---|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 120:
            name = name[:117] + "..."
        lines.append(f"| {float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} | "
                     f"{r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {float(r['MinNs'])/1e3:.2f} | "
                     f"{float(r['MaxNs'])/1e3:.2f} | `{name}` |")
    open(out, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "rocprofv3 kernel stats")
