"""Per-call-site census of k_poly_step (and k_edge_gather2) from a bench.py
log: the config-2 step's eager stamps (roofline.call_sites) and each head's
eager-step kernel classes (heads.*.kernels_eager_step).  Prints a table:
site, launches / step, us / step, algorithmic bytes / step, GB/s."""
import json
import sys


def main(path):
    line = [x for x in open(path) if x.startswith('{"metric')][-1]
    r = json.loads(line)
    rows = []
    for nm, e in (r["roofline"].get("call_sites") or {}).items():
        rows.append(("cfg2", nm, e["launches_per_step"], e["us_per_step"],
                     e["bytes_per_step"], e["gbs"]))
    g2 = (r.get("rooflines") or {}).get("k_edge_gather2")
    if g2 and "launches_per_step" not in g2:  # eager stamps (--no-replay-census)
        n = 3  # the bench's --prof-steps default
        rows.append(("cfg2", "k_edge_gather2 (eager)", round(g2["launches"] / n, 1),
                     round(g2["avg_launch_us"] * g2["launches"] / n, 1),
                     round(g2["per_launch"] * g2["launches"] / n), g2["achieved"]))
    elif g2:  # the replayed step's entry (per step)
        rows.append(("cfg2", "k_edge_gather2 (replayed)", g2["launches_per_step"],
                     g2["time_per_step_us"], g2["work_per_step"], g2["achieved"]))
    for head, h in (r.get("heads") or {}).items():
        if not isinstance(h, dict) or "kernels_eager_step" not in h:
            continue
        for nm, e in h["kernels_eager_step"]["classes"].items():
            if "poly" not in nm and "gather2" not in nm:
                continue
            rows.append((head, nm, e["launches"], round(e["ms_per_step"] * 1e3, 1),
                         e["per_launch"] * e["launches"], e["achieved"]))
    print(f"{'workload':20s} {'call site':62s} {'launch':>7s} {'us':>9s} {'MB':>9s} {'GB/s':>8s}")
    for w, nm, n, us, b, gbs in rows:
        print(f"{w:20s} {nm[:62]:62s} {n:7.1f} {us:9.1f} {b / 1e6:9.2f} {gbs or 0:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
