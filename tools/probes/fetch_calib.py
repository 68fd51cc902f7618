"""Calibrates rocprofv3 FETCH_SIZE for k_poly_step's row-gather pattern on
known byte counts (MI355X_MICROARCH.md §HBM: only the wide coalesced stream
is calibrated, at 1/2; "calibrate on a known byte count in your own access
pattern").  Every case reads X (n x d fp32, > 100 MB: far past one XCD's L2)
through k_poly_step; the algorithmic read is X once + the CSR:

  ident     one entry per row, col = row: the row-gather kernel streaming X
            in order (the calibrated pattern);
  perm      one entry per row, col = a random permutation: every X row
            gathered exactly once, in random order;
  knn       2-D k=9 nearest-neighbour graph in Morton order (a TSP-like L0
            with locality): every row gathered ~10 times, neighbours close;
  knn_rand  the same graph, rows relabelled at random (no locality).

    rocprofv3 --pmc FETCH_SIZE -d D -o f --output-format csv -- \
        python3 tools/probes/fetch_calib.py run --meta gpurun_out/fc_meta.json
    python3 tools/probes/fetch_calib.py parse D/.../f_counter_collection.csv \
        --meta gpurun_out/fc_meta.json
"""
import argparse
import csv
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                "hl-hgat_amd"))

REPS = 3


def morton(xy, bits=16):
    q = (xy * ((1 << bits) - 1)).astype(np.uint64)
    out = np.zeros(len(xy), dtype=np.uint64)
    for b in range(bits):
        out |= ((q[:, 0] >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b)
        out |= ((q[:, 1] >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b + 1)
    return out


def knn_graph(n, k, seed):
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    xy = rng.random((n, 2))
    xy = xy[np.argsort(morton(xy), kind="stable")]
    _, nb = cKDTree(xy).query(xy, k=k + 1)
    row = np.repeat(np.arange(n), k + 1)  # self + k neighbours
    col = nb.reshape(-1)
    a = np.unique(np.concatenate([np.stack([row, col], 1), np.stack([col, row], 1)]), axis=0)
    return a[:, 0], a[:, 1]


def run(args):
    import torch
    from hlhgat import ops
    dev = torch.device("cuda:0")
    n, d = args.n, args.d
    rng = np.random.default_rng(1)
    cases = {"ident": (np.arange(n), np.arange(n)),
             "perm": (np.arange(n), rng.permutation(n))}
    r, c = knn_graph(n, 9, 2)
    cases["knn"] = (r, c)
    lab = rng.permutation(n)
    r2, c2 = lab[r], lab[c]
    o = np.lexsort((c2, r2))
    cases["knn_rand"] = (r2[o], c2[o])
    X = torch.randn(n, d, device=dev)
    Y = torch.empty(n, d, device=dev)
    meta = {"n": n, "d": d, "reps": REPS, "order": [], "cases": {}}
    for name, (row, col) in cases.items():
        row_t = torch.from_numpy(np.ascontiguousarray(row)).to(dev, torch.int64)
        col_t = torch.from_numpy(np.ascontiguousarray(col)).to(dev, torch.int64)
        w = torch.ones(row_t.numel(), device=dev)
        A = ops._csr_sorted(row_t, col_t, w, n, n)
        torch.cuda.synchronize()
        for _ in range(REPS):
            ops._poly_step(A, X, Y)
            meta["order"].append(name)
        torch.cuda.synchronize()
        nnz = int(A.nnz)
        meta["cases"][name] = {"nnz": nnz, "x_bytes": 4 * n * d,
                               "csr_bytes": 8 * nnz + 4 * (n + 1),
                               "read_bytes": 4 * n * d + 8 * nnz + 4 * (n + 1),
                               "gathered_bytes": 4 * nnz * d}
    with open(args.meta, "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta["cases"]))


def parse(args):
    meta = json.load(open(args.meta))
    acc, names = {}, {}
    for r in csv.DictReader(open(args.csv)):
        if r.get("Counter_Name") != "FETCH_SIZE":
            continue
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        acc[did] = acc.get(did, 0.0) + float(r["Counter_Value"])
        names[did] = r["Kernel_Name"]
    polys = [acc[k] for k in sorted(acc) if "k_poly_step" in names[k]]
    if len(polys) != len(meta["order"]):
        sys.exit(f"{len(polys)} k_poly_step dispatches, expected {len(meta['order'])}")
    per = {}
    for name, v in zip(meta["order"], polys):
        per.setdefault(name, []).append(v * 1024.0)  # FETCH_SIZE is in KiB
    out = {"n": meta["n"], "d": meta["d"], "cases": {}}
    for name, vs in per.items():
        m = meta["cases"][name]
        raw = float(np.median(vs))
        out["cases"][name] = {"fetch_size_raw_bytes": round(raw),
                              "algorithmic_read_bytes": m["read_bytes"],
                              "gathered_bytes": m["gathered_bytes"],
                              "raw_over_algorithmic": round(raw / m["read_bytes"], 4),
                              "all_reps_raw": [round(v) for v in vs]}
    base = out["cases"].get("ident")
    if base:
        out["factor_from_ident"] = round(base["algorithmic_read_bytes"] /
                                         base["fetch_size_raw_bytes"], 4)
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    sp = ap.add_subparsers(dest="mode", required=True)
    a = sp.add_parser("run")
    a.add_argument("--meta", required=True)
    a.add_argument("--n", type=int, default=400000)
    a.add_argument("--d", type=int, default=64)
    b = sp.add_parser("parse")
    b.add_argument("csv")
    b.add_argument("--meta", required=True)
    args = ap.parse_args()
    run(args) if args.mode == "run" else parse(args)


if __name__ == "__main__":
    main()
