"""k_eig_pe timing by batch composition (where its time goes): 256 graphs of
n nodes (superpixel kNN), k = 2 (Lanczos + one eigenpair) vs k = 10.

    python tools/probes/eig_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from hlhgat import ops
    from hlhgat.pipeline import superpixel_raw, to_undirected_min
    dev = torch.device("cuda:0")
    out = {}
    for n in (32, 64, 118):
        graphs = []
        for i in range(256):
            r = superpixel_raw(100 + i, n=n)
            ei, _ = to_undirected_min(r.edge_index, r.edge_attr, n)
            graphs.append(ei[:, ei[0] < ei[1]])
        offs = np.arange(257) * n
        eb = torch.from_numpy(np.ascontiguousarray(np.concatenate(
            [e + o for e, o in zip(graphs, offs[:-1])], 1))).to(dev)
        ns = [n] * 256
        for k in (2, 10):
            for _ in range(2):
                ops.eig_pe(eb, ns, k)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                ops.eig_pe(eb, ns, k)
            b.record()
            torch.cuda.synchronize()
            out[f"n{n}_k{k}_ms"] = round(a.elapsed_time(b) / 5, 3)
        a.record()
        for _ in range(5):
            ops.hodge_build(eb, ns)
        b.record()
        torch.cuda.synchronize()
        out[f"n{n}_hodge_build_ms"] = round(a.elapsed_time(b) / 5, 3)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
