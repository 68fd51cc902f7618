"""One-launch (graph-local) polynomial basis vs the K-1 chained launches at
the config-2 shapes (1000 ZINC graphs; L0 / L1, d = 64, K = 3), isolated,
as hipGraph chains (tools/kbench.timed); forward and adjoint.

    HLHGAT_LOCAL_NT=256|512|1024 python tools/local_bench.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd"), os.path.join(REPO, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from kbench import timed  # noqa: E402


def main():
    import bench
    from hlhgat import _lib, ops
    L = _lib.LIB
    dev = torch.device("cuda:0")
    batches, caps, _, _, _ = bench.make_batches(1, 0, dev)
    b = batches[0]
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    g = torch.Generator(device="cpu").manual_seed(0)
    for side, seg in (("t", b.seg_ptr_t), ("s", b.seg_ptr_s)):
        ei, w = getattr(b, "edge_index_" + side), getattr(b, "edge_weight_" + side)
        n = getattr(b, "x_" + side).size(0)
        A = ops.hodge_operator(ei, w, n).fwd
        for F, K in ((64, 3), (36, 3)):
            X = torch.randn(n, F, generator=g).to(dev)
            T = torch.empty(K - 1, n, F, device=dev)
            G = torch.randn(K, n, F, generator=g).to(dev)
            a = (0, A.rowptr.data_ptr(), A.col.data_ptr(), A.val.data_ptr(), n, A.nnz)
            runs = {
                "fwd chained": lambda: L.hlhgat_poly_basis_fwd(*a, None, None, X.data_ptr(), F, F,
                                                               K, T.data_ptr(), st()),
                "fwd local": lambda: L.hlhgat_poly_basis_fwd_local(
                    *a, seg.data_ptr(), seg.numel() - 1, X.data_ptr(), F, F, K, T.data_ptr(), st()),
                "bwd chained": lambda: L.hlhgat_poly_basis_bwd(*a, None, None, F, K, G.data_ptr(),
                                                               st()),
                "bwd local": lambda: L.hlhgat_poly_basis_bwd_local(
                    *a, seg.data_ptr(), seg.numel() - 1, F, K, G.data_ptr(), st()),
            }
            for name, fn in runs.items():
                iso, ch = timed(fn, 15, 20)
                print(json.dumps({"side": side, "n": n, "F": F, "K": K, "op": name,
                                  "iso_us": round(iso, 2), "chain_us": round(ch, 2),
                                  "nt": os.environ.get("HLHGAT_LOCAL_NT", "auto")}), flush=True)


if __name__ == "__main__":
    main()
