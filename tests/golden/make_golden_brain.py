"""Golden fixture on the reference's own brain skeleton (HL-HGAT-DEMO data):
the skewed-degree stress case of SURVEY §8c.

    python tests/golden/make_golden_brain.py [/root/reference]

The skeleton is built as the DEMO notebook builds it (OHBM_DEMO.ipynb cells
19 / 46): fc = Group_FC.mat['fc_mean'] with fc < 0 -> 0.001, mask =
Group_FCMask.mat['sf_mask'], skeleton = triu(fc * mask, 1).to_sparse(); L0 / L1
= 2 B1 B1^T / lmax, 2 B1^T B1 / lmax with lmax from torch.linalg.eigh of the
dense L0 (the reference's adj2par1 + dense_to_sparse).  268 nodes, 8997
edges, nnz(L1) 1.37 M (152 entries per row).  The .mat files are data
(scipy.io.loadmat, no code).  The fixture stores the skeleton (edge_index,
values), lmax, and the reference HodgeLaguerreConv(8, 8, K=3) forward and
weight / input gradients on L0 and L1 for seeded inputs; the test rebuilds L1
from edge_index and lmax (fl(2 v / lmax), exactly the reference's entries,
checked here) instead of storing 1.37 M COO entries.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "hl-hgat_amd"))

from make_golden import _np, _save  # noqa: E402


def main(ref_root):
    import pyg_standin
    pyg_standin.install()
    sys.path.insert(0, ref_root)
    from scipy.io import loadmat
    import lib.Hodge_Cheb_Conv as ref           # noqa: E402  (reference code)
    import lib.Hodge_Dataset as ref_ds          # noqa: E402
    from torch_geometric.utils import dense_to_sparse  # stand-in (documented semantics)
    torch.set_num_threads(1)
    demo = os.path.join(ref_root, "HL-HGAT-DEMO", "data")
    fc = torch.tensor(loadmat(os.path.join(demo, "Group_FC.mat"))["fc_mean"])
    fc[fc < 0] = 0.001
    mask = torch.tensor(loadmat(os.path.join(demo, "Group_FCMask.mat"))["sf_mask"])
    skeleton = torch.triu(fc * mask, diagonal=1).to_sparse()
    ei = skeleton.indices()
    n = int(ei.max()) + 1
    par1 = ref_ds.adj2par1(ei, n, ei.shape[-1]).to_dense()
    L0 = torch.matmul(par1, par1.T)
    lmax = torch.linalg.eigh(L0)[0].max()
    L0 = 2 * torch.matmul(par1, par1.T) / lmax
    L1 = 2 * torch.matmul(par1.T, par1) / lmax
    eit, ewt = dense_to_sparse(L0)
    eis, ews = dense_to_sparse(L1)
    E = ei.shape[1]
    # the test's rebuild: fl(2 v / lmax) from B1 and lmax must equal L1 exactly
    from hlhgat.hodge_dataset import hodge_factor_ok
    assert hodge_factor_ok(_np(ei), n, _np(eis), _np(ews))
    arrays = dict(edge_index=_np(ei), values=_np(skeleton.values()).astype(np.float32),
                  lmax=np.float32(lmax.item()), n_nodes=np.int64(n), nnz_t=np.int64(eit.shape[1]),
                  nnz_s=np.int64(eis.shape[1]))
    # samples + checksums of the reference COO (the test rebuilds it bitwise)
    for side, (e, w) in {"t": (eit, ewt), "s": (eis, ews)}.items():
        idx = np.linspace(0, e.shape[1] - 1, 2000).astype(np.int64)
        arrays[f"{side}/coo_idx"] = idx
        arrays[f"{side}/coo_rc"] = _np(e[:, idx])
        arrays[f"{side}/coo_w"] = _np(w[idx])
        arrays[f"{side}/w_sum64"] = np.float64(w.double().sum().item())
        arrays[f"{side}/w_abs_sum64"] = np.float64(w.double().abs().sum().item())
    for side, (e, w, rows) in {"t": (eit, ewt, n), "s": (eis, ews, E)}.items():
        torch.manual_seed(7 if side == "t" else 8)
        conv = ref.HodgeLaguerreConv(8, 8, K=3)
        with torch.no_grad():
            conv.bias.uniform_(-0.5, 0.5)
        x = torch.randn(rows, 8, requires_grad=True)
        out = conv(x, e, w)
        R = torch.randn(out.shape, generator=torch.Generator().manual_seed(9))
        (out * R).sum().backward()
        arrays.update({f"{side}/x": _np(x), f"{side}/out": _np(out), f"{side}/R": _np(R),
                       f"{side}/gx": _np(x.grad), f"{side}/bias": _np(conv.bias),
                       f"{side}/gbias": _np(conv.bias.grad)})
        for k, lin in enumerate(conv.lins):
            arrays[f"{side}/w{k}"] = _np(lin.weight)
            arrays[f"{side}/gw{k}"] = _np(lin.weight.grad)
    _save("brain_skeleton", **arrays)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
