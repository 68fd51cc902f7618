"""Golden fixtures at the BASELINE configs' OWN hyperparameters, generated from
the REFERENCE itself, plus HL_filter and SAPool.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden_baseline.py [/root/reference]

* baseline_cfg3_cifar.npz: HL_HGCNN_CIFAR10SP_dense_int3_attpool with config
  3's settings (channels [2,2,2], filters [64,128,256], mlp [256], K=4, keig=10,
  pool_loc=1, l=0.5; main_cifar10SP...:35-36,186-187) on two CIFAR-like
  superpixel graphs (n=118, 8-NN) and their MLGC coarsening.
* baseline_cfg4_pepfunc.npz: HL_HGCNN_pepfunc_dense_int3_attpool with config
  4's settings (channels [2,2,2], filters [64,128,256], mlp [256], K=6,
  pool_loc=1; main_pepfunc...:27-28,36-168) on two peptide-like molecules.
* baseline_cfg5_tsp.npz: HL_HGCNN_TSP_dense_int3_pyr with config 5's settings
  (channels [4,4,4], filters [32,64,128], mlp [256], K=4; main_TSP...:41,47)
  on one 300-node TSP-like graph (9-NN).
* hl_filter_dense.npz / hl_filter_plain.npz: HL_filter (lib/Hodge_Cheb_Conv.py:
  117-188) with LeakyReLU(0.1), if_dense True / False.
* sapool.npz: SAPool (lib/Hodge_Cheb_Conv.py:36-59) on a two-level batch.

Parameters are not stored: generator and tests overwrite every parameter with
baseline_params.fill_params(model, seed).  Large gradients are stored as 256
sampled entries + max / sum (baseline_params.grad_record).  Inputs come from
hlhgat's host-side synthetic generators + collate; the models are the
reference's classes on CPU behind pyg_standin.py.  Plain .npz, no pickles;
nothing from the reference source is copied.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "hl-hgat_amd"))

from baseline_params import fill_params, grad_record  # noqa: E402
from make_golden import _np, _save  # noqa: E402

KEYS = ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
        "edge_index", "num_node1", "num_edge1")

# config -> (model kwargs, seed); the tests import this table
CFG3 = dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256], K=4, keig=10,
            pool_loc=1, l=0.5)
CFG4 = dict(channels=[2, 2, 2], filters=[64, 128, 256], mlp_channels=[256], K=6, pool_loc=1)
CFG5 = dict(channels=[4, 4, 4], filters=[32, 64, 128], mlp_channels=[256], K=4)
HLF_DENSE = dict(channels=2, filters=16, K=3, node_dim=16, edge_dim=16, leaky_slope=0.1,
                 if_dense=True)
HLF_PLAIN = dict(channels=2, filters=16, K=3, node_dim=12, edge_dim=8, leaky_slope=0.1,
                 if_dense=False)
SAPOOL = dict(d=24, dk=8)


class _RefData:
    def to(self, device):
        return self


def _ref_data(b):
    d = _RefData()
    for k in KEYS:
        setattr(d, k, getattr(b, k))
    d.num_node1 = torch.as_tensor(b.num_node1).view(-1)
    d.num_edge1 = torch.as_tensor(b.num_edge1).view(-1)
    return d


def _batch_arrays(prefix, b):
    return {f"{prefix}{k}": _np(torch.as_tensor(getattr(b, k))) for k in KEYS}


def baseline_batches():
    """The fixtures' inputs (also rebuilt by nothing else: stored in full)."""
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import cifar_like_graphs, peptides_like_graphs, tsp_like_graph
    cif = [cifar_like_graphs(50 + s) for s in range(2)]
    pep = [peptides_like_graphs(60 + s) for s in range(2)]
    two = lambda ps: (collate([p[0] for p in ps], check_hodge=True),  # noqa: E731
                      collate([p[1] for p in ps], check_hodge=True))
    tsp = collate([tsp_like_graph(70, n=300, k=9, row_order=False)], check_hodge=True)
    return two(cif), two(pep), tsp


def _grads(m):
    out = {}
    for k, p in m.named_parameters():
        if p.grad is None:
            out["nograd/" + k] = np.int8(1)
        else:
            out.update(grad_record(k, p.grad))
    return out


def attpool_case(name, m, seed, b0, b1):
    fill_params(m, seed)
    m.train()
    out = m([_ref_data(b0), _ref_data(b1)], device="cpu")
    R = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed))
    (out * R).sum().backward()
    _save(name, out=_np(out), R=_np(R), seed=np.int64(seed), **_batch_arrays("l0/", b0),
          **_batch_arrays("l1/", b1), **_grads(m))


def tsp_case_baseline(ref_model, b, seed=5):
    m = ref_model.HL_HGCNN_TSP_dense_int3_pyr(**CFG5)
    fill_params(m, seed)
    m.train()
    d = _ref_data(b)
    d.num_node1 = [int(v) for v in b.num_node1]
    d.num_edge1 = [int(v) for v in b.num_edge1]
    out, s_batch = m(d, device="cpu")
    R = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed))
    (out * R).sum().backward()
    _save("baseline_cfg5_tsp", out=_np(out), s_batch=_np(s_batch), R=_np(R),
          seed=np.int64(seed), **_batch_arrays("", b), **_grads(m))


def hl_filter_case(ref, ref_ds, ref_utils, name, kw, seed):
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(5, seed=seed)
    m = ref.HL_filter(**kw)
    fill_params(m, seed)
    m.train()
    gen = torch.Generator().manual_seed(seed)
    x_t = torch.randn(b.x_t.shape[0], kw["node_dim"], generator=gen).requires_grad_(True)
    x_s = torch.randn(b.x_s.shape[0], kw["edge_dim"], generator=gen).requires_grad_(True)
    par = ref_ds.adj2par1(b.edge_index, b.x_t.shape[0], b.x_s.shape[0])
    D = ref_utils.degree(b.edge_index.view(-1), num_nodes=b.x_t.shape[0]) + 1e-6
    y_t, y_s = m(x_t, b.edge_index_t, b.edge_weight_t, x_s, b.edge_index_s, b.edge_weight_s,
                 par, D)
    R_t = torch.randn(y_t.shape, generator=gen)
    R_s = torch.randn(y_s.shape, generator=gen)
    ((y_t * R_t).sum() + (y_s * R_s).sum()).backward()
    _save(name, seed=np.int64(seed), x_t=_np(x_t), x_s=_np(x_s), D=_np(D), out_t=_np(y_t),
          out_s=_np(y_s), R_t=_np(R_t), R_s=_np(R_s), grad_x_t=_np(x_t.grad),
          grad_x_s=_np(x_s.grad), **_batch_arrays("b/", b), **_grads(m))


def sapool_case(ref, ref_ds, ref_utils, seed=13):
    from hlhgat.hodge_dataset import collate
    from hlhgat.synthetic import cifar_like_graphs
    pairs = [cifar_like_graphs(80 + s, n=30, k=5) for s in range(3)]
    b0 = collate([p[0] for p in pairs], check_hodge=True)
    b1 = collate([p[1] for p in pairs], check_hodge=True)
    m = ref.SAPool(**SAPOOL)
    fill_params(m, seed)
    m.train()
    # pos_ts / pos_ss exactly as the reference heads build them
    # (lib/Hodge_ST_Model.py:1031-1038)
    n_batch = torch.cat([torch.tensor([i] * int(n)) for i, n in enumerate(b0.num_node1)])
    s_batch = torch.cat([torch.tensor([i] * int(n)) for i, n in enumerate(b0.num_edge1)])
    n_ahead = torch.cumsum(torch.cat([torch.zeros(1), torch.as_tensor(b1.num_node1).float()]),
                           dim=0, dtype=torch.long)[:-1]
    s_ahead = torch.cumsum(torch.cat([torch.zeros(1), torch.as_tensor(b1.num_edge1).float()]),
                           dim=0, dtype=torch.long)[:-1]
    pos_t = (b0.x_t[:, 0] + n_ahead[n_batch]).view(-1, 1)
    pos_s = (b0.x_s[:, 0] + s_ahead[s_batch]).view(-1, 1)
    gen = torch.Generator().manual_seed(seed)
    x_t = torch.randn(b0.x_t.shape[0], SAPOOL["d"], generator=gen).requires_grad_(True)
    x_s = torch.randn(b0.x_s.shape[0], SAPOOL["d"], generator=gen).requires_grad_(True)
    par = ref_ds.adj2par1(b0.edge_index, b0.x_t.shape[0], b0.x_s.shape[0])
    D = ref_utils.degree(b0.edge_index.view(-1), num_nodes=b0.x_t.shape[0]) + 1e-6
    r = m(x_t, x_s, par, D, [_ref_data(b0), _ref_data(b1)], [pos_t], [pos_s], 0, device="cpu")
    y_t, y_s, _, D1, k, *_, att_t, att_s = r
    Rs = [torch.randn(t.shape, generator=gen) for t in (y_t, y_s, att_t, att_s)]
    sum((t * q).sum() for t, q in zip((y_t, y_s, att_t, att_s), Rs)).backward()
    _save("sapool", seed=np.int64(seed), x_t=_np(x_t), x_s=_np(x_s), D=_np(D), pos_t=_np(pos_t),
          pos_s=_np(pos_s), out_t=_np(y_t), out_s=_np(y_s), att_t=_np(att_t), att_s=_np(att_s),
          D1=_np(D1), k=np.int64(k), R_t=_np(Rs[0]), R_s=_np(Rs[1]), R_at=_np(Rs[2]),
          R_as=_np(Rs[3]), grad_x_t=_np(x_t.grad), grad_x_s=_np(x_s.grad),
          **_batch_arrays("l0/", b0), **_batch_arrays("l1/", b1), **_grads(m))


if __name__ == "__main__":
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    import pyg_standin
    pyg_standin.install()
    sys.path.insert(0, ref_root)
    sys.argv = sys.argv[:1]  # the pepfunc script parses its CLI at import
    import lib.Hodge_Cheb_Conv as ref           # noqa: E402  (reference code)
    import lib.Hodge_Dataset as ref_ds          # noqa: E402
    import lib.Hodge_ST_Model as ref_model      # noqa: E402
    import main_pepfunc_HL_HGCNN_dense_int3_attpool as ref_pep  # noqa: E402
    import torch_geometric.utils as ref_utils   # noqa: E402  (stand-in)
    torch.set_num_threads(1)  # deterministic CPU reduction order

    (c0, c1), (p0, p1), tsp = baseline_batches()
    attpool_case("baseline_cfg3_cifar", ref_model.HL_HGCNN_CIFAR10SP_dense_int3_attpool(**CFG3),
                 3, c0, c1)
    attpool_case("baseline_cfg4_pepfunc", ref_pep.HL_HGCNN_pepfunc_dense_int3_attpool(**CFG4),
                 4, p0, p1)
    tsp_case_baseline(ref_model, tsp)
    hl_filter_case(ref, ref_ds, ref_utils, "hl_filter_dense", HLF_DENSE, 11)
    hl_filter_case(ref, ref_ds, ref_utils, "hl_filter_plain", HLF_PLAIN, 12)
    sapool_case(ref, ref_ds, ref_utils)
