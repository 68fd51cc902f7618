"""Golden fixtures for the attention-pooling heads (BASELINE configs 3 and 4)
and for MLGC, generated from the REFERENCE itself.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden_attpool.py [/root/reference]

* mlgc_small.npz: the reference's MLGC (lib/Hodge_Dataset.py:241-297) on three
  small graphs.  torch_cluster (1.6.0, README.md:20) is not installed, so the
  graclus call inside MLGC is answered by hlhgat.hodge_dataset.graclus (our
  restatement of torch_cluster's greedy matching); the fixture therefore pins
  everything in MLGC after the matching (cluster renumbering, edge assignment
  with inf for contracted edges, coarse B1, L0/L1 and their COO), while graclus
  itself stays "parity unpinned" (its labels are stored for the test).
* mlgc_weighted_small.npz: the reference's MLGC_weighted (lib/Hodge_Dataset.py:
  298-353), graclus and PyG's to_undirected(reduce='mean') answered by hlhgat's
  restatements (inputs/outputs of both stored).
* attpool_cifar_small.npz: HL_HGCNN_CIFAR10SP_dense_int3_attpool
  (lib/Hodge_ST_Model.py:958-1091) forward + backward on a 3-graph two-level
  batch of CIFAR-like superpixel graphs.
* attpool_pepfunc_small.npz: HL_HGCNN_pepfunc_dense_int3_attpool
  (main_pepfunc_HL_HGCNN_dense_int3_attpool.py:36-168) on a 2-graph batch of
  peptide-like molecules.

Inputs come from hlhgat's host-side synthetic generators + collate; the models
are the reference's classes run on CPU behind pyg_standin.py.  Outputs are
plain .npz arrays (no pickles).  Nothing from the reference source is copied.
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

from make_golden import _np, _save  # noqa: E402

_KEYS = ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
         "edge_index", "num_node1", "num_edge1")


class _RefData:
    def to(self, device):
        return self


def two_level_batches(pairs):
    from hlhgat.hodge_dataset import collate
    b0 = collate([p[0] for p in pairs], check_hodge=True)
    b1 = collate([p[1] for p in pairs], check_hodge=True)
    return b0, b1


def _ref_datas(b0, b1):
    out = []
    for b in (b0, b1):
        d = _RefData()
        for k in _KEYS:
            setattr(d, k, getattr(b, k))
        d.num_node1 = torch.as_tensor(b.num_node1).view(-1)
        d.num_edge1 = torch.as_tensor(b.num_edge1).view(-1)
        out.append(d)
    return out


def _model_case(name, m, b0, b1, seed):
    m.train()
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    datas = _ref_datas(b0, b1)
    out = m(datas, device="cpu")
    R = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed))
    (out * R).sum().backward()
    arrays = {"out": _np(out), "R": _np(R)}
    for lv, b in enumerate((b0, b1)):
        for k in _KEYS:
            arrays[f"l{lv}/{k}"] = _np(torch.as_tensor(getattr(b, k)))
    for k, v in sd0.items():
        arrays["sd/" + k] = _np(v)
    for k, p in m.named_parameters():
        if p.grad is None:  # unused branch (e.g. NEAtt at pool_loc when if_att is off)
            arrays["nograd/" + k] = np.int8(1)
            continue
        arrays["grad/" + k] = _np(p.grad)
    _save(name, **arrays)


def mlgc_case(ref_ds):
    from hlhgat.hodge_dataset import graclus
    from hlhgat.synthetic import cifar_like_graphs, peptides_like_graphs
    labels = []

    def graclus_standin(row, col, weight, num_nodes):
        lab = graclus(np.stack([_np(row), _np(col)]), int(num_nodes), seed=len(labels))
        labels.append(lab)
        return torch.from_numpy(lab)

    ref_ds.graclus_cluster = graclus_standin
    arrays = {}
    graphs = [cifar_like_graphs(21, n=30, k=5)[0], cifar_like_graphs(22, n=45, k=8)[0],
              peptides_like_graphs(23)[0]]
    for gi, g in enumerate(graphs):
        g.x_t, g.x_s = g.x_t[:, 1:], g.x_s[:, 1:]  # drop the cluster column
        coarse, c_node, c_edge = ref_ds.MLGC(g)
        arrays[f"g{gi}/edge_index"] = _np(g.edge_index)
        arrays[f"g{gi}/edge_index_t"] = _np(g.edge_index_t)
        arrays[f"g{gi}/num_node1"] = np.int64(g.num_node1)
        arrays[f"g{gi}/graclus"] = labels[-1]
        arrays[f"g{gi}/c_node"] = _np(c_node)
        arrays[f"g{gi}/c_edge"] = _np(c_edge)
        for k in ("edge_index", "edge_index_t", "edge_weight_t", "edge_index_s",
                  "edge_weight_s", "x_t", "x_s"):
            arrays[f"g{gi}/coarse/{k}"] = _np(getattr(coarse, k))
        arrays[f"g{gi}/coarse/num_node1"] = np.int64(coarse.num_node1)
    _save("mlgc_small", **arrays)


def mlgc_weighted_case(ref_ds):
    """MLGC_weighted (lib/Hodge_Dataset.py:298-353): torch_cluster's graclus
    and PyG's to_undirected(reduce='mean') are absent, so both calls are
    answered by hlhgat's restatements (their inputs and outputs are stored:
    the edge weights the reference computes, exp(-x_s^2), are pinned; the
    matching is parity unpinned); the map and coarse graph are the
    reference's."""
    from hlhgat.hodge_dataset import graclus, to_undirected_mean
    from hlhgat.synthetic import cifar_like_graphs, peptides_like_graphs
    seen = []

    def to_undirected_standin(edge_index, edge_attr=None, num_nodes=None, reduce="add"):
        assert reduce == "mean"
        n = int(edge_index.max()) + 1 if num_nodes is None else int(num_nodes)
        ei, w = to_undirected_mean(_np(edge_index), _np(edge_attr), n)
        return torch.from_numpy(ei), torch.from_numpy(w)

    def graclus_standin(row, col, weight, num_nodes):
        lab = graclus(np.stack([_np(row), _np(col)]), int(num_nodes), weight=_np(weight),
                      seed=100 + len(seen))
        seen.append((_np(row), _np(col), _np(weight), lab))
        return torch.from_numpy(lab)

    ref_ds.graclus_cluster = graclus_standin
    ref_ds.to_undirected = to_undirected_standin
    arrays = {}
    graphs = [cifar_like_graphs(41, n=30, k=5)[0], cifar_like_graphs(42, n=45, k=8)[0],
              peptides_like_graphs(43)[0]]
    for gi, g in enumerate(graphs):
        g.x_t, g.x_s = g.x_t[:, 1:], g.x_s[:, 1:]  # drop the cluster column
        coarse, c_node, c_edge = ref_ds.MLGC_weighted(g)
        row, col, w, lab = seen[-1]
        arrays[f"g{gi}/edge_index"] = _np(g.edge_index)
        arrays[f"g{gi}/x_s"] = _np(g.x_s)
        arrays[f"g{gi}/num_node1"] = np.int64(g.num_node1)
        arrays[f"g{gi}/graclus_edge_index"] = np.stack([row, col])
        arrays[f"g{gi}/graclus_weight"] = w
        arrays[f"g{gi}/graclus"] = lab
        arrays[f"g{gi}/c_node"] = _np(c_node)
        arrays[f"g{gi}/c_edge"] = _np(c_edge)
        for k in ("edge_index", "edge_index_t", "edge_weight_t", "edge_index_s",
                  "edge_weight_s", "x_t", "x_s"):
            arrays[f"g{gi}/coarse/{k}"] = _np(getattr(coarse, k))
        arrays[f"g{gi}/coarse/num_node1"] = np.int64(coarse.num_node1)
    _save("mlgc_weighted_small", **arrays)


if __name__ == "__main__":
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    import pyg_standin
    pyg_standin.install()
    sys.path.insert(0, ref_root)
    sys.argv = sys.argv[:1]  # the pepfunc script parses its CLI at import
    import lib.Hodge_Dataset as ref_ds          # noqa: E402  (reference code)
    import lib.Hodge_ST_Model as ref_model      # noqa: E402
    import main_pepfunc_HL_HGCNN_dense_int3_attpool as ref_pep  # noqa: E402
    from hlhgat.synthetic import cifar_like_graphs, peptides_like_graphs  # noqa: E402
    torch.set_num_threads(1)  # deterministic CPU reduction order

    mlgc_case(ref_ds)
    mlgc_weighted_case(ref_ds)

    b0, b1 = two_level_batches([cifar_like_graphs(30 + s, n=24, k=5) for s in range(3)])
    torch.manual_seed(5)
    m = ref_model.HL_HGCNN_CIFAR10SP_dense_int3_attpool(
        channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10, pool_loc=0, l=0.5)
    _model_case("attpool_cifar_small", m, b0, b1, seed=9)

    b0, b1 = two_level_batches([peptides_like_graphs(40 + s) for s in range(2)])
    torch.manual_seed(6)
    m = ref_pep.HL_HGCNN_pepfunc_dense_int3_attpool(
        channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)
    _model_case("attpool_pepfunc_small", m, b0, b1, seed=10)
