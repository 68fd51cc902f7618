"""Golden fixtures for the remaining task heads of lib/Hodge_ST_Model.py,
generated from the REFERENCE itself (round 5: VERDICT r4 "missing" #3).

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden_heads.py [/root/reference]

* head_pepfunc_pyr_small.npz: HL_HGCNN_pepfunc_dense_int3_pyr (:307-407)
* head_cifar_pyr_small.npz: HL_HGCNN_CIFAR10SP_dense_int3_pyr (:858-955)
* head_zinc_poolint3_small.npz: HL_HGCNN_zinc_dense_poolint3_pyr (:649-749)
* head_zinc_attpool_small.npz: HL_HGCNN_zinc_dense_int3_attpool (:412-541),
  two MLGC levels of CIFAR-like superpixel graphs
* head_pepfunc_attpool_lib_small.npz: the LIBRARY's
  HL_HGCNN_pepfunc_dense_int3_attpool (:173-304; the training script shadows
  it with its own class, attpool_pepfunc_small.npz), two levels of
  peptide-like molecules

The single-level heads run on ZINC-like molecule batches (the widths are
constructor arguments; the heads' structure does not depend on the dataset).
Forward on CPU behind pyg_standin.py, then the backward of sum(out * R);
inputs, the initial state_dict, outputs and every parameter gradient are
stored as plain .npz arrays (no pickles).  Nothing from the reference source
is copied.
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

from make_golden import _np, _save, small_batch  # noqa: E402
from make_golden_attpool import _model_case, two_level_batches  # noqa: E402

_KEYS = ("x_t", "x_s", "edge_index_t", "edge_weight_t", "edge_index_s", "edge_weight_s",
         "edge_index")


class _RefData:
    pass


def pyr_case(name, m, b, seed):
    m.train()
    d = _RefData()
    for k in _KEYS:
        setattr(d, k, getattr(b, k))
    d.num_node1 = [int(v) for v in b.num_node1]
    d.num_edge1 = [int(v) for v in b.num_edge1]
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    out = m(d, device="cpu")
    assert torch.isfinite(out).all(), name
    R = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed))
    (out * R).sum().backward()
    arrays = {k: _np(getattr(b, k)) for k in _KEYS}
    arrays.update(num_node1=_np(b.num_node1), num_edge1=_np(b.num_edge1), out=_np(out), R=_np(R))
    for k, v in sd0.items():
        arrays["sd/" + k] = _np(v)
    for k, p in m.named_parameters():
        if p.grad is None:
            arrays["nograd/" + k] = np.int8(1)
            continue
        arrays["grad/" + k] = _np(p.grad)
    _save(name, **arrays)


if __name__ == "__main__":
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    import pyg_standin
    pyg_standin.install()
    sys.path.insert(0, ref_root)
    import lib.Hodge_ST_Model as ref_model      # noqa: E402  (reference code)
    from hlhgat.synthetic import cifar_like_graphs, peptides_like_graphs  # noqa: E402
    torch.set_num_threads(1)  # deterministic CPU reduction order

    # ZINC-like widths: node 21 + keig 15, edge 3 + keig 15 (small_batch)
    b = small_batch(6, seed=14)
    torch.manual_seed(21)
    pyr_case("head_pepfunc_pyr_small",
             ref_model.HL_HGCNN_pepfunc_dense_int3_pyr(
                 channels=[1, 1], filters=[16, 16], mlp_channels=[32], K=3, node_dim=21,
                 edge_dim=3, keig=15), b, seed=31)
    torch.manual_seed(22)
    pyr_case("head_cifar_pyr_small",
             ref_model.HL_HGCNN_CIFAR10SP_dense_int3_pyr(
                 channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, node_dim=21,
                 edge_dim=3, keig=15, l=0.5), b, seed=32)
    torch.manual_seed(23)
    pyr_case("head_zinc_poolint3_small",
             ref_model.HL_HGCNN_zinc_dense_poolint3_pyr(
                 channels=[1, 1], filters=[16, 16], mlp_channels=[32], K=3, keig=15),
             b, seed=33)

    # two MLGC levels of CIFAR-like graphs (x_t: cluster column + 5 + keig 10)
    b0, b1 = two_level_batches([cifar_like_graphs(60 + s, n=24, k=5) for s in range(3)])
    torch.manual_seed(24)
    _model_case("head_zinc_attpool_small",
                ref_model.HL_HGCNN_zinc_dense_int3_attpool(
                    channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, node_dim=5,
                    edge_dim=4, keig=10, pool_loc=0), b0, b1, seed=34)

    b0, b1 = two_level_batches([peptides_like_graphs(70 + s) for s in range(2)])
    torch.manual_seed(25)
    _model_case("head_pepfunc_attpool_lib_small",
                ref_model.HL_HGCNN_pepfunc_dense_int3_attpool(
                    channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0),
                b0, b1, seed=35)
