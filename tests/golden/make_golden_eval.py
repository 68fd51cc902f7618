"""Eval-mode golden fixtures generated from the REFERENCE itself.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_golden_eval.py [/root/reference]

The reference's test() loop (main_zinc_HL_HGCNN_dense_int3_pyr.py:165-177)
runs model.eval() under torch.no_grad(): every BatchNorm then normalises with
its running statistics, a different route from training.  For each BASELINE
head this script

  1. overwrites every parameter with baseline_params.fill_params(model, seed);
  2. runs a few TRAINING-mode forwards under no_grad (the running statistics
     move away from their reset values, momentum 0.1);
  3. switches to eval() and runs one forward under no_grad;

and stores the eval output and every BatchNorm buffer after step 2.

* eval_cfg2_zinc.npz: HL_HGCNN_zinc_dense_int3_pyr at config 2's settings
  (channels [2,2,2], filters [64,64,64], mlp [256,256], K=3, keig=15) on
  three 12-graph ZINC-like training batches and a 10-graph eval batch (stored).
* eval_cfg3_cifar / eval_cfg4_pepfunc / eval_cfg5_tsp.npz: the heads of
  make_golden_baseline.py on that script's inputs (the baseline_cfg*.npz
  fixtures hold them), two training passes then eval on the same batch.

Plain .npz, no pickles; nothing from the reference source is copied.
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

from baseline_params import fill_params  # noqa: E402
from make_golden import _np, _save, small_batch  # noqa: E402
from make_golden_baseline import CFG3, CFG4, CFG5, KEYS, _batch_arrays  # noqa: E402

# config 2 (BASELINE configs[1]) and the eval fixture's batches
CFG2 = dict(channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[256, 256], K=3, keig=15)
ZINC_SEED = 2
ZINC_TRAIN = [(12, 31), (12, 32), (12, 33)]  # (graphs, seed) of the training passes
ZINC_EVAL = (10, 34)
HEAD_TRAIN_PASSES = 2


class _RefData:
    def to(self, device):
        return self


def ref_data(b, as_list=False):
    d = _RefData()
    for k in KEYS:
        setattr(d, k, getattr(b, k))
    if as_list:
        d.num_node1 = [int(v) for v in b.num_node1]
        d.num_edge1 = [int(v) for v in b.num_edge1]
    else:
        d.num_node1 = torch.as_tensor(b.num_node1).view(-1)
        d.num_edge1 = torch.as_tensor(b.num_edge1).view(-1)
    return d


def bn_buffers(m):
    """Every BatchNorm buffer (running_mean / running_var / num_batches_tracked)."""
    out = {}
    for k, v in m.state_dict().items():
        if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
            out["buf/" + k] = _np(v)
    return out


def zinc_eval_case(ref_model):
    m = ref_model.HL_HGCNN_zinc_dense_int3_pyr(**CFG2)
    fill_params(m, ZINC_SEED)
    arrays = {}
    m.train()
    with torch.no_grad():
        for i, (n, seed) in enumerate(ZINC_TRAIN):
            b = small_batch(n, seed)
            m(ref_data(b, as_list=True), device="cpu")
            arrays.update(_batch_arrays(f"train{i}/", b))
    bufs = bn_buffers(m)
    m.eval()
    be = small_batch(*ZINC_EVAL)
    with torch.no_grad():
        out = m(ref_data(be, as_list=True), device="cpu")
    _save("eval_cfg2_zinc", out=_np(out), seed=np.int64(ZINC_SEED),
          n_train=np.int64(len(ZINC_TRAIN)), **_batch_arrays("eval/", be), **arrays, **bufs)


def head_eval_case(name, m, seed, datas, tsp=False):
    fill_params(m, seed)
    m.train()
    with torch.no_grad():
        for _ in range(HEAD_TRAIN_PASSES):
            m(datas, device="cpu")
    bufs = bn_buffers(m)
    m.eval()
    with torch.no_grad():
        out = m(datas, device="cpu")
    if tsp:
        out = out[0]
    _save(name, out=_np(out), seed=np.int64(seed), n_train=np.int64(HEAD_TRAIN_PASSES), **bufs)


if __name__ == "__main__":
    ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    import pyg_standin
    pyg_standin.install()
    sys.path.insert(0, ref_root)
    sys.argv = sys.argv[:1]  # the pepfunc script parses its CLI at import
    import lib.Hodge_ST_Model as ref_model      # noqa: E402  (reference code)
    import main_pepfunc_HL_HGCNN_dense_int3_attpool as ref_pep  # noqa: E402
    from make_golden_baseline import baseline_batches  # noqa: E402
    torch.set_num_threads(1)  # deterministic CPU reduction order

    zinc_eval_case(ref_model)
    (c0, c1), (p0, p1), tsp = baseline_batches()
    head_eval_case("eval_cfg3_cifar", ref_model.HL_HGCNN_CIFAR10SP_dense_int3_attpool(**CFG3), 3,
                   [ref_data(c0), ref_data(c1)])
    head_eval_case("eval_cfg4_pepfunc", ref_pep.HL_HGCNN_pepfunc_dense_int3_attpool(**CFG4), 4,
                   [ref_data(p0), ref_data(p1)])
    head_eval_case("eval_cfg5_tsp", ref_model.HL_HGCNN_TSP_dense_int3_pyr(**CFG5), 5,
                   ref_data(tsp, as_list=True), tsp=True)
