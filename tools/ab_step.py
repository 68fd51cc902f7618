"""Same-process A/B of the replayed config-2 training step (bench.py's
workload): each variant builds its own model + TrainStep (one capture), then
the variants are timed in interleaved rounds so box-to-box spread cancels.

    python tools/ab_step.py base nochain nochainbwd nofusedbn [--rounds 6] [--steps 20]

Variants (A/B hooks, not product settings):
  base        the defaults
  nochain     ops.CHAINS_ENABLED = False (a fork / join per HL block)
  nochainbwd  chain-mode forward, the NodeEdgeInt backward with its own fork / join
  nofusedbn   projection and BatchNorm forward as two launches
  norows      Linear backward data gradient per (row block, column tile)
  sync        the edge chain waits for main after HL_init_conv (collate tables)
  nomlp2      the readout MLP module by module (no two-layer fused node)
  noreadside  the edge readout mean on the main stream
  noreserve   BatchNorm workspaces not reserved before the capture
  twolaunchbn the BatchNorm forward as statistics + apply launches everywhere
  splitbn     projection + BatchNorm as the projection with a statistics epilogue
              (no wait) + the apply launch
  nobarrier   twolaunchbn + splitbn: no kernel of the step waits for another workgroup
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def set_variant(name, on):
    from hlhgat import ops, _lib
    name = name.rstrip("0123456789")  # base1, base2: repeats of one variant
    ops.CHAINS_ENABLED = not (on and name == "nochain")
    ops._ext.set_chain_bwd(not (on and name == "nochainbwd"))
    _lib.LIB.hlhgat_set_proj_bn_fused(0 if (on and name == "nofusedbn") else 1)
    _lib.LIB.hlhgat_set_proj_bwd_rows(0 if (on and name == "norows") else 1)
    _lib.LIB.hlhgat_set_bn_one_launch(0 if (on and name in ("twolaunchbn", "nobarrier")) else 1)
    _lib.LIB.hlhgat_set_proj_bn_split(1 if (on and name in ("splitbn", "nobarrier")) else 0)
    from hlhgat import nn as hnn, hodge_st_model, train
    hnn.MLP_PAIRS = not (on and name == "nomlp2")
    hodge_st_model.READOUT_ON_CHAIN = not (on and name == "noreadside")
    hodge_st_model.SYNC_SIDE_ALWAYS = on and name == "sync"
    train.BN_RESERVE_CHANNELS = 0 if (on and name == "noreserve") else 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import bench
    import hlhgat
    from hlhgat.train import TrainStep
    dev = torch.device("cuda:0")
    batches, caps, _, _, _ = bench.make_batches(4, 0, dev)
    crit = hlhgat.nn.L1Loss()
    steps = {}
    for v in args.variants:
        set_variant(v, True)
        torch.manual_seed(0)
        m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**bench.MODEL_KW).to(dev).train()
        st = TrainStep(m, lambda o, b: crit(o.view(-1, 1), b.y.view(-1, 1)), lr=1e-3,
                       weight_decay=1e-3, graphs=True)
        for i in range(6):
            st(batches[i % len(batches)])
        torch.cuda.synchronize()
        set_variant(v, False)
        steps[v] = st
    res = {v: [] for v in args.variants}
    for r in range(args.rounds):
        for v in args.variants:
            st = steps[v]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                st(batches[i % len(batches)])
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / args.steps * 1e3)
    from hlhgat import ops as _ops
    _ops.check_device_errors()  # a timed-out wait / barrier voids the A/B
    out = {v: {"ms_median": sorted(x)[len(x) // 2], "ms_min": min(x),
               "ms": [round(t, 4) for t in x]} for v, x in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
