"""Which setting trips the one-launch BatchNorm barrier timeout in the
config-3 head (bench.heads_leg's loop): eager + replayed CIFAR attpool steps
with the produced-row BN / BN-backward fold on or off; reports the device
error word after each.

    python tools/probes/heads_bn_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    import bench
    import hlhgat
    from hlhgat import _lib, ops
    from hlhgat.hodge_dataset import level_caps, pad_levels
    from hlhgat.synthetic import two_level_batch
    from hlhgat.train import TrainStep
    dev = torch.device("cuda:0")
    c = bench.HEADS["cfg3_cifar_attpool"]
    raw = [two_level_batch("cifar", c["graphs"], seed=s) for s in range(4)]
    caps = level_caps(raw, 512)
    batches = [[x.to(dev) for x in pad_levels(b, caps)] for b in raw]
    out = {}
    for name, prod, fold in (("off", 0, False), ("prod", 1, False), ("fold", 0, True),
                             ("off2", 0, False)):
        _lib.LIB.hlhgat_set_bn_produced(prod)
        ops._ext.set_bn_fold(fold)
        res = {}
        for graphs in (False, True):
            ops.clear_device_errors()
            torch.manual_seed(0)
            m = getattr(hlhgat, c["cls"])(**c["kw"]).to(dev).train()
            st = TrainStep(m, lambda o, d: bench._head_loss("cifar", o, d), lr=1e-3,
                           graphs=graphs)
            for i in range(6):
                try:
                    st(batches[i % 4])
                except RuntimeError as e:
                    res[str(graphs)] = f"step {i}: {str(e)[:80]}"
                    break
            torch.cuda.synchronize()
            res.setdefault(str(graphs), "ok" if ops.device_errors() == 0 else
                           f"error word {ops.device_errors()}")
        out[name] = res
        print(json.dumps({name: res}), flush=True)
    _lib.LIB.hlhgat_set_bn_produced(0)
    ops._ext.set_bn_fold(False)


if __name__ == "__main__":
    main()
