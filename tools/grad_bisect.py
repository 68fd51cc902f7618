"""Locate where a head's backward departs from the fp64 oracle: every
NEInt / NEConv / NEAtt / HL_init_conv submodule's OUTPUT gradient (and output)
of the HIP head vs the fp64 oracle, max-norm relative, in forward order.
usage: grad_bisect.py [cifar|pepfunc|tsp]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402
import test_baseline_configs as TB  # noqa: E402
from conftest import load_golden  # noqa: E402

torch.set_num_threads(16)
cuda = torch.device("cuda:0")
which = sys.argv[1] if len(sys.argv) > 1 else "pepfunc"
name = [n for n in TB.HEADS if which in n][0]
g = load_golden(name)


def instrument(m, store):
    for mn, mod in m.named_children():
        if not any(mn.startswith(p) for p in ("NEInt", "NEConv", "NEAtt", "HL_init")):
            continue

        def wrap(fwd, mn=mn):
            def f(*a, **k):
                out = fwd(*a, **k)
                outs = out if isinstance(out, (tuple, list)) else [out]
                for i, t in enumerate(outs):
                    if torch.is_tensor(t) and t.requires_grad:
                        t.retain_grad()
                        store.append((f"{mn}[{i}]", t))
                return out
            return f
        mod.forward = wrap(mod.forward)


import hlhgat  # noqa: E402
_, cls_name, kw = TB.HEADS[name]
m = getattr(hlhgat, cls_name)(**kw)
TB.fill_params(m, int(g["seed"]))
m = m.to(cuda).train()
sh = []
instrument(m, sh)
if "tsp" in name:
    out, _ = m(TB._product_batch(g, "", cuda, False))
else:
    out = m([TB._product_batch(g, "l0/", cuda, False), TB._product_batch(g, "l1/", cuda, False)])
(out * TB.T(g["R"]).to(cuda)).sum().backward()

cls_o, _, kw = TB.HEADS[name]
mo = getattr(TB.R, cls_o)(**kw)
TB.fill_params(mo, int(g["seed"]))
mo = mo.double().train()
so = []
instrument(mo, so)
if "tsp" in name:
    oo, _ = mo(TB._data(g, "", torch.float64))
else:
    oo = mo([TB._data(g, "l0/", torch.float64), TB._data(g, "l1/", torch.float64)])
(oo * TB.T(g["R"]).double()).sum().backward()

do = dict(so)
for k, t in sh:
    r = do.get(k)
    if r is None or t.grad is None or r.grad is None:
        print(k, "missing")
        continue
    sc = max(1e-30, float(r.grad.abs().max()))
    ev = float((t.detach().cpu().double() - r.detach()).abs().max()) / max(1.0, float(r.abs().max()))
    eg = float((t.grad.cpu().double() - r.grad).abs().max()) / sc
    print(f"{k:20s} value {ev:.2e}  grad {eg:.2e}  |grad| {sc:.2e}", flush=True)
