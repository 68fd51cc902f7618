"""nei_prepack's packs against the torch construction [Wt | Ws | bt | bs]."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "hl-hgat_amd")]
import torch  # noqa: E402
import hlhgat  # noqa: E402
from hlhgat import ops  # noqa: E402

KW = dict(channels=[1, 1], filters=[32, 32], mlp_channels=[64], K=3, keig=15)
torch.manual_seed(0)
m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(**KW).to("cuda").train()
mods = [m.NEInt00, m.NEInt10]
ops.nei_prepack(mods)
torch.cuda.synchronize()
for mod in mods:
    ep, pk = mod._hlhgat_packed
    Wn, bn = mod.WV_Node[0].weight, mod.WV_Node[0].bias
    We, be = mod.WV_Edge[0].weight, mod.WV_Edge[0].bias
    d = Wn.shape[1] // 2
    Wt = torch.cat([Wn[:, d:], We[:, :d]], 0)
    Ws = torch.cat([We[:, d:], Wn[:, :d]], 0)
    bt = torch.cat([bn, torch.zeros_like(be)])
    bs = torch.cat([be, torch.zeros_like(bn)])
    ref = torch.cat([Wt.reshape(-1), Ws.reshape(-1), bt, bs])
    print("epoch", ep, "numel", pk.numel(), ref.numel(), "maxdiff", float((pk - ref).abs().max()),
          "first bad", int((pk != ref).nonzero()[0]) if bool((pk != ref).any()) else -1, flush=True)

for k in (1, 2):
    ops.nei_prepack(mods[:k])
    torch.cuda.synchronize()
    for mod in mods[:k]:
        ep, pk = mod._hlhgat_packed
        Wn = mod.WV_Node[0].weight
        d = Wn.shape[1] // 2
        print("groups", k, "first row ok", bool(torch.equal(pk[:d], Wn[0, d:])), flush=True)
for n in (4, 8, 9, 16, 40):
    src = [torch.randn(1000 + i, device="cuda") for i in range(n)]
    dst = [torch.empty_like(t) for t in src]
    ops.copy_words_batched(src, dst)
    torch.cuda.synchronize()
    print("copy_words", n, all(torch.equal(a, b) for a, b in zip(src, dst)), flush=True)
