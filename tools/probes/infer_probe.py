"""InferStep probe: the config-2 ZINC eval forward (eval fixture inputs) --
eager vs replayed (chains on / off); max |diff| per replay."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd"), os.path.join(REPO, "tests"),
          os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import hlhgat
    from hlhgat import ops
    from hlhgat.train import InferStep
    import test_eval_mode as TE
    from baseline_params import fill_params
    cuda = torch.device("cuda:0")
    name = "eval_cfg2_zinc"
    g, _, ev = TE._inputs(name, lambda gg, p: TE._product_data(gg, p, cuda))
    bufs = {k[4:]: torch.from_numpy(np.asarray(g[k])) for k in g if k.startswith("buf/")}
    if True:
        for chains in (False, True):
            ops.CHAINS_ENABLED = chains
            m = getattr(hlhgat, TE.CASES[name][1])(**TE.CASES[name][2])
            fill_params(m, int(g["seed"]))
            m.load_state_dict(bufs, strict=False)
            m = m.to(cuda).train()
            inf = InferStep(m)
            outs = [inf(ev).clone() for _ in range(4)]
            torch.cuda.synchronize()
            with torch.no_grad():
                m.eval()
                e2 = m(ev).clone()
                m.train()
            d = [float((o - outs[0]).abs().max()) for o in outs[1:]]
            print(f"chains={chains}: stats {inf.stats} "
                  f"replay-vs-eager {d} eager-vs-eager {float((e2 - outs[0]).abs().max())} "
                  f"vs ref {float((outs[0].cpu() - torch.from_numpy(g['out'])).abs().max()):.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
