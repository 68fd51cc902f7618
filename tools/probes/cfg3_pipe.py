"""The config-3 overlapped pipeline leg of bench.py on its own
(bench.cifar_pipeline_leg), with the replayed step alone beside it.

    python tools/probes/cfg3_pipe.py [--batches 8] [--cus 0,32,64,128]

One leg per CU count of the producer's stream (0 = unmasked), interleaved
--rounds times.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "hl-hgat_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=8)
    ap.add_argument("--cus", default="")
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--prio", default="", help="comma list of low / high / 0 (unmasked only)")
    args = ap.parse_args()
    import bench
    dev = torch.device("cuda:0")
    c = bench.HEADS["cfg3_cifar_attpool"]
    legs = [(int(v), None) for v in args.cus.split(",")] if args.cus else []
    legs += [(0, p) for p in args.prio.split(",")] if args.prio else []
    for rnd in range(args.rounds):
        for n, pr in legs or [(None, None)]:
            t = time.perf_counter()
            r = bench.cifar_pipeline_leg(dev, c, c["graphs"], n_batches=args.batches,
                                         producer_cus=n, producer_prio=pr)
            r.pop("caps", None)
            r.pop("what", None)
            r["wall_s"] = round(time.perf_counter() - t, 1)
            r["round"] = rnd
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
