"""The config-3 overlapped pipeline leg of bench.py on its own
(bench.cifar_pipeline_leg), with the replayed step alone beside it.

    python tools/probes/cfg3_pipe.py [--batches 8]
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
    args = ap.parse_args()
    import bench
    dev = torch.device("cuda:0")
    c = bench.HEADS["cfg3_cifar_attpool"]
    t = time.perf_counter()
    r = bench.cifar_pipeline_leg(dev, c, c["graphs"], n_batches=args.batches)
    r.pop("caps", None)
    r.pop("what", None)
    r["wall_s"] = round(time.perf_counter() - t, 1)
    print(json.dumps(r))


if __name__ == "__main__":
    main()
