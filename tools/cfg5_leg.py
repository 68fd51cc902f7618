"""Run only bench.py's config-5 SpMM roofline leg (plain / halo / factored)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "hl-hgat_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.cfg5_spmm(torch.device("cuda:0"))), flush=True)
