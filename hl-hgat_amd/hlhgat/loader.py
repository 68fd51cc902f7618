"""Native-collate data loader for packed simplex-graph datasets.

The reference feeds every training step from a torch_geometric DataLoader
(main_zinc_HL_HGCNN_dense_int3_pyr.py:223-225: batch_size 128, num_workers
4) whose workers collate PairData in Python (lib/Hodge_Dataset.py:40-48),
and the loop copies the batch to the device (:155).  At the throughput of the
replayed MI355X step (~350k graphs/s at 1000 graphs per step) a Python
collate (~50 ms per 1000 graphs on one core) would need ~15 workers.

GraphLoader instead collates with ONE native call per batch
(PackedGraphs.collate -> hlhgat_collate, csrc/collate.hip: the padded batch
and its CSR / incidence / degree / segment tables, ~2-3 ms per 1000 ZINC
graphs on one core).  The call releases the GIL (ctypes), so a few worker
THREADS prefetch batches in order, into pinned host memory when asked, and
TrainStep copies each into its captured step's static buffers.
"""
from __future__ import annotations

from collections import deque
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterator, List, Optional

import numpy as np

from .hodge_dataset import Batch, PackedGraphs

__all__ = ["GraphLoader"]


class GraphLoader:
    """Batches of ``batch_size`` graphs of a PackedGraphs dataset.

    caps: the capacity bucket every batch is padded to (hodge_dataset
      static_caps keys), so that every batch replays one captured step;
      None = the largest caps_for() of the epoch's batches (one bucket per
      epoch), False = no padding.
    shuffle: a new permutation per epoch (numpy RandomState(seed + epoch)).
    workers / prefetch: collation threads and batches kept in flight.
    pin: batches in pinned host memory (needs a ROCm device)."""

    def __init__(self, dataset: PackedGraphs, batch_size: int, caps=None, shuffle: bool = False,
                 drop_last: bool = True, workers: int = 2, prefetch: int = 4, pin: bool = False,
                 seed: int = 0, quantum: int = 512):
        if batch_size < 1 or workers < 1 or prefetch < 1:
            raise ValueError("GraphLoader: batch_size, workers and prefetch must be >= 1")
        self.dataset = dataset
        self.batch_size = int(batch_size)
        self.caps = caps
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.workers = int(workers)
        self.prefetch = int(prefetch)
        self.pin = pin
        self.seed = seed
        self.quantum = quantum
        self.epoch = 0

    def batch_indices(self, epoch: int) -> List[np.ndarray]:
        n = len(self.dataset)
        order = (np.random.RandomState(self.seed + epoch).permutation(n) if self.shuffle
                 else np.arange(n))
        bs = self.batch_size
        stop = n - n % bs if self.drop_last else n
        return [order[i:i + bs] for i in range(0, stop, bs)]

    def epoch_caps(self, idxs: List[np.ndarray]) -> Optional[Dict[str, int]]:
        if self.caps is False:
            return None
        if isinstance(self.caps, dict):
            return self.caps
        cs = [self.dataset.caps_for(i, self.quantum) for i in idxs]
        return {k: max(c[k] for c in cs) for k in cs[0]} if cs else None

    def __len__(self) -> int:
        n, bs = len(self.dataset), self.batch_size
        return n // bs if self.drop_last else -(-n // bs)

    def __iter__(self) -> Iterator[Batch]:
        idxs = self.batch_indices(self.epoch)
        caps = self.epoch_caps(idxs)
        self.epoch += 1
        with ThreadPoolExecutor(self.workers, thread_name_prefix="hlhgat-collate") as ex:
            pending = deque()
            it = iter(idxs)
            for i in it:
                pending.append(ex.submit(self.dataset.collate, i, caps, self.pin))
                if len(pending) >= self.prefetch:
                    break
            while pending:
                b = pending.popleft().result()
                nxt = next(it, None)
                if nxt is not None:
                    pending.append(ex.submit(self.dataset.collate, nxt, caps, self.pin))
                yield b
