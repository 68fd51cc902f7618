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

import queue
import threading
from collections import deque
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, Iterable, Iterator, List, Optional

import numpy as np

from .hodge_dataset import Batch, PackedGraphs

__all__ = ["GraphLoader", "StagedFeed"]


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


    def stream(self, epochs: Optional[int] = None) -> Iterator[Batch]:
        """Batches of `epochs` consecutive epochs (None = without end) from ONE
        pool of collation threads whose prefetch runs across epoch boundaries
        -- iterating the loader once per epoch restarts the pipeline (a fresh
        pool and an empty prefetch queue) every epoch, and the consumer then
        waits for the first batch's collation.  Each epoch has its own order
        and capacity bucket, as __iter__."""
        def jobs():
            e = 0
            while epochs is None or e < epochs:
                idxs = self.batch_indices(self.epoch)
                caps = self.epoch_caps(idxs)
                self.epoch += 1
                e += 1
                for i in idxs:
                    yield i, caps
        with ThreadPoolExecutor(self.workers, thread_name_prefix="hlhgat-collate") as ex:
            pending = deque()
            it = jobs()
            for i, caps in it:
                pending.append(ex.submit(self.dataset.collate, i, caps, self.pin))
                if len(pending) >= self.prefetch:
                    break
            while pending:
                b = pending.popleft().result()
                nxt = next(it, None)
                if nxt is not None:
                    pending.append(ex.submit(self.dataset.collate, nxt[0], nxt[1], self.pin))
                yield b


class StagedFeed:
    """The host side of the training loop off the thread that launches the
    steps: a feeder thread takes collated batches from ``batches`` (e.g. a
    GraphLoader, whose own threads collate ahead) and uploads each with
    ``step.stage(batch, stream)`` -- on a copy stream, straight into the
    static buffers of a captured graph of the batch's shape -- at most
    ``depth`` batches ahead of the step; iterating yields the staged handles
    in order, each to be passed to ``step(...)`` before the next is taken.

        feed = StagedFeed(loader, step, depth=2)   # step = TrainStep(..., stage_slots=4)
        for st in feed:
            loss = step(st)

    The replay call releases the GIL, so the feeder's Python work and the
    copies' enqueueing overlap the launch thread's.  ``step.stage_slots``
    must be >= depth + 1 (depth staged batches waiting + one replaying);
    with fewer, a staged batch goes to fresh device tensors and is copied in
    at its step (correct, one device copy more).  depth + 2 is better: the
    feeder waits on the host for the slot's previous replay to finish
    (train.STAGE_WAIT), and one slot more makes that replay an older one.
    ``thread=False`` stages from the consumer's own thread instead (no
    feeder thread; it then also does those waits).  The reference loop this
    serves: main_zinc_HL_HGCNN_dense_int3_pyr.py:151-162 (for data in
    loader: data.to(device); step), with DataLoader(num_workers=4) (:223-225).
    """

    _END = object()

    def __init__(self, batches: Iterable, step, depth: int = 2, stream=None,
                 thread: bool = True):
        import torch
        if depth < 1:
            raise ValueError("StagedFeed: depth must be >= 1")
        self.batches = batches
        self.step = step
        self.depth = int(depth)
        if stream is None:
            from . import ops
            stream = ops.own_stream(step.device, "copy")
        self.stream = stream
        self._q: "queue.Queue" = queue.Queue()
        self._room = threading.Semaphore(self.depth)
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.use_thread = bool(thread)
        self.timing = {"source": 0.0, "room": 0.0, "stage": 0.0, "n": 0}
        self._last = None  # the handle last handed to the consumer (maybe not stepped)

    def _run(self):
        import time
        it = iter(self.batches)
        clock = time.perf_counter
        try:
            t0 = clock()
            for b in it:
                t1 = clock()
                while not self._room.acquire(timeout=0.1):
                    if self._stop.is_set():
                        return
                if self._stop.is_set():
                    return
                t2 = clock()
                st = self.step.stage(b, self.stream)
                t3 = clock()
                self._q.put(st)
                # feeder time per batch: waiting for the source, for room
                # (the consumer), in stage() (diagnostics, bench loader leg)
                self.timing["source"] += t1 - t0
                self.timing["room"] += t2 - t1
                self.timing["stage"] += t3 - t2
                self.timing["n"] += 1
                t0 = clock()
            self._q.put(self._END)
        except BaseException as e:  # handed to the consumer
            self._q.put(e)
        finally:
            close = getattr(it, "close", None)  # stop a generator source's own workers
            if close is not None:
                close()

    def _inline(self):
        # thread=False: the consumer's own thread stages `depth` batches ahead
        # (between its step calls) -- no second Python thread contending for
        # the GIL with the training loop
        import time
        clock = time.perf_counter
        it = iter(self.batches)
        ahead = deque()
        try:
            while True:
                while len(ahead) < self.depth:
                    t0 = clock()
                    b = next(it, self._END)
                    if b is self._END:
                        break
                    t1 = clock()
                    ahead.append(self.step.stage(b, self.stream))
                    t2 = clock()
                    self.timing["source"] += t1 - t0
                    self.timing["stage"] += t2 - t1
                    self.timing["n"] += 1
                if not ahead:
                    return
                self._last = ahead.popleft()
                yield self._last
        finally:
            # a feed closed early: give back what was staged but not stepped
            for st in ahead:
                self.step.unstage(st)
            self._unstage_last()
            close = getattr(it, "close", None)
            if close is not None:
                close()

    def __iter__(self):
        if not self.use_thread:
            yield from self._inline()
            return
        self._stop.clear()
        self._thread = threading.Thread(target=self._run, name="hlhgat-stage", daemon=True)
        self._thread.start()
        try:
            while True:
                item = self._q.get()
                if item is self._END:
                    return
                if isinstance(item, BaseException):
                    raise item
                self._last = item
                yield item
                self._room.release()  # the consumer has stepped it: room for one more
        finally:
            self.close()

    def _unstage_last(self):
        st, self._last = self._last, None
        if st is not None:
            self.step.unstage(st)  # a no-op when the consumer stepped it

    def close(self):
        """Stop the feeder and give back every batch it staged that was not
        stepped (TrainStep.unstage): the ones queued for the consumer, and the
        one last handed out if the consumer left before stepping it."""
        self._stop.set()
        t, self._thread = self._thread, None
        if t is not None and t is not threading.current_thread():
            # unblock a feeder waiting for room, then let it finish its batch
            self._room.release()
            t.join(timeout=30)
            if t.is_alive():
                return  # still inside stage(): its handle cannot be reclaimed yet
        while True:
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                break
            if item is not self._END and not isinstance(item, BaseException):
                self.step.unstage(item)
        self._unstage_last()
