"""Per-sample data path of BASELINE config 3 (CIFAR10 superpixels, attpool
head), batched and fed to the device.

The reference rebuilds every sample in its Dataset.get() EVERY epoch
(main_cifar10SP_HL_HGCNN_dense_int3_attpool.py:67-125): PyG
to_undirected(reduce='min') and the i<j half of the kNN edges, dropout_edge
augmentation (a quarter of the samples, p = 0.5), the dense B1 and L0 = B1
B1^T, a dense eigh for lambda_max, L0 = 2 B1 B1^T / lmax, L1 = 2 B1^T B1 /
lmax, eig_pe(L0) (lib/Hodge_Dataset.py:97-112: eigenvectors 1..k-1 of an
eigh), edge PE |pe[i] + pe[j]|, the feature concatenations, one MLGC level
(lib/Hodge_Dataset.py:241-295: graclus, the fine -> coarse map, the coarse
graph's own dense eigh and Laplacians), and random sign flips of the PE
columns; then the DataLoader collates the level lists.

SuperpixelPipeline does the same for a whole batch of graphs at once:

  host (numpy, vectorised over the batch): the undirected edge lists (once,
    at construction: they do not change between epochs), the dropout masks,
    graclus + the MLGC map (native, hlhgat_graclus / hlhgat_mlgc_map), the
    offsets of the block-diagonal batch;
  device: the eigenvector PE and lambda_max of every level-0 graph in ONE
    launch (hlhgat_eig_pe: per graph, fp64 Lanczos with full
    re-orthogonalisation, Sturm multisection, inverse iteration; it replaced
    a batched rocSOLVER eigh of the block-padded L0 stack, 3.9 ms and a host
    sync per 256 graphs), the coarse level's lambda_max (hlhgat_hodge_lmax),
    both levels' Hodge Laplacians (hlhgat_hodge_build: the L0 / L1 rows in
    the reference's dense_to_sparse order, sizes known on the host), the
    feature concatenations, the sign flips;

and returns the two level batches on the device, collated, marked sorted /
symmetric and with the factored L1 declared (every L1 the builder emits is
alpha B1^T B1 exactly, alpha = fl(2 / lmax) per graph), ready for the head.
device="cpu" runs the same steps on the host with the reference's own
arithmetic (dense eigh lambda_max, hodge_laplacians) -- the restatement the
golden test pins (tests/golden/make_golden_pipeline.py).

Parity: structure, features, cluster maps and coarse graphs are exact;
lambda_max (fp64 Lanczos vs float32 eigh) within 1e-6 relative, so the
Laplacian entries are; PE columns equal the reference's up to sign (the reference flips them at
random, and an eigenvector's sign is arbitrary), checked where the
eigenvalue is separated from its neighbours.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from .hodge_dataset import (Batch, PairData, _h2d, collate, dense_to_sparse, graclus,
                            hodge_laplacians, mlgc_batch, mlgc_batch_flat, mlgc_map)

__all__ = ["SuperpixelPipeline", "to_undirected_min", "superpixel_raw"]


def to_undirected_min(edge_index, attr, n: int):
    """PyG to_undirected(edge_index, edge_attr, reduce='min') (called at
    main_cifar10SP...:71): both directions, coalesced in (row, col) order,
    duplicates reduced by min.  Returns (int64 [2, E'], float32 [E'])."""
    ei = np.asarray(edge_index, dtype=np.int64)
    a = np.asarray(attr, dtype=np.float32).reshape(-1)
    r = np.concatenate([ei[0], ei[1]])
    c = np.concatenate([ei[1], ei[0]])
    aa = np.concatenate([a, a])
    o = np.lexsort((c, r))
    r, c, aa = r[o], c[o], aa[o]
    first = np.ones(r.size, dtype=bool)
    first[1:] = (r[1:] != r[:-1]) | (c[1:] != c[:-1])
    starts = np.flatnonzero(first)
    return np.stack([r[starts], c[starts]]), np.minimum.reduceat(aa, starts)


def superpixel_raw(seed: int, n: int = 118, k: int = 8):
    """A CIFAR10-superpixel-like raw sample in the layout of PyG's
    GNNBenchmarkDataset('CIFAR10') items: x [n, 3] (mean RGB), pos [n, 2],
    a DIRECTED kNN edge_index [2, n k] with edge_attr [n k] (a distance
    weight), y [1]."""
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(seed)
    pos = rng.random((n, 2)).astype(np.float32)
    dist, nbr = cKDTree(pos).query(pos, k=min(k + 1, n))
    src = np.repeat(np.arange(n), nbr.shape[1] - 1)
    dst = nbr[:, 1:].reshape(-1)
    w = np.exp(-(dist[:, 1:].reshape(-1) / 0.1) ** 2).astype(np.float32)
    d = PairData()
    d.x = torch.from_numpy(rng.random((n, 3)).astype(np.float32))
    d.pos = torch.from_numpy(pos)
    d.edge_index = torch.from_numpy(np.stack([src, dst]).astype(np.int64))
    d.edge_attr = torch.from_numpy(w)
    d.y = torch.tensor([int(rng.integers(10))])
    return d


class SuperpixelPipeline:
    """Config-3 per-sample work for batches of raw superpixel graphs.

    graphs: raw samples (x, pos, edge_index, edge_attr, y; superpixel_raw).
    keig: the dataset's keig (the reference's trainset uses keig + 1 = 11,
      main_cifar10SP...:206; eig_pe is called with k=10 -> 9 PE columns).
    aug: dropout_edge augmentation as the reference's training set."""

    NODE_DIM, EDGE_DIM = 5, 4

    def __init__(self, graphs: Sequence, keig: int = 11, aug: bool = True, pe_k: int = 10):
        self.keig = keig
        self.aug = aug
        self.pe_k = pe_k
        self.n = np.array([int(g.x.shape[0]) for g in graphs], dtype=np.int64)
        self.x = [np.asarray(g.x, dtype=np.float32) for g in graphs]
        self.pos = [np.asarray(g.pos, dtype=np.float32) for g in graphs]
        self.y = [torch.as_tensor(g.y) for g in graphs]
        # to_undirected(reduce='min') + the i<j half (main_cifar10SP...:71-73):
        # fixed per sample, so done once here instead of in every get()
        self.ei, self.attr = [], []
        for g, n in zip(graphs, self.n):
            ei, a = to_undirected_min(g.edge_index, g.edge_attr, int(n))
            keep = ei[0] < ei[1]
            self.ei.append(ei[:, keep])
            self.attr.append(a[keep])
        # the same, concatenated (local node ids), for the vectorised batch gather
        self.m = np.array([e.shape[1] for e in self.ei], dtype=np.int64)
        self.e_off = np.concatenate([[0], np.cumsum(self.m)]).astype(np.int64)
        self.ei_all = (np.concatenate(self.ei, axis=1) if len(self.ei)
                       else np.zeros((2, 0), np.int64))
        self.attr_all = (np.concatenate(self.attr) if len(self.attr)
                         else np.zeros(0, np.float32))
        self.x_all = np.concatenate(self.x) if len(self.x) else np.zeros((0, 3), np.float32)
        self.pos_all = np.concatenate(self.pos) if len(self.pos) else np.zeros((0, 2), np.float32)
        self.n_off = np.concatenate([[0], np.cumsum(self.n)]).astype(np.int64)
        self.y_all = (torch.cat([y.reshape(-1) for y in self.y]) if len(self.y)
                      else torch.zeros(0, dtype=torch.int64))

    def __len__(self) -> int:
        return len(self.n)

    # -- host steps ------------------------------------------------------------
    @staticmethod
    def _segments(starts, lengths):
        """Concatenated index ranges [starts[b], starts[b] + lengths[b])."""
        tot = int(lengths.sum())
        if tot == 0:
            return np.zeros(0, np.int64)
        off = np.concatenate([[0], np.cumsum(lengths)[:-1]])
        return np.repeat(starts - off, lengths) + np.arange(tot, dtype=np.int64)

    def _select(self, idx, rng):
        """The batch's graphs, vectorised over the batch: dropout_edge(p = 0.5)
        on the samples drawn for augmentation (torch.rand(1) > 0.75,
        main_cifar10SP...:74-77), then the kept i<j edges (local node ids),
        their attributes and per-graph edge counts, and graclus's random node
        order per graph (keys drawn once, sorted within each graph)."""
        B = len(idx)
        ns = self.n[idx]
        m = self.m[idx]
        eidx = self._segments(self.e_off[idx], m)
        gid_e = np.repeat(np.arange(B), m)
        if self.aug:
            drop = rng.random(B) > 0.75
            keep = ~drop[gid_e] | (rng.random(eidx.size) >= 0.5)
        else:
            keep = np.ones(eidx.size, dtype=bool)
        eidx, gid_e = eidx[keep], gid_e[keep]
        ei = self.ei_all[:, eidx]
        attr = self.attr_all[eidx]
        E_g = np.bincount(gid_e, minlength=B).astype(np.int64)
        # a random permutation of each graph's nodes: argsort of random keys
        # per row of a [B, nmax] table whose padding keys sort last
        nmax = int(ns.max()) if B else 0
        pad = np.arange(nmax)[None, :] >= ns[:, None]
        keys = rng.random((B, nmax))
        keys[pad] = 2.0
        perm = np.argsort(keys, axis=1)[~pad]
        return ns, ei, attr, E_g, gid_e, perm

    def _pe_signs(self, rng, B, width):
        """The reference's random PE sign flips for B graphs: ones on the first
        columns, +-1 on the last keig - 1 (main_cifar10SP...:113-124)."""
        s = np.ones((B, width), np.float32)
        s[:, width - (self.keig - 1):] = -1 + 2 * rng.integers(0, 2, (B, self.keig - 1))
        return s

    # -- the batch -------------------------------------------------------------
    def batch(self, idx, seed: int = 0, device="cuda", perms=None) -> List[Batch]:
        """[level-0 batch, level-1 batch] of graphs idx.  seed drives the
        augmentation, graclus's node order and the sign flips (perms: an
        explicit graclus node order per graph, e.g. to replay a fixture)."""
        rng = np.random.default_rng(seed)
        idx = np.asarray([int(i) for i in idx], dtype=np.int64)
        self._tick(None)
        ns, ei, attr, E_g, gid_e, perm = self._select(idx, rng)
        if perms is not None:
            perm = np.concatenate([np.asarray(p, np.int64) for p in perms])
        self._tick("dropout + edge lists")
        # MLGC on the host: graclus on L0's pattern (= the edges, both ways; its
        # self-loops are dropped by graclus) with unit weights, the fine -> coarse map
        # (all graphs in one native call on host threads: hlhgat_mlgc_batch)
        mg = mlgc_batch_flat(ei, E_g, ns, perm)
        self._tick("MLGC (native batch)")
        if str(device) == "cpu":
            e_off = np.concatenate([[0], np.cumsum(E_g)])
            eis = [ei[:, e_off[b]:e_off[b + 1]] for b in range(len(idx))]
            attrs = [attr[e_off[b]:e_off[b + 1]] for b in range(len(idx))]
            lv0, lv1 = self._levels_host(idx, eis, attrs, [int(n) for n in ns], mg.per_graph())
        else:
            lv0, lv1 = self._levels_device(idx, ei, attr, ns, E_g, gid_e, mg, torch.device(device))
        # sign flips of the PE columns (after the cluster column is prepended),
        # one row of signs per graph broadcast over its nodes / edges
        B = len(idx)
        sg = np.concatenate([self._pe_signs(rng, B, lv0.x_t.shape[1]),
                             self._pe_signs(rng, B, lv0.x_s.shape[1])], 1)
        sg = _h2d(sg, lv0.x_t.device)
        wt = lv0.x_t.shape[1]
        lv0.x_t.mul_(sg[:, :wt].index_select(0, lv0._gid_t))
        lv0.x_s.mul_(sg[:, wt:].index_select(0, lv0._gid_s))
        del lv0._gid_t, lv0._gid_s
        self._tick("PE sign flips")
        return [lv0, lv1]

    # stage timing (tools/probes/pipeline_stages.py): PROFILE = True makes
    # every stage boundary synchronise the device and accumulate its ms
    PROFILE = False

    def _tick(self, name):
        if not self.PROFILE:
            return
        import time
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
        now = time.perf_counter()
        if name is not None:
            st = self.__dict__.setdefault("stage_ms", {})
            st[name] = st.get(name, 0.0) + (now - self._t0) * 1e3
        self._t0 = now

    def _features(self, i, ei, attr, pe):
        """x_t = [x, pos, pe], x_s = [attr, |x_i - x_j|, |pe_i + pe_j|], each
        zero-padded to the reference's widths (main_cifar10SP...:86-91,
        :113-124; the cluster column is prepended later)."""
        x, pos = self.x[i], self.pos[i]
        node = np.concatenate([x, pos, pe], axis=1)
        edge = np.concatenate([attr.reshape(-1, 1), np.abs(x[ei[0]] - x[ei[1]]),
                               np.abs(pe[ei[0]] + pe[ei[1]])], axis=1)
        return node, edge

    def _pad_width(self, a, width):
        if a.shape[1] < width:
            a = np.concatenate([a, np.zeros((a.shape[0], width - a.shape[1]), a.dtype)], 1)
        return a[:, :width]

    def _levels_host(self, idx, eis, attrs, ns, cmaps):
        """device='cpu': the reference's arithmetic, graph by graph (dense eigh
        for lambda_max and the PE, hodge_laplacians, dense_to_sparse)."""
        from scipy.linalg import eigh
        f0, f1 = [], []
        wt = self.NODE_DIM + self.keig
        ws = self.EDGE_DIM + self.keig
        for i, ei, attr, n, (c_node, c_edge, ei1, n1) in zip(idx, eis, attrs, ns, cmaps):
            L0, L1, _, _ = hodge_laplacians(ei, n)
            vals, vecs = eigh(L0.numpy())
            pe = np.real(vecs[:, vals.argsort()])[:, 1:self.pe_k].astype(np.float32)
            node, edge = self._features(i, ei, attr, pe)
            x_t = self._pad_width(np.concatenate([c_node.reshape(-1, 1).astype(np.float32),
                                                  node], 1), wt)
            x_s = self._pad_width(np.concatenate([c_edge.reshape(-1, 1), edge], 1), ws)
            eit, ewt = dense_to_sparse(L0)
            eis_, ews = dense_to_sparse(L1)
            g = PairData(x_s=torch.from_numpy(x_s), edge_index_s=eis_, edge_weight_s=ews,
                         x_t=torch.from_numpy(x_t), edge_index_t=eit, edge_weight_t=ewt,
                         y=self.y[i])
            g.edge_index = torch.from_numpy(ei)
            g.num_node1, g.num_edge1, g.num_nodes = n, int(ei.shape[1]), n
            g._hodge_sorted = True
            f0.append(g)
            C0, C1, _, _ = hodge_laplacians(ei1, n1)
            eit, ewt = dense_to_sparse(C0)
            eis_, ews = dense_to_sparse(C1)
            c = PairData(x_s=torch.ones(ei1.shape[1], 1), edge_index_s=eis_, edge_weight_s=ews,
                         x_t=torch.ones(n1, 1), edge_index_t=eit, edge_weight_t=ewt)
            c.edge_index = torch.from_numpy(ei1)
            c.num_node1, c.num_edge1, c.num_nodes = n1, int(ei1.shape[1]), n1
            c._hodge_sorted = True
            f1.append(c)
        lv0 = collate(f0, check_hodge=False)
        lv0._gid_t = torch.repeat_interleave(torch.arange(len(f0)), torch.as_tensor(ns))
        lv0._gid_s = torch.repeat_interleave(torch.arange(len(f0)),
                                             torch.as_tensor([e.shape[1] for e in eis]))
        return lv0, collate(f1, check_hodge=False)

    def _levels_device(self, idx, ei, attr, ns, E_g, gid_e, mg, dev):
        """Both levels on the device.  The host arrays travel in two
        asynchronous uploads from pinned memory (one int64, one float32; the
        device tensors are views of them); the Hodge builder gets its sizes from the host (the nnz of L0
        and L1 follow from the degrees), so nothing here waits on the device
        but the eigh's own error check."""
        from . import ops
        B = len(idx)
        N, E = int(ns.sum()), int(ei.shape[1])
        n_off = np.concatenate([[0], np.cumsum(ns)]).astype(np.int64)
        gid_n = np.repeat(np.arange(B), ns)
        ei_b = ei + n_off[gid_e]  # block-diagonal batch (PairData offsets)
        # coarse level: each graph's coarse edges at the head of its edge slot
        n1 = mg.cn
        m1 = mg.cm
        o1 = np.concatenate([[0], np.cumsum(n1)]).astype(np.int64)
        e_off = np.concatenate([[0], np.cumsum(E_g)]).astype(np.int64)
        cidx = self._segments(e_off[:-1], m1)
        gid_c = np.repeat(np.arange(B), m1)
        ei1 = mg.ce[:, cidx] + o1[gid_c]
        N1, E1 = int(o1[-1]), int(ei1.shape[1])
        nodes = self._segments(self.n_off[idx], ns)

        def nnz(e, n):
            # the degree formulas (and the Laplacians themselves) assume a
            # simple graph: unique edges with i < j
            if e.shape[1] and ((e[0] >= e[1]).any() or
                               np.unique(e[0] * n + e[1]).size != e.shape[1]):
                raise ValueError("hlhgat: coarse edges are not unique i < j pairs")
            deg = np.bincount(e.reshape(-1), minlength=n)
            return int((deg > 0).sum()) + 2 * e.shape[1], int((deg * deg).sum()) - e.shape[1]
        ints = [ei_b.reshape(-1), ei1.reshape(-1), ns, E_g, n1, m1,
                self.y_all.numpy()[idx].astype(np.int64), gid_n, gid_e]
        flts = [self.x_all[nodes].reshape(-1), self.pos_all[nodes].reshape(-1), attr,
                mg.c_node.astype(np.float32), mg.c_edge]
        idev = _h2d(np.concatenate(ints), dev)
        fdev = _h2d(np.concatenate(flts), dev)

        def cut(t, sizes):
            out, o = [], 0
            for z in sizes:
                out.append(t[o:o + z])
                o += z
            return out
        ei_d, ei1_d, ns_d, Eg_d, n1_d, m1_d, y_d, gid_d, gide_d = cut(
            idev, [a.size for a in ints])
        ei_d, ei1_d = ei_d.view(2, E), ei1_d.view(2, E1)
        x, pos, attr_d, c_node, c_edge = cut(fdev, [a.size for a in flts])
        x, pos = x.view(N, 3), pos.view(N, 2)
        self._tick("device levels: edge upload")
        # eig_pe and lambda_max of every graph in one launch (hlhgat_eig_pe:
        # fp64 Lanczos with full re-orthogonalisation per graph), then the
        # Hodge Laplacians with that lambda_max
        pe, lam64 = ops.eig_pe(ei_d, ns_d, self.pe_k, max_nodes=int(ns.max()), n_nodes=N)
        self._tick("device levels: eig_pe + lambda_max")
        ei_t, w_t, ei_s, w_s, lam = ops.hodge_build(ei_d, ns_d, lmax=lam64.to(torch.float32),
                                                    sizes=(N,) + nnz(ei_b, N))
        self._tick("device levels: Hodge build (fine)")
        src, dst = ei_d[0], ei_d[1]
        wt, ws = self.NODE_DIM + self.keig, self.EDGE_DIM + self.keig
        k1 = pe.shape[1]
        lv0 = Batch()
        lv0.num_graphs = B
        # x_t = [cluster, x, pos, pe, 0...], x_s = [cluster, attr, |x_i - x_j|,
        # |pe_i + pe_j|, 0...] written straight into their padded widths
        xt = torch.zeros(N, wt, device=dev)
        xt[:, 0] = c_node
        xt[:, 1:4] = x
        xt[:, 4:6] = pos
        xt[:, 6:6 + k1] = pe[:, :wt - 6]
        xs = torch.zeros(E, ws, device=dev)
        xs[:, 0] = c_edge
        xs[:, 1] = attr_d
        xs[:, 2:5] = (x[src] - x[dst]).abs()
        xs[:, 5:5 + k1] = (pe[src] + pe[dst]).abs()[:, :ws - 5]
        lv0.x_t, lv0.x_s = xt, xs
        lv0.edge_index_t, lv0.edge_weight_t = ei_t, w_t
        lv0.edge_index_s, lv0.edge_weight_s = ei_s, w_s
        lv0.edge_index = ei_d
        lv0.y = y_d
        # per-graph counts on the device, as Batch.to leaves them (the step's
        # forward reads them inside a capture)
        lv0.num_node1, lv0.num_edge1 = ns_d, Eg_d
        lv0.num_nodes = N
        lv0._gid_t, lv0._gid_s = gid_d, gide_d
        self._tick("device levels: features")
        c_t, c_wt, c_s, c_ws, _ = ops.hodge_build(ei1_d, n1_d, sizes=(N1,) + nnz(ei1, N1))
        self._tick("device levels: Hodge build (coarse)")
        lv1 = Batch()
        lv1.num_graphs = B
        lv1.x_t = torch.ones(N1, 1, device=dev)
        lv1.x_s = torch.ones(E1, 1, device=dev)
        lv1.edge_index_t, lv1.edge_weight_t = c_t, c_wt
        lv1.edge_index_s, lv1.edge_weight_s = c_s, c_ws
        lv1.edge_index = ei1_d
        lv1.num_node1, lv1.num_edge1 = n1_d, m1_d
        lv1.num_nodes = N1
        for lv in (lv0, lv1):
            lv.hodge_sorted = {"edge_index_s": True, "edge_index_t": True}
            lv.l1_factor = False
            lv._mark()
        # every L1 of the builder is fl(2 / lmax) B1^T B1 exactly (entries
        # fl(fl(2 v) / lmax), v in {2, +-1}): the factored L1 holds by
        # construction -- declared where it pays (hodge_dataset.FACTOR_MIN_ROW)
        from .hodge_dataset import FACTOR_MIN_ROW
        if ei_s.shape[1] >= FACTOR_MIN_ROW * max(E, 1):
            ops.set_hodge_factor(lv0.edge_index_s, lv0.edge_index, lv0.num_nodes)
            lv0.l1_factor = True
        return lv0, lv1
