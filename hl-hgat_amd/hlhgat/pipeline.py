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
  device: both levels' Hodge Laplacians and lambda_max for every graph in
    two launches each (hlhgat_hodge_lmax: fp64 Lanczos, one workgroup per
    graph; hlhgat_hodge_build: the L0 / L1 rows in the reference's
    dense_to_sparse order), the eigenvector PE as ONE batched dense eigh of
    the block-padded L0 stack (rocSOLVER through torch.linalg.eigh), the
    feature concatenations, the sign flips;

and returns the two level batches on the device, collated, marked sorted /
symmetric and with the factored L1 declared (every L1 the builder emits is
alpha B1^T B1 exactly, alpha = fl(2 / lmax) per graph), ready for the head.
device="cpu" runs the same steps on the host with the reference's own
arithmetic (dense eigh lambda_max, hodge_laplacians) -- the restatement the
golden test pins (tests/golden/make_golden_pipeline.py).

Parity: structure, features, cluster maps and coarse graphs are exact;
lambda_max (Lanczos vs eigh) within 1e-6 relative, so the Laplacian entries
are; PE columns equal the reference's up to sign (the reference flips them at
random, and an eigenvector's sign is arbitrary), checked where the
eigenvalue is separated from its neighbours.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from .hodge_dataset import (Batch, PairData, collate, dense_to_sparse, graclus, hodge_laplacians,
                            mlgc_batch, mlgc_map)

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

    def __len__(self) -> int:
        return len(self.n)

    # -- host steps ------------------------------------------------------------
    def _dropout(self, idx, rng) -> List[np.ndarray]:
        """Edge keep-masks: dropout_edge(p=0.5) on the samples drawn for
        augmentation (torch.rand(1) > 0.75, main_cifar10SP...:74-77)."""
        masks = []
        for i in idx:
            E = self.ei[i].shape[1]
            if self.aug and rng.random() > 0.75:
                masks.append(rng.random(E) >= 0.5)
            else:
                masks.append(np.ones(E, dtype=bool))
        return masks

    def _pe_sign(self, rng, width):
        """The reference's random PE sign flips: ones on the first columns,
        +-1 on the last keig - 1 (main_cifar10SP...:113-124)."""
        return np.concatenate([np.ones(width - (self.keig - 1), np.float32),
                               (-1 + 2 * rng.integers(0, 2, self.keig - 1)).astype(np.float32)])

    # -- the batch -------------------------------------------------------------
    def batch(self, idx, seed: int = 0, device="cuda", perms=None) -> List[Batch]:
        """[level-0 batch, level-1 batch] of graphs idx.  seed drives the
        augmentation, graclus's node order and the sign flips (perms: an
        explicit graclus node order per graph, e.g. to replay a fixture)."""
        rng = np.random.default_rng(seed)
        idx = [int(i) for i in idx]
        masks = self._dropout(idx, rng)
        eis = [self.ei[i][:, m] for i, m in zip(idx, masks)]
        attrs = [self.attr[i][m] for i, m in zip(idx, masks)]
        ns = [int(self.n[i]) for i in idx]
        # MLGC on the host: graclus on L0's pattern (= the edges, both ways; its
        # self-loops are dropped by graclus) with unit weights, the fine -> coarse map
        # (all graphs in one native call on host threads: hlhgat_mlgc_batch)
        pl = [perms[b] if perms is not None else rng.permutation(n) for b, n in enumerate(ns)]
        cmaps = mlgc_batch(eis, ns, pl)
        if str(device) == "cpu":
            lv0, lv1 = self._levels_host(idx, eis, attrs, ns, cmaps)
        else:
            lv0, lv1 = self._levels_device(idx, eis, attrs, ns, cmaps, torch.device(device))
        # sign flips of the PE columns (after the cluster column is prepended)
        st = torch.from_numpy(np.stack([self._pe_sign(rng, lv0.x_t.shape[1]) for _ in idx]))
        ss = torch.from_numpy(np.stack([self._pe_sign(rng, lv0.x_s.shape[1]) for _ in idx]))
        nt = torch.as_tensor(lv0.num_node1).to(lv0.x_t.device)
        ne = torch.as_tensor(lv0.num_edge1).to(lv0.x_t.device)
        lv0.x_t = lv0.x_t * torch.repeat_interleave(st.to(lv0.x_t.device), nt, dim=0,
                                                    output_size=lv0.x_t.shape[0])
        lv0.x_s = lv0.x_s * torch.repeat_interleave(ss.to(lv0.x_t.device), ne, dim=0,
                                                    output_size=lv0.x_s.shape[0])
        return [lv0, lv1]

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
        return collate(f0, check_hodge=False), collate(f1, check_hodge=False)

    def _levels_device(self, idx, eis, attrs, ns, cmaps, dev):
        from . import ops
        B = len(idx)
        n_off = np.concatenate([[0], np.cumsum(ns)])
        ei_b = np.ascontiguousarray(np.concatenate([e + o for e, o in zip(eis, n_off[:-1])], axis=1))
        E_g = [int(e.shape[1]) for e in eis]
        ei_d = torch.from_numpy(ei_b).to(dev)
        ei_t, w_t, ei_s, w_s, lam = ops.hodge_build(ei_d, ns)
        # eig_pe on the device: ONE batched eigh of the block-padded L0 stack
        # (padding rows / columns carry a diagonal above every real eigenvalue,
        # so each graph's smallest eigenpairs are its own, with zero padding)
        nmax = max(ns)
        big = 10.0  # > lambda(L0) <= 2 after the 2 / lmax scaling
        L = torch.zeros(B, nmax, nmax, device=dev)
        gid = torch.repeat_interleave(torch.arange(B, device=dev),
                                      torch.as_tensor(ns, device=dev), output_size=int(n_off[-1]))
        loc = torch.arange(int(n_off[-1]), device=dev) - torch.as_tensor(n_off[:-1], device=dev)[gid]
        L[gid[ei_t[0]], loc[ei_t[0]], loc[ei_t[1]]] = w_t
        pad = torch.arange(nmax, device=dev).unsqueeze(0) >= torch.as_tensor(ns, device=dev).unsqueeze(1)
        L = L + torch.diag_embed(pad.to(L.dtype) * big)
        vals, vecs = torch.linalg.eigh(L)  # ascending per graph
        pe_all = vecs[:, :, 1:self.pe_k]  # [B, nmax, k-1]
        pe = pe_all[gid, loc]  # [N, k-1]
        # features on the device
        x = torch.from_numpy(np.concatenate([self.x[i] for i in idx])).to(dev)
        pos = torch.from_numpy(np.concatenate([self.pos[i] for i in idx])).to(dev)
        attr = torch.from_numpy(np.concatenate(attrs)).to(dev)
        src, dst = ei_d[0], ei_d[1]
        node = torch.cat([x, pos, pe], 1)
        edge = torch.cat([attr.view(-1, 1), (x[src] - x[dst]).abs(), (pe[src] + pe[dst]).abs()], 1)
        c_node = torch.from_numpy(np.concatenate([c[0] for c in cmaps]).astype(np.float32)).to(dev)
        c_edge = torch.from_numpy(np.concatenate([c[1] for c in cmaps])).to(dev)

        def width(a, w):
            if a.shape[1] < w:
                a = torch.cat([a, a.new_zeros(a.shape[0], w - a.shape[1])], 1)
            return a[:, :w].contiguous()
        lv0 = Batch()
        lv0.num_graphs = B
        lv0.x_t = width(torch.cat([c_node.view(-1, 1), node], 1), self.NODE_DIM + self.keig)
        lv0.x_s = width(torch.cat([c_edge.view(-1, 1), edge], 1), self.EDGE_DIM + self.keig)
        lv0.edge_index_t, lv0.edge_weight_t = ei_t, w_t
        lv0.edge_index_s, lv0.edge_weight_s = ei_s, w_s
        lv0.edge_index = ei_d
        lv0.y = torch.cat([self.y[i] for i in idx]).to(dev)
        lv0.num_node1 = torch.tensor(ns)
        lv0.num_edge1 = torch.tensor(E_g)
        lv0.num_nodes = int(n_off[-1])
        # coarse level: the MLGC graphs, Laplacians on the device again
        n1 = [int(c[3]) for c in cmaps]
        o1 = np.concatenate([[0], np.cumsum(n1)])
        ei1 = torch.from_numpy(np.ascontiguousarray(np.concatenate(
            [c[2] + o for c, o in zip(cmaps, o1[:-1])], axis=1))).to(dev)
        c_t, c_wt, c_s, c_ws, _ = ops.hodge_build(ei1, n1)
        lv1 = Batch()
        lv1.num_graphs = B
        lv1.x_t = torch.ones(int(o1[-1]), 1, device=dev)
        lv1.x_s = torch.ones(ei1.shape[1], 1, device=dev)
        lv1.edge_index_t, lv1.edge_weight_t = c_t, c_wt
        lv1.edge_index_s, lv1.edge_weight_s = c_s, c_ws
        lv1.edge_index = ei1
        lv1.num_node1 = torch.tensor(n1)
        lv1.num_edge1 = torch.tensor([int(c[2].shape[1]) for c in cmaps])
        lv1.num_nodes = int(o1[-1])
        for lv in (lv0, lv1):
            lv.hodge_sorted = {"edge_index_s": True, "edge_index_t": True}
            lv.l1_factor = False
            lv._mark()
        # every L1 of the builder is fl(2 / lmax) B1^T B1 exactly (entries
        # fl(fl(2 v) / lmax), v in {2, +-1}): the factored L1 holds by
        # construction -- declared where it pays (hodge_dataset.FACTOR_MIN_ROW)
        from .hodge_dataset import FACTOR_MIN_ROW
        if ei_s.shape[1] >= FACTOR_MIN_ROW * max(ei_d.shape[1], 1):
            ops.set_hodge_factor(lv0.edge_index_s, lv0.edge_index, lv0.num_nodes)
            lv0.l1_factor = True
        return lv0, lv1
