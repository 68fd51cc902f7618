"""Host-side logic: PairData batching, layouts, module names (CPU only)."""
import numpy as np
import pytest
import torch

from conftest import load_golden


def test_collate_offsets_follow_pairdata_inc():
    """lib/Hodge_Dataset.py:40-48: edge_index_s += N_s, edge_index_t and
    edge_index += N_t per preceding graph."""
    from hlhgat.synthetic import zinc_like_graph
    from hlhgat.hodge_dataset import collate
    gs = [zinc_like_graph(i) for i in range(3)]
    b = collate(gs)
    nt = [g.x_t.shape[0] for g in gs]
    ns = [g.x_s.shape[0] for g in gs]
    assert b.x_t.shape[0] == sum(nt) and b.x_s.shape[0] == sum(ns)
    e0 = gs[0].edge_index_s.shape[1]
    assert torch.equal(b.edge_index_s[:, e0:e0 + gs[1].edge_index_s.shape[1]],
                       gs[1].edge_index_s + ns[0])
    c0 = gs[0].edge_index.shape[1]
    assert torch.equal(b.edge_index[:, c0:c0 + gs[1].edge_index.shape[1]],
                       gs[1].edge_index + nt[0])
    t0 = gs[0].edge_index_t.shape[1]
    assert torch.equal(b.edge_index_t[:, t0:t0 + gs[1].edge_index_t.shape[1]],
                       gs[1].edge_index_t + nt[0])
    assert b.num_node1.tolist() == nt and b.num_edge1.tolist() == ns
    assert b.hodge_sorted == {"edge_index_s": True, "edge_index_t": True}


def test_hodge_laplacian_structure():
    """L0 = 2 B1 B1^T / lmax, L1 = 2 B1^T B1 / lmax (lib/Hodge_Dataset.py:451-456):
    nnz(L0) = N + 2E for a graph without isolated nodes, nnz(L1) = E + sum d(d-1),
    spectrum of both in [0, 2]."""
    from hlhgat.synthetic import zinc_like_graph
    g = zinc_like_graph(5)
    n, E = g.x_t.shape[0], g.x_s.shape[0]
    assert g.edge_index_t.shape[1] == n + 2 * E
    deg = np.bincount(g.edge_index.numpy().reshape(-1), minlength=n)
    assert g.edge_index_s.shape[1] == E + int((deg * (deg - 1)).sum())
    L1 = torch.zeros(E, E)
    L1[g.edge_index_s[0], g.edge_index_s[1]] = g.edge_weight_s
    ev = torch.linalg.eigvalsh(L1.double())
    assert ev.min() > -1e-5 and ev.max() < 2 + 1e-5


def test_is_sorted_symmetric():
    from hlhgat.hodge_dataset import is_sorted_symmetric
    ei = np.array([[0, 0, 1, 1], [0, 1, 0, 1]])
    w = np.array([1.0, 2.0, 2.0, 3.0])
    assert is_sorted_symmetric(ei, w)
    assert not is_sorted_symmetric(ei, np.array([1.0, 2.0, 2.5, 3.0]))
    assert not is_sorted_symmetric(ei[:, ::-1].copy(), w[::-1].copy())


def test_adj2par1_dense_matches_reference_golden():
    from hlhgat.hodge_dataset import adj2par1
    g = load_golden("adj2par1_small")
    par = adj2par1(torch.from_numpy(g["edge_index"]), int(g["n_nodes"]),
                   g["edge_index"].shape[1])
    assert np.array_equal(par.to_dense().numpy(), g["dense"])


def test_boundary_from_sparse_roundtrip():
    from hlhgat.hodge_dataset import adj2par1, boundary_from_sparse
    ei = torch.tensor([[0, 0, 1, 2], [1, 2, 2, 3]])
    par = adj2par1(ei, 4, 4).to_sparse_coo()
    assert torch.equal(boundary_from_sparse(par).edge_index, ei)


def test_state_dict_keys_match_reference_checkpoint_names():
    """Product and oracle modules share the reference's state_dict keys; the
    gnn.Sequential module_{i} / gnn.BatchNorm .module naming follows
    HL-HGAT-DEMO/weights/HL_HGAT_Brain.pt."""
    import hlhgat
    from oracle.hodge_ref import RefZincModel
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[2, 2, 2], filters=[64, 64, 64],
                                            mlp_channels=[256, 256], K=3, keig=15)
    r = RefZincModel(channels=[2, 2, 2], filters=[64, 64, 64], mlp_channels=[256, 256],
                     K=3, keig=15)
    assert list(m.state_dict().keys()) == list(r.state_dict().keys())
    keys = set(m.state_dict().keys())
    for k in ("HL_init_conv.module_0.lins.0.weight", "HL_init_conv.module_1.module.running_mean",
              "HL_init_conv.module_4.bias", "NEInt00.WV_Node.0.weight", "NEInt21.WV_Edge.4.bias",
              "NEConv21.module_5.module.weight", "mlp1.0.weight", "out.bias"):
        assert k in keys, k
    assert sum(p.numel() for p in m.parameters()) == 658433  # 0.66M


def test_reference_golden_state_dict_loads_into_product():
    import hlhgat
    g = load_golden("zinc_model_small")
    m = hlhgat.HL_HGCNN_zinc_dense_int3_pyr(channels=[1, 1], filters=[16, 16],
                                            mlp_channels=[32], K=3, keig=15)
    missing, unexpected = m.load_state_dict(
        {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd/")}, strict=True)
    assert not missing and not unexpected


def test_sequential_routing_and_names():
    from hlhgat.nn import Sequential
    seq = Sequential("a, b", [(torch.nn.Identity(), "a -> a"), (lambda x, y: x + y, "a, b -> c"),
                              (torch.nn.ReLU(), "c -> c")])
    out = seq(torch.tensor([-1.0, 2.0]), torch.tensor([0.5, 0.5]))
    assert torch.equal(out, torch.tensor([0.0, 2.5]))
    assert "module_0" in dict(seq.named_children()) and callable(seq.module_1)


def test_synthetic_zinc_statistics():
    """Synthetic ZINC-like batch matches the survey's shape statistics."""
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(300, seed=1)
    assert 21.5 < b.num_node1.float().mean() < 25.0
    assert 23.0 < b.num_edge1.float().mean() < 27.0
    assert b.x_t.shape[1] == 36 and b.x_s.shape[1] == 18


def test_sequential_two_chain_split_cpu():
    """The node / edge chains of an HL block are detected as independent
    (they run on two HIP streams on the GPU); on CPU the result is the
    modules applied in turn."""
    import torch
    from hlhgat.nn import Sequential
    torch.manual_seed(0)
    lt, ls = torch.nn.Linear(4, 3), torch.nn.Linear(5, 3)
    seq = Sequential("x_t, w_t, x_s, w_s", [
        (lt, "x_t -> x_t"), (torch.nn.ReLU(), "x_t -> x_t"), (torch.nn.Dropout(0.0), "x_t -> x_t"),
        (ls, "x_s -> x_s"), (torch.nn.Tanh(), "x_s -> x_s"),
        (lambda a, b: [a, b], "x_t, x_s -> x")])
    assert seq._split == 3
    xt, xs = torch.randn(6, 4), torch.randn(7, 5)
    a, b = seq(xt, None, xs, None)
    assert torch.equal(a, torch.relu(lt(xt)))
    assert torch.equal(b, torch.tanh(ls(xs)))
    chain = Sequential("x", [(lt, "x -> y"), (torch.nn.ReLU(), "y -> y")])
    assert chain._split is None


def test_dense_concat_matches_torch_cat():
    """ops.DenseConcat (one slab for the dense HL concatenation,
    lib/Hodge_ST_Model.py:631-632) gives torch.cat's values and gradients."""
    from hlhgat import ops
    torch.manual_seed(0)
    N = 7
    x = torch.randn(N, 3, requires_grad=True)
    ws = [torch.randn(3, 4)] + [torch.randn(4 * k, 4) for k in range(1, 4)]

    def run(dense):
        y0 = torch.tanh(x @ ws[0])
        d = ops.DenseConcat(N, 16, x) if dense else None
        x0 = y0
        if dense:
            d.append(y0)
        for k in range(1, 4):
            xin = d.view() if dense else x0
            y = torch.sin(xin @ ws[k])
            if dense:
                d.append(y)
            else:
                x0 = torch.cat([x0, y], -1)
        return (y ** 2).sum() + (d.view() if dense else x0).sum()

    l1 = run(False)
    g1, = torch.autograd.grad(l1, x)
    l2 = run(True)
    g2, = torch.autograd.grad(l2, x)
    assert torch.equal(l1.detach(), l2.detach())
    assert torch.allclose(g1, g2, rtol=0, atol=1e-6)


def test_row_order_collate_offsets_and_permutation():
    """locality_order is a permutation; collate offsets it like edge_index."""
    from hlhgat.hodge_dataset import collate, locality_order
    from hlhgat.synthetic import tsp_like_graph
    gs = [tsp_like_graph(s, n=300, k=5) for s in range(2)]
    for g in gs:
        for k, n in (("row_order_s", g.x_s.shape[0]), ("row_order_t", g.x_t.shape[0])):
            o = getattr(g, k)
            assert torch.equal(torch.sort(o).values, torch.arange(n))
    b = collate(gs, check_hodge=False)
    ns = [g.x_s.shape[0] for g in gs]
    assert torch.equal(b.row_order_s[:ns[0]], gs[0].row_order_s)
    assert torch.equal(b.row_order_s[ns[0]:], gs[1].row_order_s + ns[0])
    assert torch.equal(torch.sort(b.row_order_s).values, torch.arange(sum(ns)))
    # RCM shrinks the bandwidth of L1 substantially
    ei = gs[0].edge_index_s.numpy()
    o = locality_order(ei, ns[0]).numpy()
    inv = np.empty_like(o)
    inv[o] = np.arange(len(o))
    assert np.abs(inv[ei[0]] - inv[ei[1]]).max() < np.abs(ei[0] - ei[1]).max()


def test_pad_batch_structure():
    from hlhgat.hodge_dataset import is_sorted_symmetric, pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(30, seed=2)
    caps = static_caps(b, 128)
    p = pad_batch(b, caps)
    assert p.x_t.shape[0] == caps["rows_t"] and p.x_s.shape[0] == caps["rows_s"]
    assert p.edge_index_t.shape[1] == caps["nnz_t"] and p.edge_index_s.shape[1] == caps["nnz_s"]
    assert p.edge_index.shape[1] == caps["rows_s"]
    for side in ("t", "s"):
        ei, w = getattr(p, "edge_index_" + side), getattr(p, "edge_weight_" + side)
        assert is_sorted_symmetric(ei.numpy(), w.numpy())
        n = getattr(b, "x_" + side).shape[0]
        assert int(getattr(p, "n_valid_" + side)) == n
        assert float(getattr(p, "x_" + side)[n:].abs().sum()) == 0.0
    assert int(p.valid_mask_t.sum()) == b.x_t.shape[0]
    assert torch.equal(p.num_node1, b.num_node1) and torch.equal(p.num_edge1, b.num_edge1)


def test_batch_to_rejects_counts_beyond_rows():
    """Batch.to checks on the host that the per-graph counts fit the rows
    (the capturable forward's repeat_interleave(output_size=rows) trusts it);
    padded rows beyond the sum are fine."""
    from hlhgat.hodge_dataset import pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(5, seed=1)
    pad_batch(b, static_caps(b, 128)).to("cpu")  # sum < rows: padding, accepted
    b.num_edge1 = b.num_edge1.clone()
    b.num_edge1[0] += 1
    with pytest.raises(ValueError, match="num_edge1 sums to"):
        b.to("cpu")


def test_incidence_csr_host_build():
    """Collate-time incidence CSR of |B1| (hodge_dataset.incidence_csr): row v
    lists the edges with an endpoint at v, ascending (adj2par1,
    lib/Hodge_Dataset.py:169-191); pad_batch's self-edges appear twice."""
    from hlhgat.hodge_dataset import incidence_csr, pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_batch
    b = zinc_like_batch(20, seed=4)
    for batch in (b, pad_batch(b, static_caps(b, 128))):
        ei, n = batch.edge_index.numpy(), batch.x_t.shape[0]
        rp, eids = batch.inc_rowptr.numpy(), batch.inc_eids.numpy()
        assert rp.dtype == np.int32 and eids.dtype == np.int32
        assert rp.shape == (n + 1,) and eids.shape == (2 * ei.shape[1],)
        for v in range(n):
            want = sorted(np.nonzero(ei[0] == v)[0].tolist() + np.nonzero(ei[1] == v)[0].tolist())
            assert eids[rp[v]:rp[v + 1]].tolist() == want, v
    from hlhgat.hodge_dataset import degree
    d = degree(b.edge_index.reshape(-1), num_nodes=b.x_t.shape[0])
    assert torch.equal(b.deg_t, d) and torch.equal(b.inv_deg_t, 1 / d)
    p = pad_batch(b, static_caps(b, 128))
    dp = degree(p.edge_index.reshape(-1), num_nodes=p.x_t.shape[0]).masked_fill(~p.valid_mask_t, 1)
    assert torch.equal(p.deg_t, dp) and torch.equal(p.inv_deg_t, 1 / dp)
    for batch in (b, p):  # Laplacian CSRs built with the batch (rows = edge_index[0])
        for side in ("t", "s"):
            ei = getattr(batch, "edge_index_" + side).numpy()
            n = getattr(batch, "x_" + side).shape[0]
            crp = getattr(batch, "csr_rowptr_" + side).numpy()
            assert crp.dtype == np.int32 and crp.shape == (n + 1,)
            assert np.array_equal(np.diff(crp), np.bincount(ei[0], minlength=n))
            assert np.array_equal(getattr(batch, "csr_col_" + side).numpy(), ei[1])
    # isolated nodes: degree 0 and 1/0 = inf, as degree() and torch's reciprocal give
    from hlhgat.hodge_dataset import node_degree
    rp, _ = incidence_csr(np.array([[0], [2]]), 4)
    d, r = node_degree(rp)
    assert d.tolist() == [1.0, 0.0, 1.0, 0.0] and torch.equal(r, 1 / d)
    d, r = node_degree(rp, valid=3)
    assert d.tolist() == [1.0, 0.0, 1.0, 1.0]
    rp, eids = incidence_csr(np.zeros((2, 0), dtype=np.int64), 3)
    assert rp.tolist() == [0, 0, 0, 0] and eids.numel() == 0
    with pytest.raises(ValueError):
        incidence_csr(np.array([[0], [5]]), 3)


def test_fastconv_adj_t_forms_agree():
    """HodgeLaguerreFastConv.forward(x, adj_t) accepts the DEMO's
    SparseTensor(row=ei[0], col=ei[1], value=w).t() (duck-typed .coo()), a
    torch sparse tensor holding A^T, or (edge_index, edge_weight); all map to
    the same propagate edge list (HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py:179-180)."""
    from hlhgat import HodgeLaguerreFastConv
    ei = torch.tensor([[0, 1, 1, 2, 3], [1, 0, 2, 3, 3]])
    w = torch.tensor([0.5, 0.25, 1.5, 2.0, 3.0])

    class _ST:  # torch_sparse.SparseTensor(...).t(): rows = targets, sorted
        def coo(self):
            perm = torch.argsort(ei[1] * 10 + ei[0])
            return ei[1][perm], ei[0][perm], w[perm]

    dense_t = torch.zeros(4, 4).index_put_((ei[1], ei[0]), w, accumulate=True)
    for adj in (_ST(), dense_t.to_sparse_coo(), dense_t.to_sparse_csr(), (ei, w)):
        e2, w2 = HodgeLaguerreFastConv.adj_to_edge_index(adj)
        got = torch.zeros(4, 4).index_put_((e2[1], e2[0]), w2, accumulate=True)
        assert torch.equal(got, dense_t)
    assert HodgeLaguerreFastConv(4, 4, K=3)._kind != HodgeLaguerreFastConv(
        4, 4, K=3, demo_recurrence=False)._kind


def _check_halo(ei, n, order, ht, max_rows, max_halo, max_nnz=3072):
    tp, hp = ht["halo_tile_ptr"].numpy(), ht["halo_ptr"].numpy()
    hc, srp = ht["halo"].numpy(), ht["halo_srp"].numpy()
    lc, ep = ht["halo_lcol"].numpy().view(np.uint16), ht["halo_eperm"].numpy()
    assert tp[0] == 0 and tp[-1] == n and np.all(np.diff(tp) > 0)
    assert np.all(np.diff(tp) <= max_rows) and np.all(np.diff(hp) <= max_halo)
    assert np.all(np.diff(srp[tp]) <= max_nnz)
    rowptr = np.concatenate([[0], np.cumsum(np.bincount(ei[0], minlength=n))])
    sched = np.arange(n) if order is None else np.asarray(order)
    assert srp[-1] == ei.shape[1] and np.array_equal(np.sort(ep), np.arange(ei.shape[1]))
    for t in range(len(tp) - 1):
        halo = hc[hp[t]:hp[t + 1]]
        assert np.all(np.diff(halo) > 0)  # ascending, distinct
        for p in range(tp[t], tp[t + 1]):
            r = sched[p]
            i = np.arange(srp[p], srp[p + 1])
            assert np.array_equal(ep[i], np.arange(rowptr[r], rowptr[r + 1]))
            assert np.array_equal(halo[lc[i]], ei[1][ep[i]])


def test_halo_tiles_invariants():
    """hlhgat_halo_tiles (native host builder): tiles partition the row
    schedule, each halo holds exactly its rows' distinct columns (sorted),
    lcol points every CSR entry at its column inside the halo."""
    from hlhgat.hodge_dataset import halo_tiles, locality_order
    from hlhgat.synthetic import tsp_like_graph
    g = tsp_like_graph(3, n=600, k=6, halo=False)
    for ei, n, order in ((g.edge_index_s.numpy(), g.x_s.shape[0], g.row_order_s.numpy()),
                         (g.edge_index_t.numpy(), g.x_t.shape[0], None)):
        for max_rows, max_halo, max_nnz in ((128, 256, 3072), (16, 64, 3072), (3, 40, 3072),
                                            (128, 256, 100)):
            ht = halo_tiles(ei, n, order, max_rows=max_rows, max_halo=max_halo, max_nnz=max_nnz)
            _check_halo(ei, n, order, ht, max_rows, max_halo, max_nnz)
            hd = ht["halo_hdr"].numpy()
            tp, hp, srp = ht["halo_tile_ptr"].numpy(), ht["halo_ptr"].numpy(), ht["halo_srp"].numpy()
            assert np.array_equal(hd[:, 0], tp[:-1]) and np.array_equal(hd[:, 3], np.diff(hp))
            assert np.array_equal(hd[:, 5], np.diff(srp[tp]))
    assert locality_order(g.edge_index_s.numpy(), g.x_s.shape[0]).numel() == g.x_s.shape[0]


def test_halo_tiles_reject_and_collate():
    from hlhgat.hodge_dataset import collate, halo_tiles
    from hlhgat.synthetic import tsp_like_graph
    g = tsp_like_graph(4, n=400, k=6)
    ei = g.edge_index_s.numpy()
    assert halo_tiles(ei, g.x_s.shape[0], None, max_halo=3) is None  # a row has > 3 columns
    b = collate([g, tsp_like_graph(5, n=300, k=6)], check_hodge=False)
    ht = {k: getattr(b, k + "_s") for k in ("halo_tile_ptr", "halo_ptr", "halo", "halo_srp",
                                             "halo_lcol", "halo_eperm", "halo_hdr")}
    _check_halo(b.edge_index_s.numpy(), b.x_s.shape[0], b.row_order_s.numpy(), ht, 128, 256)


def test_mlgc_matches_reference_golden():
    """MLGC (lib/Hodge_Dataset.py:241-297) against the reference's own MLGC run
    on the same graphs (tests/golden/make_golden_attpool.py).  torch_cluster is
    absent, so the reference's graclus call was answered by hlhgat's graclus
    restatement (labels stored): graclus itself is parity unpinned; renumbering,
    edge assignment (inf = contracted edge), coarse B1 and L0/L1 are pinned."""
    from hlhgat.hodge_dataset import PairData, graclus, mlgc
    g = load_golden("mlgc_small")
    for gi in range(3):
        p = f"g{gi}/"
        n = int(g[p + "num_node1"])
        ei, eit = g[p + "edge_index"], g[p + "edge_index_t"]
        assert np.array_equal(graclus(eit, n, seed=gi), g[p + "graclus"])
        d = PairData(x_s=torch.zeros(ei.shape[1], 1), x_t=torch.zeros(n, 1),
                     edge_index_t=torch.from_numpy(eit))
        d.edge_index = torch.from_numpy(ei)
        d.num_node1 = n
        coarse, c_node, c_edge = mlgc(d, seed=gi)
        assert np.array_equal(c_node.numpy().reshape(-1), g[p + "c_node"].reshape(-1))
        ce, ref_ce = c_edge.numpy().reshape(-1), g[p + "c_edge"].reshape(-1)
        assert np.array_equal(np.isinf(ce), np.isinf(ref_ce))
        assert np.array_equal(ce[~np.isinf(ce)], ref_ce[~np.isinf(ref_ce)])
        assert coarse.num_node1 == int(g[p + "coarse/num_node1"])
        for k in ("edge_index", "edge_index_t", "edge_index_s"):
            assert np.array_equal(getattr(coarse, k).numpy(), g[p + "coarse/" + k]), k
        for k in ("edge_weight_t", "edge_weight_s", "x_t", "x_s"):
            np.testing.assert_allclose(getattr(coarse, k).numpy(), g[p + "coarse/" + k],
                                       rtol=1e-5, atol=1e-6, err_msg=k)


def test_graclus_is_a_matching():
    """Every graclus cluster has one or two members, a pair is joined by an
    edge, its id is the smaller member, and no two unmatched neighbours remain
    (greedy maximality, torch_cluster 1.6.0 graclus semantics)."""
    from hlhgat.hodge_dataset import graclus
    from hlhgat.synthetic import knn_edges
    rng = np.random.default_rng(3)
    ei = knn_edges(rng.random((300, 2)), 6)
    sym = np.concatenate([ei, ei[::-1]], axis=1)
    lab = graclus(sym, 300, seed=1)
    adj = set(map(tuple, sym.T.tolist()))
    alone = []
    for c in np.unique(lab):
        mem = np.flatnonzero(lab == c)
        assert 1 <= mem.size <= 2 and c == mem.min()
        if mem.size == 2:
            assert (int(mem[0]), int(mem[1])) in adj
        else:
            alone.append(int(mem[0]))
    alone = set(alone)
    for u, v in adj:
        assert not (u in alone and v in alone and u != v)


def test_hodge_factor_check():
    """hodge_factor_ok: every L1 the Hodge builder emits is alpha B1^T B1
    exactly (lib/Hodge_Dataset.py:451-456) -- the reference's own TSP fixture,
    CIFAR-like, ZINC-like and MLGC-coarsened graphs; a perturbed weight, a
    dropped entry or a flipped edge orientation is rejected.  collate turns the
    factored L1 on for high-degree batches only, pad_batch turns it off."""
    from hlhgat.hodge_dataset import collate, hodge_factor_ok, pad_batch, static_caps
    from hlhgat.synthetic import cifar_like_graphs, zinc_like_graph
    g = load_golden("tsp_model_small")
    assert hodge_factor_ok(g["edge_index"], g["x_t"].shape[0], g["edge_index_s"],
                           g["edge_weight_s"])
    for c in (cifar_like_graphs(1)[0], cifar_like_graphs(2)[1], zinc_like_graph(3)):
        ei, eis, w = c.edge_index.numpy(), c.edge_index_s.numpy(), c.edge_weight_s.numpy()
        n = c.x_t.shape[0]
        assert hodge_factor_ok(ei, n, eis, w)
        w2 = w.copy()
        w2[3] = np.nextafter(w2[3], np.float32(np.inf))
        assert not hodge_factor_ok(ei, n, eis, w2)
        assert not hodge_factor_ok(ei, n, eis[:, 1:], w[1:])
        assert not hodge_factor_ok(ei[::-1], n, eis, w)
    assert collate([cifar_like_graphs(s)[0] for s in range(2)]).l1_factor
    zb = collate([zinc_like_graph(s) for s in range(4)])
    assert not zb.l1_factor
    cb = collate([cifar_like_graphs(s)[0] for s in range(2)])
    # padding edges are zero columns of B1 with alpha_e = 0: the factor holds
    # for the padded batch too (hodge_dataset.pad_batch)
    pb = pad_batch(cb, static_caps(cb))
    assert pb.l1_factor
    ei, eis, w = pb.edge_index.numpy(), pb.edge_index_s.numpy(), pb.edge_weight_s.numpy()
    ns, nt = cb.x_s.shape[0], cb.x_t.shape[0]
    real = (eis[0] < ns) & (eis[1] < ns)
    assert hodge_factor_ok(ei[:, :ns], nt, eis[:, real], w[real])
    assert np.all(w[~real] == 0) and np.all(eis[0][~real] == eis[1][~real])


def test_brain_skeleton_coo_rebuild_matches_reference():
    """The DEMO brain skeleton (HL-HGAT-DEMO/data, 268 nodes, 8997 edges,
    nnz(L1) 1.37 M): hodge_coo_from_boundary(edge_index, lmax) reproduces the
    reference's dense-built L0 / L1 COO bitwise at 2000 sampled entries, in
    entry count, weight sum and |weight| sum; the L1 is alpha B1^T B1."""
    from hlhgat.hodge_dataset import hodge_coo_from_boundary, hodge_factor_ok
    g = load_golden("brain_skeleton")
    ei_t, w_t, ei_s, w_s = hodge_coo_from_boundary(g["edge_index"], int(g["n_nodes"]),
                                                   float(g["lmax"]))
    for side, (e, w) in {"t": (ei_t, w_t), "s": (ei_s, w_s)}.items():
        assert e.shape[1] == int(g[f"nnz_{side}"])
        idx = g[f"{side}/coo_idx"]
        assert np.array_equal(e.numpy()[:, idx], g[f"{side}/coo_rc"])
        assert np.array_equal(w.numpy()[idx], g[f"{side}/coo_w"])
        assert float(w.double().sum()) == float(g[f"{side}/w_sum64"])
        assert float(w.double().abs().sum()) == float(g[f"{side}/w_abs_sum64"])
    assert hodge_factor_ok(g["edge_index"], int(g["n_nodes"]), ei_s.numpy(), w_s.numpy())


def test_boundary_operator_views_match_reference_adj2par1():
    """adj2par1 views (.abs(), .t(), .transpose(0, 1)) densify to the reference's
    sparse B1 (adj2par1_small golden) and its |.| / transpose; products need the
    ROCm device (no CPU fallback)."""
    import pytest
    import torch
    from conftest import load_golden
    from hlhgat.hodge_dataset import adj2par1
    g = load_golden("adj2par1_small")
    ei = torch.from_numpy(g["edge_index"])
    P = adj2par1(ei, int(g["n_nodes"]), ei.shape[1])
    dense = torch.from_numpy(g["dense"])
    assert torch.equal(P.to_dense(), dense)
    assert torch.equal(P.abs().to_dense(), dense.abs())
    assert torch.equal(P.transpose(0, 1).to_dense(), dense.t())
    assert torch.equal(P.t().abs().to_dense(), dense.abs().t())
    assert P.t().shape == (ei.shape[1], int(g["n_nodes"])) and P.T.t().shape == P.shape
    assert P.t().incidence is not None and P.abs()._base is P
    with pytest.raises(RuntimeError, match="ROCm"):
        torch.sparse.mm(P.transpose(0, 1), torch.ones(int(g["n_nodes"]), 3))


def test_mlgc_weighted_matches_reference_golden():
    """MLGC_weighted (lib/Hodge_Dataset.py:298-353) against the reference's own
    run (tests/golden/make_golden_attpool.py): the weights the reference hands
    to graclus (to_undirected mean of exp(-x_s^2)) are pinned through our
    to_undirected_mean; graclus is parity unpinned (labels stored); the map
    and coarse graph are pinned."""
    from hlhgat.hodge_dataset import PairData, graclus, mlgc_weighted, to_undirected_mean
    g = load_golden("mlgc_weighted_small")
    for gi in range(3):
        p = f"g{gi}/"
        n = int(g[p + "num_node1"])
        ei, xs = g[p + "edge_index"], g[p + "x_s"]
        w_ref = np.exp(-(xs[:, 0].astype(np.float32) ** 2))
        ei_u, w_u = to_undirected_mean(ei, w_ref, n)
        assert np.array_equal(ei_u, g[p + "graclus_edge_index"])
        np.testing.assert_allclose(w_u, g[p + "graclus_weight"], rtol=1e-6, atol=0)
        assert np.array_equal(graclus(ei_u, n, weight=w_u, seed=100 + gi), g[p + "graclus"])
        d = PairData(x_s=torch.from_numpy(xs), x_t=torch.zeros(n, 1))
        d.edge_index = torch.from_numpy(ei)
        d.num_node1 = n
        coarse, c_node, c_edge = mlgc_weighted(d, seed=100 + gi)
        assert np.array_equal(c_node.numpy().reshape(-1), g[p + "c_node"].reshape(-1))
        ce, ref_ce = c_edge.numpy().reshape(-1), g[p + "c_edge"].reshape(-1)
        assert np.array_equal(np.isinf(ce), np.isinf(ref_ce))
        assert np.array_equal(ce[~np.isinf(ce)], ref_ce[~np.isinf(ref_ce)])
        assert coarse.num_node1 == int(g[p + "coarse/num_node1"])
        for k in ("edge_index", "edge_index_t", "edge_index_s"):
            assert np.array_equal(getattr(coarse, k).numpy(), g[p + "coarse/" + k]), k
        for k in ("edge_weight_t", "edge_weight_s", "x_t", "x_s"):
            np.testing.assert_allclose(getattr(coarse, k).numpy(), g[p + "coarse/" + k],
                                       rtol=1e-5, atol=1e-6, err_msg=k)


def test_native_mlgc_equals_oracle_restatement():
    """The native host builders (hlhgat_graclus / hlhgat_mlgc_map in
    libhlhgat.so) against the oracle's pure-Python restatement
    (oracle/hodge_ref.py graclus / mlgc_map / to_undirected_mean), bitwise, on
    random multigraphs with self-loops, duplicates, isolated nodes, weights
    with ties, and empty inputs."""
    from hlhgat import hodge_dataset as hd
    from oracle import hodge_ref as ref
    rng = np.random.default_rng(11)
    for n, E in [(0, 0), (1, 0), (4, 1), (7, 3), (60, 250), (400, 3000)]:
        ei = rng.integers(0, max(n, 1), size=(2, E)) if n else np.zeros((2, 0), np.int64)
        sym = np.concatenate([ei, ei[::-1]], axis=1)
        for w in (None, rng.integers(0, 3, sym.shape[1]).astype(np.float64),
                  rng.random(sym.shape[1])):
            for seed in range(2):
                perm = np.random.default_rng(seed).permutation(n)
                lab = hd.graclus(sym, n, weight=w, seed=seed)
                assert np.array_equal(lab, ref.graclus(sym, n, weight=w, perm=perm)), (n, E)
                for a, b in zip(hd.mlgc_map(lab, ei), ref.mlgc_map(lab, ei)):
                    assert np.array_equal(np.asarray(a), np.asarray(b)), (n, E)
        if E:
            w = rng.random(E).astype(np.float32)
            for a, b in zip(hd.to_undirected_mean(ei, w, n), ref.to_undirected_mean(ei, w, n)):
                assert np.array_equal(a, b)


def test_native_mlgc_rejects_bad_input():
    from hlhgat import hodge_dataset as hd
    from hlhgat._lib import HlhgatError
    with pytest.raises(HlhgatError, match="out of range"):
        hd.graclus(np.array([[0, 5], [1, 0]]), 3)
    with pytest.raises(HlhgatError, match="out of range"):
        hd.mlgc_map(np.array([0, 0, 7]), np.array([[0], [1]]))


# ---------------------------------------------------------------------------
# native loader: PackedGraphs.collate (hlhgat_collate) == collate + pad_batch
# ---------------------------------------------------------------------------
def _same_batch(a, b):
    # (_arena: the storage PackedGraphs.collate carves its tensors from)
    ta = {k for k, v in vars(a).items() if torch.is_tensor(v) and k != "_arena"}
    tb = {k for k, v in vars(b).items() if torch.is_tensor(v) and k != "_arena"}
    assert ta == tb, (sorted(ta - tb), sorted(tb - ta))
    for k in ta:
        x, y = getattr(a, k), getattr(b, k)
        assert x.dtype == y.dtype and x.shape == y.shape and torch.equal(x, y), k
    for k in ("num_graphs", "num_nodes", "hodge_sorted", "l1_factor"):
        assert getattr(a, k) == getattr(b, k), k


def test_native_collate_equals_python_collate_and_pad():
    """hlhgat_collate (csrc/collate.hip) builds, bitwise, every array of
    hodge_dataset.collate (unpadded) and of collate + pad_batch (padded):
    features, offset COO blocks, B1 edge list, y, graph sizes, the Laplacian
    / incidence CSRs, degrees, segment offsets and the padding."""
    import numpy as np
    from hlhgat.hodge_dataset import PackedGraphs, collate, pad_batch, static_caps
    from hlhgat.synthetic import zinc_like_graph
    gs = [zinc_like_graph(5000 + i, keig=15) for i in range(160)]
    ds = PackedGraphs(gs)
    for idx in (np.arange(37), np.random.RandomState(3).permutation(160)[:101], np.array([7])):
        ref = collate([gs[i] for i in idx], check_hodge=False)
        _same_batch(ds.collate(idx), ref)
        assert ds.sizes(idx) == (ref.x_t.shape[0], ref.x_s.shape[0], ref.edge_index_t.shape[1],
                                 ref.edge_index_s.shape[1])
        for q in (64, 512):
            caps = static_caps(ref, q)
            assert ds.caps_for(idx, q) == caps
            _same_batch(ds.collate(idx, caps), pad_batch(ref, caps))


def test_native_collate_rejects_bad_input():
    import numpy as np
    import pytest
    from hlhgat._lib import HlhgatError
    from hlhgat.hodge_dataset import PackedGraphs
    from hlhgat.synthetic import zinc_like_graph
    ds = PackedGraphs([zinc_like_graph(i, keig=15) for i in range(4)])
    with pytest.raises(HlhgatError, match="out of range"):
        ds.collate(np.array([0, 4]))
    caps = ds.caps_for(np.arange(4), 64)
    with pytest.raises(ValueError):
        ds.collate(np.arange(4), dict(caps, rows_t=10))
    g = zinc_like_graph(9, keig=15)
    g.edge_index_t = g.edge_index_t.flip(1)  # not row-sorted
    with pytest.raises(ValueError, match="row-sorted"):
        PackedGraphs([g])
    # the native collate validates the packed arrays themselves (they point
    # into host memory it writes through): indices outside their graph, and
    # rows out of order, are refused before any write
    for arr, v, what in (("lt_col", 10 ** 6, "L0 entry"), ("ls_row", -1, "L1 entry"),
                         ("b1_dst", 999, "B1 edge"), ("lt_row", 0, "L0 entry")):
        ds2 = PackedGraphs([zinc_like_graph(i, keig=15) for i in range(3)])
        a = getattr(ds2, arr)
        k = int(ds2.lt_ptr[2]) - 1 if arr == "lt_row" else 5  # lt_row: unsorted in graph 1
        a[k] = v
        with pytest.raises(HlhgatError, match=what):
            ds2.collate(np.arange(3))


def test_graph_loader_batches_in_order_and_shuffled():
    """GraphLoader: native collation on worker threads, batches in order;
    one capacity bucket per epoch; a shuffled epoch covers every graph once."""
    import numpy as np
    from hlhgat.hodge_dataset import PackedGraphs, collate, pad_batch
    from hlhgat.loader import GraphLoader
    from hlhgat.synthetic import zinc_like_graph
    gs = [zinc_like_graph(7000 + i, keig=15) for i in range(90)]
    ds = PackedGraphs(gs)
    ld = GraphLoader(ds, 20, workers=3, prefetch=2)
    got = list(ld)
    assert len(got) == len(ld) == 4
    caps = ld.epoch_caps(ld.batch_indices(0))
    for i, b in enumerate(got):
        _same_batch(b, pad_batch(collate(gs[20 * i:20 * i + 20], check_hodge=False), caps))
    sh = GraphLoader(ds, 30, shuffle=True, caps=False, seed=5)
    seen = np.concatenate(sh.batch_indices(0))
    assert sorted(seen.tolist()) == list(range(90))
    assert not np.array_equal(seen, np.arange(90))
    b0 = next(iter(sh))
    _same_batch(b0, collate([gs[i] for i in sh.batch_indices(0)[0]], check_hodge=False))


def test_graph_loader_stream_equals_epochs():
    """GraphLoader.stream (one collation pool prefetching across epochs) yields
    the batches of consecutive per-epoch iterations, bitwise, shuffled epochs
    included; closing it mid-epoch stops its threads."""
    from hlhgat.hodge_dataset import PackedGraphs
    from hlhgat.loader import GraphLoader
    from hlhgat.synthetic import zinc_like_graph
    gs = [zinc_like_graph(7100 + i, keig=15) for i in range(50)]
    ds = PackedGraphs(gs)
    ref = GraphLoader(ds, 12, shuffle=True, seed=3, workers=2, prefetch=3)
    want = [b for _ in range(3) for b in ref]
    got = list(GraphLoader(ds, 12, shuffle=True, seed=3, workers=2, prefetch=3).stream(3))
    assert len(got) == len(want) == 3 * 4
    for a, b in zip(got, want):
        _same_batch(a, b)
    it = GraphLoader(ds, 12, workers=2, prefetch=3).stream()
    for _ in range(6):  # past an epoch boundary of the endless stream
        next(it)
    it.close()


class _FakeStaged:
    def __init__(self, b):
        self.b, self.done = b, False

    def __eq__(self, other):
        return other == ("st", self.b)


class _FakeStep:
    """Stand-in for TrainStep's staging interface (stage / __call__ /
    unstage), recording the calls."""

    def __init__(self, limit=3):
        import threading
        self.staged, self.stepped, self.unstaged = [], [], []
        self.lock = threading.Lock()
        self.limit = limit

    def stage(self, b, stream):
        with self.lock:
            self.staged.append(b)
            out = len(self.staged) - len(self.stepped) - len(self.unstaged)
            assert out <= self.limit, "staged too far ahead"
        return _FakeStaged(b)

    def __call__(self, st):
        assert not st.done
        st.done = True
        with self.lock:
            self.stepped.append(st.b)

    def unstage(self, st):
        if st.done:
            return
        st.done = True
        with self.lock:
            self.unstaged.append(st.b)


@pytest.mark.parametrize("thread", [True, False])
def test_staged_feed_order_and_depth(thread):
    """StagedFeed's host logic (no device: a stand-in step records stage()
    calls): every batch is staged once, in order, handed over in order, and
    never more than `depth` staged batches wait beyond the one being stepped;
    a source error reaches the consumer."""
    from hlhgat.loader import StagedFeed

    step = _FakeStep()
    feed = StagedFeed(iter(range(17)), step, depth=2, stream=object(), thread=thread)
    for st in feed:
        assert st == ("st", len(step.stepped))
        step(st)
    assert step.staged == step.stepped == list(range(17))
    assert step.unstaged == []

    def bad():
        yield 0
        raise ValueError("source failed")

    step = _FakeStep()
    feed = StagedFeed(bad(), step, depth=2, stream=object(), thread=thread)
    with pytest.raises(ValueError, match="source failed"):
        for st in feed:
            pass
    assert step.unstaged == [0]  # handed out, never stepped: given back


@pytest.mark.parametrize("thread", [True, False])
@pytest.mark.parametrize("before_step", [False, True])
def test_staged_feed_early_close_unstages(thread, before_step):
    """a feed left early (break; the endless GraphLoader.stream()
    is only ever left that way) gives back every batch it staged and nobody
    stepped -- the queued ones and, when the consumer broke before stepping
    it, the one last handed out -- so the step's outstanding / pending counts
    return to what was stepped, and staging can go on (repeatedly)."""
    import itertools
    from hlhgat.loader import StagedFeed

    step = _FakeStep()
    for rnd in range(4):
        feed = StagedFeed(itertools.count(100 * rnd), step, depth=2, stream=object(),
                          thread=thread)
        for k, st in enumerate(feed):
            if before_step and k == 3:
                break
            step(st)
            if k == 3:
                break
        assert sorted(step.stepped + step.unstaged) == sorted(step.staged), rnd
    assert len(step.stepped) == (12 if before_step else 16)
    if not thread:  # the inline feed stages `depth` ahead deterministically
        assert len(step.unstaged) >= 4, step.unstaged


def test_native_mlgc_batch_equals_per_graph():
    """hlhgat_mlgc_batch (one call, host threads) gives per graph exactly the
    per-graph graclus(both directions, unit weights, perm) + mlgc_map."""
    import numpy as np
    from hlhgat.hodge_dataset import graclus, mlgc_batch, mlgc_map
    from hlhgat.synthetic import knn_edges
    rng = np.random.default_rng(4)
    eis, ns, perms = [], [], []
    for g in range(23):
        n = int(rng.integers(1, 90))
        ei = (knn_edges(rng.random((n, 2)), min(8, max(n - 1, 1))) if n > 1
              else np.zeros((2, 0), np.int64))
        ei = np.asarray(ei, np.int64)
        ei = ei[:, ei[0] < ei[1]]
        eis.append(ei)
        ns.append(n)
        perms.append(rng.permutation(n))
    for threads in (1, 4):
        got = mlgc_batch(eis, ns, perms, threads=threads)
        for ei, n, p, (cn, ce, e1, n1) in zip(eis, ns, perms, got):
            both = np.concatenate([ei, ei[::-1]], axis=1)
            lab = graclus(both, n, weight=np.ones(both.shape[1]), perm=p)
            rn, rce, re1, rn1 = mlgc_map(lab, ei)
            assert np.array_equal(cn, rn) and np.array_equal(ce, rce)
            assert np.array_equal(e1, re1) and n1 == rn1


@pytest.mark.parametrize("name,cls,kw", [
    ("head_pepfunc_pyr_small", "HL_HGCNN_pepfunc_dense_int3_pyr",
     dict(channels=[1, 1], filters=[16, 16], mlp_channels=[32], K=3, node_dim=21, edge_dim=3,
          keig=15)),
    ("head_cifar_pyr_small", "HL_HGCNN_CIFAR10SP_dense_int3_pyr",
     dict(channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, node_dim=21, edge_dim=3,
          keig=15, l=0.5)),
    ("head_zinc_poolint3_small", "HL_HGCNN_zinc_dense_poolint3_pyr",
     dict(channels=[1, 1], filters=[16, 16], mlp_channels=[32], K=3, keig=15)),
    ("head_zinc_attpool_small", "HL_HGCNN_zinc_dense_int3_attpool",
     dict(channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, node_dim=5, edge_dim=4,
          keig=10, pool_loc=0)),
    ("head_pepfunc_attpool_lib_small", "hodge_st_model.HL_HGCNN_pepfunc_dense_int3_attpool",
     dict(channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)),
    ("attpool_pepfunc_small", "HL_HGCNN_pepfunc_dense_int3_attpool",
     dict(channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, pool_loc=0)),
    ("attpool_cifar_small", "HL_HGCNN_CIFAR10SP_dense_int3_attpool",
     dict(channels=[1, 1], filters=[16, 32], mlp_channels=[32], K=3, keig=10, pool_loc=0,
          l=0.5))])
def test_head_state_dict_matches_reference(name, cls, kw):
    """Every head's constructor builds the reference's module tree: the same
    state_dict keys, in the same order, with the same shapes as the
    reference's own instance stored in the golden fixture (make_golden_heads /
    make_golden_attpool), so a reference checkpoint loads unchanged."""
    import hlhgat
    obj = hlhgat
    for part in cls.split("."):
        obj = getattr(obj, part)
    g = load_golden(name)
    ref = [(k[3:], tuple(g[k].shape)) for k in g if k.startswith("sd/")]
    ours = [(k, tuple(v.shape)) for k, v in obj(**kw).state_dict().items()]
    assert ours == ref


def test_factor_tables_equal_the_device_build_restated():
    """hodge_dataset.factor_tables (collate time, numpy) == what
    ops._build_factor computes on the device when the batch carries no
    tables, restated with the same torch ops on the CPU: alpha by an
    accumulating index_put of the L1 diagonal / 2, the signed incidence in
    CSR order, the int32 edge ends -- bit for bit, for a collated batch and
    its padded copy (padding edges: alpha 0, self-edge signs +1)."""
    from hlhgat.hodge_dataset import collate, pad_batch, static_caps
    from hlhgat.synthetic import cifar_like_graphs
    cb = collate([cifar_like_graphs(s)[0] for s in range(3)])
    assert cb.l1_factor and cb.fac_alpha is not None
    for b in (cb, pad_batch(cb, static_caps(cb))):
        ei_s, w = b.edge_index_s, b.edge_weight_s
        E = b.x_s.shape[0]
        diag = ei_s[0] == ei_s[1]
        alpha = torch.zeros(E, dtype=torch.float32)
        alpha.index_put_((ei_s[0],), torch.where(diag, w * 0.5, torch.zeros_like(w)),
                         accumulate=True)
        rp, eids = b.inc_rowptr.long(), b.inc_eids.long()
        node = torch.repeat_interleave(torch.arange(rp.numel() - 1), rp[1:] - rp[:-1])
        head = b.edge_index[1][eids]
        sign = torch.where(head == node, 1.0, -1.0).to(torch.float32)
        ends = b.edge_index.t().to(torch.int32).contiguous()
        assert torch.equal(b.fac_alpha, alpha)
        assert torch.equal(b.fac_sign, sign)
        assert torch.equal(b.fac_ends, ends)
        assert b.fac_alpha.dtype == torch.float32 and b.fac_ends.dtype == torch.int32


def test_pool_tables_equal_the_device_cluster_csr_restated():
    """hodge_dataset.pool_tables == the cluster CSR hodge_cheb_conv.cluster_mean
    builds on the device from pos = x[:, 0] + level offsets (inf -> the
    dropped bucket), restated with torch ops on the CPU (stable sort of the
    members by cluster), for a two-level list and its padded copy."""
    from hlhgat.hodge_dataset import level_caps, pad_levels, pool_tables
    from hlhgat.synthetic import two_level_batch
    raw = two_level_batch("cifar", 5, seed=3)
    pool_tables(raw)
    padded = pad_levels(raw, level_caps([raw], 128))
    for datas in (raw, padded):
        d0, d1 = datas
        for side, cnt in (("t", "num_node1"), ("s", "num_edge1")):
            x0 = getattr(d0, "x_" + side)[:, 0]
            n_seg = getattr(d1, "x_" + side).shape[0]
            counts = getattr(d0, cnt).long()
            ahead = torch.zeros(counts.numel(), dtype=torch.float32)
            ahead[1:] = torch.cumsum(getattr(d1, cnt).long(), 0)[:-1].float()
            n = x0.numel()
            tail = max(n - int(counts.sum()), 0)
            per = torch.repeat_interleave(torch.cat([ahead, torch.zeros(1)]),
                                          torch.cat([counts, torch.tensor([tail])]))[:n]
            pos = x0 + per
            idx = torch.where(torch.isinf(pos), torch.full_like(pos, float(n_seg)), pos).long()
            order = torch.sort(idx, stable=True).indices
            rowptr = torch.zeros(n_seg + 2, dtype=torch.int64)
            rowptr[1:] = torch.cumsum(torch.bincount(idx, minlength=n_seg + 1), 0)
            assert torch.equal(getattr(d0, "pool_rows_" + side), order.to(torch.int32)), side
            assert torch.equal(getattr(d0, "pool_rowptr_" + side), rowptr.to(torch.int32)), side
