/*
 * hlhgat.h — C-ABI of the MI355X-native (gfx950) Hodge-Laplacian
 * message-passing hot path of HL-HGAT.
 *
 * Every entry point takes plain device pointers, sizes and a HIP stream
 * (passed as void*), launches asynchronously on that stream and returns
 * HLHGAT_OK (0) or an error code; hlhgat_last_error() returns a
 * thread-local message for the last failure.  No entry point allocates
 * device memory or synchronises the stream (graph-capture safe); scratch
 * space is supplied by the caller (see the *_workspace_bytes queries).
 *
 * Layout conventions (DESIGN.md "Data layout in HBM"):
 *  - features are fp32, row-major [rows][ld] with ld >= width;
 *  - a sparse operator A (L0, L1, |B1|) is CSR with int32 rowptr[n+1],
 *    int32 col[nnz], fp32 val[nnz] (val == NULL means all ones);
 *  - a polynomial basis slab is k-major: block k is [n][F] contiguous.
 *
 * Reference interfaces replaced (paths relative to deepika090/HL-HGAT):
 *  - PyG MessagePassing.propagate + message(x_j, norm) = norm*x_j, aggr='add'
 *      lib/Hodge_Cheb_Conv.py:412,416,424,430,494,502,442-443,518-519
 *      -> hlhgat_csr_*, hlhgat_spmm, hlhgat_poly_step
 *  - HodgeLaguerreConv.forward recurrence   lib/Hodge_Cheb_Conv.py:480-515
 *  - HodgeChebConv.forward recurrence       lib/Hodge_Cheb_Conv.py:394-439
 *      -> hlhgat_poly_basis_fwd / hlhgat_poly_basis_bwd
 *  - torch_geometric Linear / nn.Linear projections (lins[k], WV_*, WQ/WK)
 *      lib/Hodge_Cheb_Conv.py:462-465,497,509,270-289,276-289
 *      -> hlhgat_proj_fwd / hlhgat_proj_bwd_data / hlhgat_proj_bwd_weight
 *  - adj2par1 + torch.sparse.mm(|B1|, .) and (|B1|^T, .)
 *      lib/Hodge_Dataset.py:169-191, lib/Hodge_Cheb_Conv.py:294-295,100-101
 *      -> hlhgat_incidence_csr, hlhgat_edge_gather2 (+ hlhgat_poly_step as
 *         the node-side segment mean)
 *  - NodeEdgeInt/MSI only_att score     lib/Hodge_Cheb_Conv.py:297-305,103-111
 *      -> hlhgat_att_score_fwd / hlhgat_att_score_bwd
 *  - torch_scatter.scatter_mean / global_mean_pool (cluster pooling, readout)
 *      lib/Hodge_Cheb_Conv.py:50-53, lib/Hodge_ST_Model.py:636
 *      -> hlhgat_segment_mean_fwd / hlhgat_segment_mean_bwd
 */
#ifndef HLHGAT_H_
#define HLHGAT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HLHGAT_OK 0
#define HLHGAT_EINVAL 1 /* bad argument (shape, alignment, null pointer) */
#define HLHGAT_EHIP 2   /* HIP runtime error */

#define HLHGAT_POLY_LAGUERRE 0 /* HodgeLaguerreConv recurrence */
#define HLHGAT_POLY_CHEB 1     /* HodgeChebConv recurrence */
/* HL-HGAT-DEMO HodgeLaguerreFastConv as published: its k >= 2 terms
 * propagate the layer input x instead of Tx_1
 * (HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py:561); needed to reproduce outputs of
 * models trained with it (HL-HGAT-DEMO/weights/HL_HGAT_Brain.pt). */
#define HLHGAT_POLY_LAGUERRE_DEMO 2

#define HLHGAT_SIGMA_SIGMOID 0 /* nn.Sigmoid (NodeEdgeInt default) */
#define HLHGAT_SIGMA_RELU 1    /* nn.ReLU (attpool heads) */

/* ---- library ---------------------------------------------------------- */
int hlhgat_version(void);
const char* hlhgat_last_error(void);

/* ---- CSR construction ------------------------------------------------- */
/* Scratch bytes needed by hlhgat_csr_from_coo for nnz entries. */
size_t hlhgat_csr_workspace_bytes(int64_t nnz);

/* COO (row[e], col[e], w[e]) -> CSR keyed by row.  Entries are ordered by
 * (row, col) exactly as torch.sparse coalesce orders them, duplicates kept
 * (propagate sums duplicates, so does the SpMM).  w may be NULL (val NULL).
 * Rows/cols are int64 (PyG edge_index); both must lie in [0,n_rows) and
 * [0,n_cols).  `perm` (optional, int32[nnz]) receives the source entry of
 * each CSR slot.  Replaces the gather/scatter set-up of PyG propagate
 * (lib/Hodge_Cheb_Conv.py:494,502) and the coalesce inside torch.sparse.mm
 * (lib/Hodge_Cheb_Conv.py:294-295). */
int hlhgat_csr_from_coo(const int64_t* row, const int64_t* col, const float* w,
                        int64_t nnz, int64_t n_rows, int64_t n_cols,
                        int32_t* rowptr, int32_t* col_out, float* val_out,
                        int32_t* perm, void* workspace, size_t workspace_bytes,
                        void* stream);

/* Fast path for COO already sorted by (row, col) — e.g. dense_to_sparse output
 * of the Hodge builder (lib/Hodge_Dataset.py:467-468) shifted by PairData
 * batching (lib/Hodge_Dataset.py:40-48).  Caller guarantees sortedness;
 * hlhgat_coo_check_sorted can verify it on device. */
int hlhgat_csr_from_sorted_coo(const int64_t* row, const int64_t* col,
                               const float* w, int64_t nnz, int64_t n_rows,
                               int32_t* rowptr, int32_t* col_out,
                               float* val_out, void* stream);

/* Writes 1 to *flag_dev if (row,col) is non-decreasing lexicographically and
 * every index is in range, else 0. */
int hlhgat_coo_check_sorted(const int64_t* row, const int64_t* col, int64_t nnz,
                            int64_t n_rows, int64_t n_cols, int32_t* flag_dev,
                            void* stream);

/* Incidence CSR of |B1| (adj2par1, lib/Hodge_Dataset.py:169-191): for each
 * node v, the edges e with edge_index[0][e]==v or edge_index[1][e]==v, in
 * increasing e.  edge_index is int64 [2][n_edges] (row 0 = i, row 1 = j).
 * Needs hlhgat_csr_workspace_bytes(2*n_edges) of scratch. */
int hlhgat_incidence_csr(const int64_t* edge_index, int64_t n_edges,
                         int64_t n_nodes, int32_t* rowptr, int32_t* edge_ids,
                         void* workspace, size_t workspace_bytes, void* stream);

/* ---- halo tiles (LDS-staged SpMM for large Laplacians) ----------------- */
/* A tiling of a CSR operator's rows for the LDS-staged SpMM: tile t owns the
 * schedule positions [tile_ptr[t], tile_ptr[t+1]) (rows order[p], order = the
 * operator's row schedule, NULL = natural) and the distinct columns those
 * rows reference, halo[halo_ptr[t] .. halo_ptr[t+1]) (ascending).  The
 * entries are re-laid in SCHEDULE order: position p's entries are
 * [srp[p], srp[p+1]) of lcol (tile-local column = index into the tile's
 * halo) and sval (the CSR values permuted the same way; NULL = all ones).
 * One workgroup stages a tile's entries and the halo rows of X in LDS with
 * bulk coalesced loads, then every row is summed from LDS: each X row is read
 * from L2 once per tile instead of once per entry (TSP-scale L1: ~20 entries
 * per row, ~5 uses per staged row).  Per-row summation order is the CSR
 * order, so results are bitwise those of the plain SpMM.  Built on the HOST
 * by hlhgat_halo_tiles; sval on device by hlhgat_gather_f32(val, eperm). */
typedef struct hlhgat_halo {
  const int32_t* hdr;       /* [n_tiles][8] {p0, rows, halo0, n_halo, e0, n_entries, 0, 0} */
  const int32_t* tile_ptr;  /* [n_tiles+1] schedule positions */
  const int32_t* halo_ptr;  /* [n_tiles+1] offsets into halo */
  const int32_t* halo;      /* distinct columns of each tile, ascending */
  const int32_t* srp;       /* [n_rows+1] entry offsets in schedule order */
  const uint16_t* lcol;     /* [nnz] tile-local column, schedule order */
  const float* sval;        /* [nnz] values, schedule order (NULL = ones) */
  int64_t n_tiles;
  int32_t max_halo;         /* bounds of any tile (size the LDS image) */
  int32_t max_rows;
  int32_t max_nnz;
} hlhgat_halo_t;

/* HOST function (host pointers, no stream): pack consecutive rows of the
 * schedule greedily into tiles of <= max_rows rows, <= max_nnz entries and
 * <= max_halo distinct columns.  Outputs (capacities): tile_ptr, halo_ptr and
 * srp n_rows+1; halo, lcol and eperm nnz (eperm[i] = CSR entry of
 * schedule-ordered entry i); hdr 8*n_rows (per-tile header, see
 * hlhgat_halo_t).  Returns HLHGAT_EINVAL if one row alone exceeds
 * max_halo columns or max_nnz entries (use the plain SpMM then). */
int hlhgat_halo_tiles(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                      int64_t n_cols, const int32_t* order, int32_t max_rows,
                      int32_t max_nnz, int32_t max_halo, int32_t* tile_ptr,
                      int32_t* halo_ptr, int32_t* halo, int32_t* srp, uint16_t* lcol,
                      int32_t* eperm, int32_t* hdr, int64_t* n_tiles, int64_t* n_halo);

/* ---- multi-level graph coarsening (HOST functions, host pointers) --------
 * hlhgat_graclus replaces the torch_cluster 1.6.0 graclus_cluster call of
 * MLGC / MLGC_weighted (lib/Hodge_Dataset.py:252-253, :311): greedy matching
 * over edge_index [2, n_edges] (row-major: rows then cols; self-loops
 * ignored; weight NULL = all ones) visiting nodes in perm order (the
 * reference draws torch.randperm; the caller passes its permutation), each
 * unmatched node paired with the last of its unmatched neighbours (ascending
 * column order) whose weight is >= the best so far, starting from 0 (the
 * weighted branch of torch_cluster's graclus_cpu: ties to the last, zero
 * weights match); both get id min(u, v), an unpaired node keeps id u.
 * cluster: [n_nodes] out. */
int hlhgat_graclus(const int64_t* edge_index, const double* weight, int64_t n_edges,
                   int64_t n_nodes, const int64_t* perm, int64_t* cluster);
/* hlhgat_mlgc_map replaces the per-edge loop of MLGC (lib/Hodge_Dataset.py:
 * 254-275, same at :312-333): c_node[u] = rank of cluster[u] among the
 * distinct ids; c_edge[i] = +inf if edge i's ends share a coarse node, else
 * the index of coarse edge (min, max) numbered in first-seen order, written
 * to coarse_edges [2, n_edges capacity] (row 0 = min at [0..), row 1 = max
 * at [n_edges..)).  Unlike the reference's float key imax + 1e-4 * imin,
 * pairs never collide (the reference's key does once a level has > 10^4
 * coarse nodes). */
int hlhgat_mlgc_map(const int64_t* cluster, int64_t n_nodes, const int64_t* edge_index,
                    int64_t n_edges, int64_t* c_node, float* c_edge, int64_t* coarse_edges,
                    int64_t* n_coarse_nodes, int64_t* n_coarse_edges);
/* One MLGC level for a batch of graphs, the per-sample work of the
 * reference's CIFAR10SP get() (main_cifar10SP_HL_HGCNN_dense_int3_attpool.py:
 * 94-103: MLGC on every sample): per graph g, hlhgat_graclus over its i<j
 * edge list taken both ways (unit weights, node order perm) then
 * hlhgat_mlgc_map over the i<j list, the graphs spread over n_threads host
 * threads.  Indices are local to each graph: its nodes are [node_ptr[g],
 * node_ptr[g+1]) of perm / c_node, its edges [edge_ptr[g], edge_ptr[g+1]) of
 * edges ([2][E], E = edge_ptr[n_graphs]) / c_edge; its coarse edges go to
 * columns [edge_ptr[g], edge_ptr[g] + coarse_e[g]) of coarse_edges ([2][E]);
 * coarse_n[g] = its coarse node count. */
int hlhgat_mlgc_batch(int64_t n_graphs, const int64_t* node_ptr, const int64_t* edge_ptr,
                      const int64_t* edges, const int64_t* perm, int n_threads, int64_t* c_node,
                      float* c_edge, int64_t* coarse_edges, int64_t* coarse_n,
                      int64_t* coarse_e);

/* ---- native data loader (HOST functions, host pointers) -----------------
 * Replaces the reference's per-step DataLoader collation of PairData
 * (lib/Hodge_Dataset.py:40-48; main_zinc_HL_HGCNN_dense_int3_pyr.py:223-225)
 * plus the batch tables the device step reads.  A packed dataset holds every
 * graph's arrays back to back (InMemoryDataset-style slices, graph-local
 * indices): */
typedef struct {
  int64_t n_graphs;
  const int64_t* node_ptr; /* [G+1] x_t rows (nodes) per graph, cumulative */
  const int64_t* edge_ptr; /* [G+1] x_s rows (edges) */
  const int64_t* lt_ptr;   /* [G+1] L0 COO entries */
  const int64_t* ls_ptr;   /* [G+1] L1 COO entries */
  const float* x_t;        /* [N][f_t] */
  int64_t f_t;
  const float* x_s;        /* [E][f_s] */
  int64_t f_s;
  const int32_t* lt_row;   /* L0 COO, graph-local node ids, row-sorted */
  const int32_t* lt_col;
  const float* lt_w;
  const int32_t* ls_row;   /* L1 COO, graph-local edge ids, row-sorted */
  const int32_t* ls_col;
  const float* ls_w;
  const int32_t* b1_src;   /* [E] B1 edge list (edge_index), graph-local */
  const int32_t* b1_dst;
  const float* y;          /* [G][y_dim] (y_dim 0: none) */
  int64_t y_dim;
} hlhgat_packed_graphs_t;
/* The collated batch: capacities in (rows_t, rows_s, nnz_t, nnz_s equal to
 * the batch's sizes = no padding; rows above them = hodge_dataset.pad_batch's
 * padding), caller-allocated outputs (the table pointers may be NULL to skip
 * a table); n_t / n_s out = the real rows. */
typedef struct {
  int64_t rows_t, rows_s, nnz_t, nnz_s;
  float* x_t;               /* [rows_t][f_t] */
  float* x_s;               /* [rows_s][f_s] */
  int64_t* edge_index_t;    /* [2][nnz_t] */
  float* edge_weight_t;     /* [nnz_t] */
  int64_t* edge_index_s;    /* [2][nnz_s] */
  float* edge_weight_s;     /* [nnz_s] */
  int64_t* edge_index;      /* [2][rows_s] */
  float* y;                 /* [B][y_dim] */
  int64_t* num_node1;       /* [B] */
  int64_t* num_edge1;       /* [B] */
  int32_t* csr_rowptr_t;    /* [rows_t+1] */
  int32_t* csr_col_t;       /* [nnz_t] */
  int32_t* csr_rowptr_s;    /* [rows_s+1] */
  int32_t* csr_col_s;       /* [nnz_s] */
  int32_t* inc_rowptr;      /* [rows_t+1] incidence CSR of |B1| */
  int32_t* inc_eids;        /* [2 rows_s] */
  float* deg_t;             /* [rows_t] degree (padding rows: 1) */
  float* inv_deg_t;         /* [rows_t] fp32 1 / degree */
  int32_t* seg_ptr_t;       /* [B+1] */
  int32_t* seg_ptr_s;       /* [B+1] */
  uint8_t* valid_mask_t;    /* [rows_t] row < n_t */
  int64_t n_t, n_s;         /* out */
} hlhgat_collated_t;
/* sizes[4] = (nodes, edges, L0 entries, L1 entries) of the graphs idx[0..n). */
int hlhgat_collate_sizes(const hlhgat_packed_graphs_t* d, const int64_t* idx, int64_t n_idx,
                         int64_t* sizes);
/* Collate graphs idx[0..B) (in that order) into *out: bitwise the arrays of
 * hodge_dataset.collate followed by pad_batch. */
int hlhgat_collate(const hlhgat_packed_graphs_t* d, const int64_t* idx, int64_t B,
                   hlhgat_collated_t* out);

/* dst[i] = src[idx[i]] for i < n (device; e.g. halo sval = val[eperm]). */
int hlhgat_gather_f32(const float* src, const int32_t* idx, int64_t n, float* dst,
                      void* stream);

/* ---- SpMM and fused polynomial step ----------------------------------- */
/* `halo` (optional, below) selects the LDS-staged kernel: see hlhgat_halo_t.
 * It must describe this operator with this row_order; NULL = plain kernel. */
/* Y = A·X (PyG propagate with aggr='add', source_to_target, when A is the
 * CSR keyed by edge_index[1]).  X,Y [n][d] with row strides ldx, ldy.
 * row_order (optional, int32[n_rows], a permutation) is the order in which
 * rows are SCHEDULED (e.g. hlhgat_locality_order): results are identical for
 * any order (each row's entries are still summed in CSR order); only which
 * rows share an XCD's L2 at a time changes.  NULL = natural order. */
int hlhgat_spmm(const int32_t* rowptr, const int32_t* col, const float* val,
                int64_t n_rows, int64_t nnz, const int32_t* row_order,
                const hlhgat_halo_t* halo, const float* X, int64_t ldx,
                int64_t d, float* Y, int64_t ldy, void* stream);

/* Generic fused step (one launch):
 *   Y = (alpha * rs[r] * (A·X)[r] + beta*X[r] + gamma*Z[r]) / div
 *       + p*P[r] + q*Q[r]
 * Z, P, Q, rs (row scale) may be NULL (term dropped).  Y may alias P (each
 * row is read then written by the same lanes).  A is n_rows x n_rows when
 * beta != 0; otherwise X may have any row count >= max(col)+1. */
int hlhgat_poly_step(const int32_t* rowptr, const int32_t* col,
                     const float* val, const float* rs, int64_t n_rows,
                     int64_t nnz, const int32_t* row_order,
                     const hlhgat_halo_t* halo, const float* X,
                     int64_t ldx, int64_t d,
                     const float* Z, int64_t ldz, const float* P, int64_t ldp,
                     const float* Q, int64_t ldq, float alpha, float beta,
                     float gamma, float div, float p, float q, float* Y,
                     int64_t ldy, void* stream);

/* hlhgat_poly_step over a rectangular incidence operator (rows: n_rows nodes;
 * columns: the n_src edges, each referenced by exactly two rows): the same
 * kernel, timed as HLHGAT_PROF_INCIDENCE with the gathered operand counted as
 * n_src rows (what it reads), not n_rows.  Y = alpha rs (A X) + gamma Z.  Replaces the torch.sparse.mm(|B1|, .) of
 * lib/Hodge_Cheb_Conv.py:294 (and the node-side adjoint of :295). */
int hlhgat_incidence_step(const int32_t* rowptr, const int32_t* col, const float* val,
                          const float* rs, int64_t n_rows, int64_t nnz, int64_t n_src,
                          const float* X, int64_t ldx, int64_t d, const float* Z, int64_t ldz,
                          float alpha, float gamma, float* Y, int64_t ldy, void* stream);

/* Polynomial basis T_1..T_{K-1} of X over A (K >= 1; K==1 is a no-op).
 * kind = HLHGAT_POLY_LAGUERRE: T_1 = X - A X,
 *        T_{k+1} = (-A T_k + (2k+1) T_k - k T_{k-1}) / (k+1)
 *        (lib/Hodge_Cheb_Conv.py:494,507)
 * kind = HLHGAT_POLY_CHEB:     T_1 = A X, T_{k+1} = 2 A T_k - T_{k-1}
 *        (lib/Hodge_Cheb_Conv.py:416,430-432)
 * kind = HLHGAT_POLY_LAGUERRE_DEMO: T_1 = X - A X,
 *        T_{k+1} = (-A X + (2k+1) T_k - k T_{k-1}) / (k+1)
 *        (HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py:554,561,566; K <= 16)
 * X: [n][F] row stride ldx.  T: (K-1) contiguous blocks of [n][F]. */
int hlhgat_poly_basis_fwd(int kind, const int32_t* rowptr, const int32_t* col,
                          const float* val, int64_t n, int64_t nnz,
                          const int32_t* row_order, const hlhgat_halo_t* halo,
                          const float* X, int64_t ldx, int64_t F, int K, float* T,
                          void* stream);

/* Adjoint of hlhgat_poly_basis_fwd.  On entry G holds K contiguous blocks
 * [n][F]: G_k = dLoss/dT_k from the consumers of each T_k (block 0 = the
 * direct gradient of X).  On exit block 0 holds dLoss/dX.  Blocks 1..K-1 are
 * used as scratch.  The CSR passed must be A^T (== A for the symmetric Hodge
 * Laplacians). */
int hlhgat_poly_basis_bwd(int kind, const int32_t* rowptr_t,
                          const int32_t* col_t, const float* val_t, int64_t n,
                          int64_t nnz, const int32_t* row_order,
                          const hlhgat_halo_t* halo, int64_t F,
                          int K, float* G, void* stream);

/* ---- Hodge-factored L1 (large, high-degree edge Laplacians) ------------ */
/* Every L1 the reference builds is 2 B1^T B1 / lmax in fp32
 * (lib/Hodge_Dataset.py:451-456, :780-799; MLGC :283-287): its entries are
 * fl(2 v / lmax) with v in {2, +-1}, so L1 = alpha_e * B1^T B1 EXACTLY, with
 * alpha_e = L1[e,e] / 2 (constant per graph).  Then
 *     L1 X = alpha * B1^T (B1 X):   Z = B1 X   (node rows: signed sum of the
 *                                              node's incident edge rows)
 *                                   Y[e] = alpha_e (Z[j] - Z[i])
 * which gathers ~4 feature rows per edge instead of nnz(L1)/E (~20 at
 * BASELINE config 5, ~18 at config 3).  Same real-arithmetic result as the
 * CSR SpMM; fp32 rounding differs (measured <= 3e-7 relative at config 5),
 * so this path is NOT bitwise equal to propagate; the CSR path is.  The
 * caller (hlhgat.ops.set_hodge_factor, checked on the host by
 * hodge_dataset.hodge_factor_ok) guarantees the identity. */
typedef struct hlhgat_hodge_factor {
  const int32_t* node_rowptr; /* [n_nodes+1] incidence CSR of B1 (node rows) */
  const int32_t* node_edge;   /* [2 n_edges] incident edge ids, ascending */
  const float* node_sign;     /* [2 n_edges] -1 (node = edge_index[0][e]) / +1 */
  const int32_t* node_order;  /* optional row schedule of the node rows */
  int64_t n_nodes;
  const int32_t* ends;        /* [n_edges][2] (edge_index[0][e], edge_index[1][e]) */
  const float* alpha;         /* [n_edges] L1[e,e] / 2 */
  const int32_t* edge_order;  /* optional row schedule of the edge rows */
  int64_t n_edges;
} hlhgat_hodge_factor_t;

/* Floats of scratch (Z = B1 X) the factored entry points need for width F. */
int64_t hlhgat_hodge_factor_work_floats(int64_t n_nodes, int64_t F);

/* Y = L1 X through the factorisation (two launches).  X, Y [n_edges][d]. */
int hlhgat_hodge_spmm(const hlhgat_hodge_factor_t* f, const float* X, int64_t ldx,
                      int64_t d, float* Y, int64_t ldy, float* work, void* stream);

/* hlhgat_poly_step with A = L1 factored: Y = (alpha (L1 X)[r] + beta X[r] +
 * gamma Z[r]) / div + p P[r] + q Q[r]  (two launches; no row scale). */
int hlhgat_hodge_poly_step(const hlhgat_hodge_factor_t* f, const float* X, int64_t ldx,
                           int64_t d, const float* Z, int64_t ldz, const float* P, int64_t ldp,
                           const float* Q, int64_t ldq, float alpha, float beta, float gamma,
                           float div, float p, float q, float* Y, int64_t ldy, float* work,
                           void* stream);

/* hlhgat_poly_basis_fwd / _bwd with every L1 application factored (each
 * step = one incidence launch + one fused edge-step launch whose epilogue is
 * the recurrence's).  L1 is symmetric, so the adjoint uses the same factor.
 * Replaces the same reference lines as hlhgat_poly_basis_fwd / _bwd. */
int hlhgat_poly_basis_fwd_factored(int kind, const hlhgat_hodge_factor_t* f,
                                   const float* X, int64_t ldx, int64_t F, int K, float* T,
                                   float* work, void* stream);
int hlhgat_poly_basis_bwd_factored(int kind, const hlhgat_hodge_factor_t* f, int64_t F,
                                   int K, float* G, float* work, void* stream);

/* ---- on-device Hodge Laplacian builder -------------- */
/* Replaces the per-graph dense construction of the reference
 * (lib/Hodge_Dataset.py:451-468, :780-799; DEMO notebook cells 11, 19):
 * par1 = adj2par1(...).to_dense(); L0 = par1 par1^T; lmax = eigh(L0).max();
 * L0 = 2 par1 par1^T / lmax; L1 = 2 par1^T par1 / lmax; dense_to_sparse.
 * Input: a block-diagonal batch's edge list (int64 [2][E], i < j per edge,
 * PairData offsets) and its incidence CSR (hlhgat_incidence_csr).
 *
 * hlhgat_hodge_lmax: lmax of every graph's L0 = B1 B1^T (graph g = nodes
 * [node_ptr[g], node_ptr[g+1])), one wave per graph (vectors and the local
 * adjacency in LDS when they fit in 48 KB), fp64 Lanczos by the three-term
 * recurrence with local re-orthogonalisation (`steps` <= 64 iterations; the
 * largest Ritz value converges first and loss of orthogonality only adds
 * ghost copies) and Sturm bisection of the tridiagonal matrix.  Workspace:
 * 3 n_nodes doubles (the vectors of graphs that miss the LDS).  The
 * reference's float32 eigh agrees to its own rounding (~1e-7 relative), so
 * entries built from this lmax may differ from the reference's by an ulp. */
int64_t hlhgat_hodge_lmax_workspace_bytes(int64_t n_nodes, int steps);
int hlhgat_hodge_lmax(const int32_t* inc_rowptr, const int32_t* inc_edge,
                      const int64_t* edge_index, int64_t n_edges, int64_t n_nodes,
                      const int64_t* node_ptr, int64_t n_graphs, int steps, double* lmax,
                      void* workspace, int64_t workspace_bytes, void* stream);
/* hlhgat_eig_pe: the eigenvector positional encodings of every graph of the
 * batch and its lambda_max in ONE launch, replacing the reference's per-sample
 * dense eighs (eig_pe, lib/Hodge_Dataset.py:97-112, called at
 * main_cifar10SP_HL_HGCNN_dense_int3_attpool.py:86-91 on L0 = 2 B1 B1^T / lmax,
 * and torch.linalg.eigh(L0).max(), lib/Hodge_Dataset.py:782).  Per graph, one
 * workgroup, fp64: Lanczos with full re-orthogonalisation (restarted when an
 * invariant subspace closes), eigenvalues of the tridiagonal matrix by Sturm
 * multisection, its eigenvectors by inverse iteration, pe = Q y.  Output:
 * pe[v][0 .. k-2] (float32, row stride ldpe) = eigenvectors 1 .. k-1 of the
 * unscaled L0 = B1 B1^T (ascending eigenvalues; the same vectors as the
 * scaled L0's), zero columns where the graph has fewer than k nodes;
 * lmax[g] = the largest eigenvalue of the unscaled L0 (fp64).  Eigenvectors
 * are defined up to sign (and rotation within equal eigenvalues).
 * max_nodes >= every graph's node count (sizes the workspace slice a graph
 * too large for the LDS uses: one slice per workgroup, min(n_graphs, CUs)
 * workgroups, so the size depends on the current device); 2 <= k <= 64. */
int64_t hlhgat_eig_pe_workspace_bytes(int64_t n_graphs, int64_t max_nodes, int k);
int hlhgat_eig_pe(const int32_t* inc_rowptr, const int32_t* inc_edge, const int64_t* edge_index,
                  int64_t n_edges, int64_t n_nodes, const int64_t* node_ptr, int64_t n_graphs,
                  int64_t max_nodes, int k, float* pe, int64_t ldpe, double* lmax,
                  void* workspace, int64_t workspace_bytes, void* stream);
/* Row sizes of L0 (deg(v) + 1, 0 for an isolated node) and L1 (deg(i) +
 * deg(j) - 1); exclusive-scan them into the row pointers. */
int hlhgat_hodge_row_sizes(const int32_t* inc_rowptr, const int64_t* edge_index,
                           int64_t n_edges, int64_t n_nodes, int32_t* sizes_l0,
                           int32_t* sizes_l1, void* stream);
/* L0 / L1 in CSR, columns ascending, entries fl(fl(2 v) / lam_node[row's
 * graph]) -- the reference's float32 arithmetic -- with v the integer entry
 * of B1 B1^T (deg, -1) / B1^T B1 (2, +1 same-end, -1 tail-to-head).
 * cap_l0 / cap_l1 = the entries col_l* / val_l* hold: a row that would end
 * past them (row pointers sized for a simple graph given a multigraph)
 * writes nothing and raises HLHGAT_DEVERR_HODGE_SIZE. */
int hlhgat_hodge_build(const int32_t* inc_rowptr, const int32_t* inc_edge,
                       const int64_t* edge_index, int64_t n_edges, int64_t n_nodes,
                       const float* lam_node, const int32_t* rowptr_l0, int32_t* col_l0,
                       float* val_l0, int64_t cap_l0, const int32_t* rowptr_l1,
                       int32_t* col_l1, float* val_l1, int64_t cap_l1, void* stream);

/* ---- dense per-simplex projections (fp32 MFMA) ------------------------ */
#define HLHGAT_MAX_BLOCKS 16

/* Forward:  C[m][n] = beta_acc*C[m][n] + sum_b sum_k A_b[m][k]*W_b[n][k]
 *                     + bias[n]
 * A_b: [M][kb[b]] row stride lda[b]; W_b: [N][kb[b]] row stride ldw[b]
 * (nn.Linear weight layout).  accumulate != 0 adds into C.  bias may be NULL.
 * Replaces out = sum_k lins[k](T_k) + bias (lib/Hodge_Cheb_Conv.py:487,497,
 * 509,512-513) and Linear(cat[a,b]) (lib/Hodge_Cheb_Conv.py:307-308). */
int hlhgat_proj_fwd(int nblocks, const float* const* A, const int64_t* lda,
                    const float* const* W, const int64_t* ldw,
                    const int64_t* kb, int64_t M, int64_t N, const float* bias,
                    float* C, int64_t ldc, int accumulate, void* stream);

/* Data gradient:  dA_b[m][k] (+)= sum_n dC[m][n] * W_b[n][k]. */
int hlhgat_proj_bwd_data(int nblocks, const float* dC, int64_t lddc,
                         const float* const* W, const int64_t* ldw,
                         const int64_t* kb, int64_t M, int64_t N,
                         float* const* dA, const int64_t* ldda,
                         int accumulate, void* stream);

/* Scratch floats needed by hlhgat_proj_bwd_weight. */
int64_t hlhgat_proj_bwd_weight_workspace_floats(int nblocks, const int64_t* kb,
                                                int64_t M, int64_t N,
                                                int with_bias);

/* Weight / bias gradient (deterministic split-M reduction, no atomics):
 *   dW_b[n][k] (+)= sum_m dC[m][n] * A_b[m][k];   dbias[n] (+)= sum_m dC[m][n]
 * dbias may be NULL. */
int hlhgat_proj_bwd_weight(int nblocks, const float* dC, int64_t lddc,
                           const float* const* A, const int64_t* lda,
                           const int64_t* kb, int64_t M, int64_t N,
                           float* const* dW, const int64_t* lddw, float* dbias,
                           int accumulate, float* workspace,
                           int64_t workspace_floats, void* stream);

/* The Linear backward (torch.nn.Linear / the HodgeLaguerreConv projections,
 * lib/Hodge_Cheb_Conv.py:63-66 backward) in two launches when the operands are
 * 16-B aligned: the weight / bias gradient's split partials of
 * hlhgat_proj_bwd_weight (nb_w blocks; `workspace` sized by
 * hlhgat_proj_bwd_weight_workspace_floats) together with the data gradient of
 * hlhgat_proj_bwd_data (nb_d blocks) in one, then the split reduction;
 * bit-identical to those two calls; either side may be empty (nb = 0).
 * Unaligned operands fall back to the two calls.  The weight gradient is
 * written (accumulate = 0); accumulate_d != 0 adds the data gradient into
 * dA (e.g. straight into the gradient slab of the dense concatenation,
 * hlhgat.ops.DenseConcat). */
int hlhgat_proj_bwd(int64_t M, int64_t N, const float* dC, int64_t lddc,
                    int nb_w, const float* const* A, const int64_t* lda,
                    const int64_t* kb_w, float* const* dW, const int64_t* lddw,
                    float* dbias, int nb_d, const float* const* W,
                    const int64_t* ldw, const int64_t* kb_d, float* const* dA,
                    const int64_t* ldda, int accumulate_d, float* workspace,
                    int64_t workspace_floats, void* stream);

/* Deferred split reduction.  hlhgat_proj_bwd_defer is hlhgat_proj_bwd whose
 * weight-gradient split reduction may be handed back instead of launched:
 *   - defer_out != NULL and the one-launch path is taken: the reduction is
 *     NOT launched; its descriptor goes to *defer_out and *deferred = 1.  The
 *     caller must keep `workspace` alive and run the descriptor (merge it into
 *     a later call on the same stream, or hlhgat_reduce_run) before anything
 *     reads dW / dbias;
 *   - merge != NULL: a descriptor deferred earlier ON THE SAME STREAM; its
 *     reduction runs as extra workgroups of this call's launch (or as its own
 *     launch first when this call cannot take the one-launch path).
 * The reduction itself is unchanged, so dW / dbias are bitwise those of
 * hlhgat_proj_bwd; what goes away is one dependent launch per Linear
 * backward on the stream's chain. */
typedef struct {
  int64_t words[160];
} hlhgat_reduce_desc_t;
int hlhgat_proj_bwd_defer(int64_t M, int64_t N, const float* dC, int64_t lddc, int nb_w,
                          const float* const* A, const int64_t* lda, const int64_t* kb_w,
                          float* const* dW, const int64_t* lddw, float* dbias, int nb_d,
                          const float* const* W, const int64_t* ldw, const int64_t* kb_d,
                          float* const* dA, const int64_t* ldda, int accumulate_d,
                          float* workspace, int64_t workspace_floats,
                          const hlhgat_reduce_desc_t* merge, hlhgat_reduce_desc_t* defer_out,
                          int* deferred, void* stream);
int hlhgat_reduce_run(const hlhgat_reduce_desc_t* desc, void* stream);

/* ---- boundary-operator interaction ------------------------------------ */
/* out[e] = ca*sa[i]*x[i] + cb*sb[j]*x[j] (+ z[e]) (+ out[e] if accumulate)
 * with (i,j) = edge_index[:,e] (sa/sb per-node scale vectors, z a per-edge
 * addend [n_edges][ldz]; each may be NULL).  With ca=cb=0.5 and no scales
 * this is x_t2s = (|B1|^T x_t)/2 (lib/Hodge_Cheb_Conv.py:295). */
int hlhgat_edge_gather2(const int64_t* edge_index, int64_t n_edges,
                        const float* x, int64_t ldx, int64_t d, const float* sa,
                        const float* sb, float ca, float cb, const float* z,
                        int64_t ldz, float* out, int64_t ldo, int accumulate,
                        void* stream);

/* The TSP edge readout x_t2s = |B1^T x_t| / 2 (lib/Hodge_ST_Model.py:846-848)
 * with g == NULL: out[e] = |x[j] - x[i]| / 2 for edge e = (i, j)
 * (edge_index [2][n_edges]); with g: its backward's edge factor
 * out[e] = (g[e] / 2) * sgn(x[j] - x[i]) (then B1 out, hlhgat_poly_step on
 * the signed incidence CSR, gives dx).  Bitwise the unfused
 * sparse.mm / abs / div and their backwards. */
int hlhgat_edge_absdiff(const int64_t* edge_index, int64_t n_edges, const float* x,
                        int64_t ldx, int64_t d, const float* g, int64_t ldg, float* out,
                        int64_t ldo, void* stream);

/* ---- attention score (NodeEdgeInt only_att) ---------------------------- */
/* a[r] = sigma((w_cross*<Qc[r],Kr[r]> + w_self*<Qs[r],Kr[r]>) / sqrt_dk)
 * with w_cross = (1-lambda), w_self = lambda (lib/Hodge_Cheb_Conv.py:299-304).
 * Qc, Qs, Kr: [n][dk] with row strides. */
int hlhgat_att_score_fwd(int64_t n, int64_t dk, const float* Qc, int64_t ldqc,
                         const float* Qs, int64_t ldqs, const float* Kr,
                         int64_t ldk, float w_cross, float w_self,
                         float sqrt_dk, int sigma, float* a, void* stream);

/* Backward of hlhgat_att_score_fwd given a (the forward output) and da. */
int hlhgat_att_score_bwd(int64_t n, int64_t dk, const float* Qc, int64_t ldqc,
                         const float* Qs, int64_t ldqs, const float* Kr,
                         int64_t ldk, float w_cross, float w_self,
                         float sqrt_dk, int sigma, const float* a,
                         const float* da, float* dQc, float* dQs, float* dK,
                         int64_t ldg, void* stream);

/* The NEAtt product x0 * att of the attention-pooling heads
 * (main_pepfunc_HL_HGCNN_dense_int3_attpool.py:134-136, lib/Hodge_ST_Model.py:
 * 276-280): y[r][:] = x[r][:] * a[r] over n rows of d features (y may be a
 * column block of a wider slab, ldy). */
int hlhgat_row_scale_fwd(int64_t n, int64_t d, const float* x, int64_t ldx,
                         const float* a, float* y, int64_t ldy, void* stream);
/* Its backward in one pass: dx[r][:] = dy[r][:] * a[r] and
 * da[r] = sum_j dy[r][j] * x[r][j]. */
int hlhgat_row_scale_bwd(int64_t n, int64_t d, const float* x, int64_t ldx,
                         const float* a, const float* dy, int64_t lddy, float* dx,
                         int64_t lddx, float* da, void* stream);

/* ---- segment mean (scatter_mean / global_mean_pool) -------------------- */
/* out[s] = mean over rows r of CSR segment s of x[r] (rows listed in
 * seg_rows, or contiguous when seg_rows == NULL); empty segments give 0. */
int hlhgat_segment_mean_fwd(const int32_t* seg_ptr, const int32_t* seg_rows,
                            int64_t n_seg, const float* x, int64_t ldx,
                            int64_t d, float* out, int64_t ldo, void* stream);
/* dx[r] = dout[seg(r)] / |seg| for every row r of a segment.  Contiguous
 * segments (seg_rows NULL): rows [0, seg_ptr[0]) and [seg_ptr[n_seg], n_rows)
 * of dx get exact zeros (global_mean_pool's adjoint, lib/Hodge_ST_Model.py:636),
 * so every one of the n_rows rows is written.  Listed members (scatter_mean):
 * n_rows is ignored and rows in no segment are left untouched (caller
 * zero-fills). */
int hlhgat_segment_mean_bwd(const int32_t* seg_ptr, const int32_t* seg_rows,
                            int64_t n_seg, const float* dout, int64_t ldo,
                            int64_t d, float* dx, int64_t ldx, int64_t n_rows,
                            void* stream);

/* Backward of the MLGC cluster pooling (scatter_mean over pos_ts / pos_ss,
 * lib/Hodge_ST_Model.py:1066-1069) from the pool tables
 * (hlhgat.hodge_dataset.pool_tables): seg_ptr has n_seg + 2 entries and its
 * extra segment n_seg lists the rows in no cluster (inf cluster id: padding
 * rows, edges between clusters), so seg_rows[0 .. seg_ptr[n_seg+1]) is a
 * permutation of the n_rows rows.  dx[r] = dout[s] / |s| for a member of
 * cluster s, exact zeros for the extra segment's rows: every row of dx is
 * written (no caller zero fill). */
int hlhgat_pool_mean_bwd(const int32_t* seg_ptr, const int32_t* seg_rows,
                         int64_t n_seg, const float* dout, int64_t ldo,
                         int64_t d, float* dx, int64_t ldx, int64_t n_rows,
                         void* stream);

/* ---- BatchNorm1d (training) + optional fused ReLU ---------------------- */
/* gnn.BatchNorm / nn.BatchNorm1d in training mode over x [n][C] (batch
 * statistics, biased variance for normalisation, unbiased for the running
 * update, momentum as torch), followed by ReLU when relu != 0 — the
 * conv -> BatchNorm -> ReLU tail of every HL block (lib/Hodge_ST_Model.py:
 * 556-566) and of NodeEdgeInt's WV_* MLPs (lib/Hodge_Cheb_Conv.py:276-289).
 * weight/bias may be NULL (affine=False); running stats may be NULL.
 * The workspace must be zero-filled before its first use and must not be
 * shared by launches that run concurrently; the kernels leave it reusable. */
int64_t hlhgat_bn_workspace_bytes(int64_t n, int64_t C);
/* n_valid (optional, device int32 scalar): rows >= *n_valid are capacity
 * padding of a static-shape batch: excluded from the statistics, their
 * outputs (and, backward, input gradients) written as 0.  NULL = all n. */
/* Eval-mode BatchNorm1d (+ ReLU) from the running statistics, one launch:
 * y = relu?((x - running_mean) * (w / sqrt(running_var + eps)) + b).  Replaces
 * torch's eval-mode batch_norm (+ relu) in the reference's test() loops
 * (lib/Hodge_ST_Model.py:556-566 under model.eval(); main_zinc...:165-177).
 * weight / bias may be NULL (1 / 0). */
int hlhgat_bn_apply_running(const float* x, int64_t ldx, int64_t n, int64_t C,
                            const float* weight, const float* bias, const float* running_mean,
                            const float* running_var, float eps, int relu, float* y,
                            int64_t ldy, void* stream);
int hlhgat_bn_fwd_train(const float* x, int64_t ldx, int64_t n,
                        const int32_t* n_valid, int64_t C,
                        const float* weight, const float* bias,
                        float* running_mean, float* running_var,
                        int64_t* num_batches_tracked, float momentum, float eps,
                        int relu, float* y, int64_t ldy, float* save_mean,
                        float* save_invstd, void* workspace,
                        int64_t workspace_bytes, void* stream);
/* Backward; y (the forward output) supplies the ReLU mask, NULL if no ReLU.
 * dweight/dbias may be NULL. */
/* The two halves of hlhgat_bn_fwd_train: statistics only (save_mean /
 * save_invstd, running stats, num_batches_tracked) and apply only
 * (y = relu?(x * s + t) with s = weight * invstd, t = bias - mean * s; rows
 * >= *n_valid written as 0). */
int hlhgat_bn_stats_train(const float* x, int64_t ldx, int64_t n, const int32_t* n_valid,
                          int64_t C, float* running_mean, float* running_var,
                          int64_t* num_batches_tracked, float momentum, float eps,
                          float* save_mean, float* save_invstd, void* workspace,
                          int64_t workspace_bytes, void* stream);
int hlhgat_bn_apply(const float* x, int64_t ldx, int64_t n, const int32_t* n_valid, int64_t C,
                    const float* weight, const float* bias, const float* save_mean,
                    const float* save_invstd, int relu, float* y, int64_t ldy, void* stream);

/* BatchNorm forward statistics and normalisation in one launch
 * (k_bn_fwd_grid: rows held in registers while the finalising workgroup --
 * the last to arrive -- publishes the statistics) or as two; default 1 (env
 * HLHGAT_BN_ONE_LAUNCH=0 turns it off).  Both give bitwise the same results.
 * The one launch is taken when its grid (<= 256 workgroups) is at most half
 * of the device's resident-workgroup capacity for it.  It assumes nothing
 * about residency: a workgroup waits for the statistics at most
 * hlhgat_set_bn_wait_us microseconds, then hands its rows to the finaliser
 * and exits (the finaliser normalises them from x with the same operations),
 * so the launch completes with the same bits beside any other kernels. */
/* Projection + BatchNorm1d (+ ReLU) forward, training mode: the
 * hlhgat_proj_fwd GEMM x = sum_b A_b W_b^T + bias (stored to x: the backward
 * reads it), then hlhgat_bn_fwd_train on x into y -- in ONE launch
 * (k_proj_bn_fwd: the projection's workgroups finish the BatchNorm from
 * their registers after a bounded grid-wide reduction) when N % 64 == 0, the
 * operands are 16-B aligned with ld % 4 == 0, ceil(M / 64) <= 512 and the
 * grid fits half of the chip's resident capacity; otherwise the two calls.
 * Its wait is bounded like k_bn_fwd_grid's: a workgroup that gives up leaves
 * its tile to the finaliser, which normalises it from the stored x.
 * Replaces Linear -> BatchNorm1d -> ReLU and HodgeLaguerreConv -> BatchNorm
 * -> ReLU (lib/Hodge_Cheb_Conv.py:276-289, lib/Hodge_ST_Model.py:556-566).
 * Statistics equal the two-call path's to fp64 summation order (not
 * bitwise).  Workspace: hlhgat_bn_workspace_bytes(M, N). */
int hlhgat_proj_bn_fwd(int nblocks, const float* const* A, const int64_t* lda,
                       const float* const* W, const int64_t* ldw, const int64_t* kb, int64_t M,
                       int64_t N, const float* bias, float* x, int64_t ldx,
                       const int32_t* n_valid, const float* bn_weight, const float* bn_bias,
                       float* running_mean, float* running_var, int64_t* num_batches_tracked,
                       float momentum, float eps, int relu, float* y, int64_t ldy,
                       float* save_mean, float* save_invstd, void* workspace,
                       int64_t workspace_bytes, void* stream);
/* Large-tile projection kernels (128 x 128 workgroup tiles, 2 x 2 32x32x2
 * MFMA accumulators per wave; the config 3-5 shapes): mode 0 = never (the
 * default: slower inside the measured two-chain steps),
 * -1 = by shape (per-operation rules from the config-5 census; min_m rows at
 * least, default 32769, env HLHGAT_GEMM_BIG_MIN_M), 1 = every 16-B aligned
 * shape.  Env HLHGAT_GEMM_BIG sets the initial mode.  min_m <= 0 keeps the
 * current threshold. */
int hlhgat_set_gemm_big(int mode, int64_t min_m);
/* 0: the fused Linear backward (hlhgat_proj_bwd / _defer) uses one
 * data-gradient workgroup per (row block, 64-column tile) instead of one per
 * row block covering every column tile (N <= 64); bitwise the same (tests). */
int hlhgat_set_proj_bwd_rows(int on);
/* 0: hlhgat_proj_bn_fwd always takes the two-call path (tests). */
int hlhgat_set_proj_bn_fused(int on);
/* 1: hlhgat_proj_bn_fwd's fused path as two launches -- the projection with
 * the statistics in its epilogue (its last workgroup finalises them; no
 * workgroup waits), then the BatchNorm apply over x -- bitwise the same y. */
int hlhgat_set_proj_bn_split(int on);
/* Diagnostics: k_proj_bn_fwd stamps s_memrealtime (100 MHz) into buf, 8
 * words per workgroup (blockIdx.y * gridDim.x + blockIdx.x): start, main loop
 * done, partials written, group level done, statistics known (finaliser:
 * generation bumped; others: poll returned), y stored, flags (1: last of its
 * group, 2: finaliser); launches whose grid needs more than `words` words
 * stamp nothing.  buf = NULL, words = 0: off (default). */
int hlhgat_set_proj_bn_stamps(void* buf, int64_t words);
/* Workgroups k_proj_bn_fwd may use (half of the resident capacity). */
int hlhgat_proj_bn_fused_capacity(int64_t* out);
int hlhgat_set_bn_one_launch(int on);
int hlhgat_get_bn_one_launch(void);
/* Microseconds a one-launch BatchNorm workgroup waits for its tile's
 * statistics before it hands its rows to the finaliser (default 1000; 0 =
 * hand over at once unless already final: a test hook that forces the
 * hand-over path, bitwise the same results). */
int hlhgat_set_bn_wait_us(unsigned wait_us);

/* Times a one-launch BatchNorm workgroup gave up waiting for its tile's
 * statistics (and handed its rows over): reads the device counter
 * (synchronising). */
int hlhgat_bn_wait_timeouts(unsigned* out);
/* The first HLHGAT_BN_LOG_MAX give-ups since the last reset, as recorded by
 * the workgroup that gave up: *logged = give-ups recorded in all (may exceed
 * what is copied); out[0 .. min(*logged, max, HLHGAT_BN_LOG_MAX)). */
#define HLHGAT_BN_LOG_MAX 64
typedef struct {
  uint32_t kernel;    /* 1 = k_bn_fwd_grid, 2 = k_proj_bn_fwd */
  uint32_t tile;      /* column tile (blockIdx.y) */
  uint32_t block;     /* row partition / row block (blockIdx.x) */
  uint32_t total;     /* arrivals the finaliser needs (workgroups; groups for k_proj_bn_fwd) */
  uint32_t arrivals;  /* arrivals counted when the wait ran out */
  uint32_t gen0;      /* the tile's generation when the workgroup arrived */
  uint32_t gen_seen;  /* the generation read after giving up */
  uint32_t wait_us;   /* the wait bound in force */
  uint32_t outcome;   /* 1 = reclaimed its rows (final by then), 2 = handed to the finaliser */
} hlhgat_bn_giveup_t;
int hlhgat_bn_giveup_log(hlhgat_bn_giveup_t* out, int max, int* logged);
/* Zero the give-up counter and log (synchronises the device). */
int hlhgat_bn_giveup_reset(void);

/* The reduction half of hlhgat_bn_bwd_train: dweight, dbias and dx's
 * coefficients coef[3][C] (A, B, C of dx = A g + (B (x - mean) + C)), for a
 * consumer that forms dx itself. */
int hlhgat_bn_bwd_reduce(const float* x, int64_t ldx, const float* y, int64_t ldy,
                         const float* dy, int64_t lddy, int64_t n, const int32_t* n_valid,
                         int64_t C, const float* weight, const float* save_mean,
                         const float* save_invstd, float* coef, float* dweight, float* dbias,
                         void* workspace, int64_t workspace_bytes, void* stream);
int hlhgat_bn_bwd_train(const float* x, int64_t ldx, const float* y, int64_t ldy,
                        const float* dy, int64_t lddy, int64_t n,
                        const int32_t* n_valid, int64_t C,
                        const float* weight, const float* save_mean,
                        const float* save_invstd, float* dx, int64_t lddx,
                        float* dweight, float* dbias, void* workspace,
                        int64_t workspace_bytes, void* stream);

/* ---- SyncBatchNorm (batch statistics over every data-parallel rank) ----- */
/* torch.nn.SyncBatchNorm semantics for the BatchNorm1d layers of the path
 * (lib/Hodge_ST_Model.py:556-566, lib/Hodge_Cheb_Conv.py:276-289) when the
 * batch is sharded by graph over ranks (parity caveat 1):
 *   1. hlhgat_bn_sums_fwd: this rank's fp64 column sums into
 *      sums[hlhgat_bn_sums_len(C)] = [S0[C] = sum x, S1[C] = sum x^2, n_valid];
 *   2. the caller all-gathers them into gathered[world][2C+1] (RCCL);
 *   3. hlhgat_bn_sync_fwd_apply: every rank totals the gathered sums in rank
 *      order (fp64), finishes mean / invstd / running statistics exactly as
 *      hlhgat_bn_fwd_train does and writes y.
 * Backward: hlhgat_bn_sums_bwd (sum g, sum g (x - mean) with g = dy masked
 * by the ReLU of y; this rank's dweight / dbias, which data-parallel
 * gradient averaging then combines as torch's SyncBatchNorm does), all-gather,
 * hlhgat_bn_sync_bwd_apply (dx with the global sums and count).  y / dx of
 * the _sums_ calls only select the layout (pass the tensors the apply will
 * use): with one rank the results are bitwise those of hlhgat_bn_fwd_train /
 * hlhgat_bn_bwd_train.  The workspace is hlhgat_bn_workspace_bytes' one. */
int64_t hlhgat_bn_sums_len(int64_t C);
int hlhgat_bn_sums_fwd(const float* x, int64_t ldx, const float* y, int64_t ldy, int64_t n,
                       const int32_t* n_valid, int64_t C, double* sums, void* workspace,
                       int64_t workspace_bytes, void* stream);
int hlhgat_bn_sync_fwd_apply(const float* x, int64_t ldx, int64_t n, const int32_t* n_valid,
                             int64_t C, const double* gathered, int world, const float* weight,
                             const float* bias, float* running_mean, float* running_var,
                             int64_t* num_batches_tracked, float momentum, float eps, int relu,
                             float* y, int64_t ldy, float* save_mean, float* save_invstd,
                             void* stream);
int hlhgat_bn_sums_bwd(const float* x, int64_t ldx, const float* y, int64_t ldy,
                       const float* dy, int64_t lddy, float* dx_layout, int64_t lddx, int64_t n,
                       const int32_t* n_valid, int64_t C, const float* save_mean,
                       const float* save_invstd, double* sums, float* dweight, float* dbias,
                       void* workspace, int64_t workspace_bytes, void* stream);
int hlhgat_bn_sync_bwd_apply(const float* x, int64_t ldx, const float* y, int64_t ldy,
                             const float* dy, int64_t lddy, int64_t n, const int32_t* n_valid,
                             int64_t C, const float* weight, const float* save_mean,
                             const float* save_invstd, const double* gathered, int world,
                             float* dx, int64_t lddx, void* stream);

/* ---- optimizer ------------------------------------------------------------ */
/* torch.optim.Adam (fused, capturable; L2 weight decay added to the gradient)
 * on ONE flat fp32 parameter buffer of n elements (hlhgat.train.TrainStep
 * keeps every parameter there), the reference's optimiser
 * (main_zinc_*.py).  `step` is the device fp32 step count: the update uses
 * step + 1, as torch increments it before the update, and a one-thread
 * launch then stores it.  Same double-precision hyper-parameter arithmetic
 * as torch's fused Adam (up to FMA contraction). */
int hlhgat_adam_flat(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                     int64_t n, float* step, double lr, double beta1, double beta2, double eps,
                     double weight_decay, void* stream);
/* The same update split around the step's backward, one launch fewer:
 * hlhgat_adam_prepare (at the start of the step) zeroes the n-element
 * gradient buffer and increments `step`; hlhgat_adam_flat_prepared (after the
 * backward) is hlhgat_adam_flat using `step` as already incremented.  The
 * pair gives the bits of zeroing the gradient + hlhgat_adam_flat. */
int hlhgat_adam_prepare(float* grad, int64_t n, float* step, void* stream);
int hlhgat_adam_flat_prepared(float* param, const float* grad, float* exp_avg,
                              float* exp_avg_sq, int64_t n, const float* step, double lr,
                              double beta1, double beta2, double eps, double weight_decay,
                              void* stream);

/* L1 loss, torch.nn.L1Loss(reduction="mean") of the ZINC training loop
 * (torch's sub / abs / mean and its five backward launches):
 *   fwd: loss[0] = sum_i |x_i - y_i| / n   (one workgroup, fixed order);
 *   bwd: dx_i = (gout[0] / n) * sgn(x_i - y_i), torch's MeanBackward then
 *        AbsBackward arithmetic (sgn(0) = sgn(NaN) = 0): bitwise torch's dx.
 * gout is a device scalar (the upstream gradient of the loss). */
int hlhgat_l1_loss_fwd(const float* x, const float* y, int64_t n, float* loss, void* stream);
int hlhgat_l1_loss_bwd(const float* x, const float* y, int64_t n, const float* gout, float* dx,
                       void* stream);

/* BCE with logits, torch.nn.BCEWithLogitsLoss (no weight / pos_weight) of the
 * peptides-func and TSP loops (main_pepfunc...:181-183, main_TSP...:316-321):
 * loss = sum_i ((1 - y_i) x_i - log_sigmoid(x_i)) / div (div = n: "mean",
 * 1: "sum"), one workgroup, fixed summation order; backward
 * dx = (g / div) (sigmoid(x) - y) in ATen's MulBackward + LogSigmoidBackward
 * arithmetic.  One launch each way. */
int hlhgat_bce_logits_fwd(const float* x, const float* y, int64_t n, float div, float* loss,
                          void* stream);
int hlhgat_bce_logits_bwd(const float* x, const float* y, int64_t n, float div,
                          const float* gout, float* dx, void* stream);

/* ---- workspaces --------------------------------------------------------- */
/* Zero `bytes` (a multiple of 4) at p with a kernel on `stream` (graph-capture
 * safe; used to initialise the BatchNorm workspace counters). */
int hlhgat_zero_fill(void* p, size_t bytes, void* stream);

/* n <= HLHGAT_MAX_COPY_BLOCKS strided fp32 rectangles in ONE launch:
 * dst[b][r*ldd[b] + c] = src[b] ? src[b][r*lds[b] + c] : 0, r < rows[b],
 * c < cols[b].  Packs the NodeEdgeInt first-Linear weights (replaces the
 * torch.cat of lib/Hodge_Cheb_Conv.py:307-308's split weight blocks). */
#define HLHGAT_MAX_COPY_BLOCKS 64
int hlhgat_copy2d_batched(int n, const float* const* src, const int64_t* lds,
                          float* const* dst, const int64_t* ldd, const int64_t* rows,
                          const int64_t* cols, void* stream);

/* ---- device error word ------------------------------------------------- */
/* A host-visible (pinned, mapped) word that kernels raise bits in when they
 * detect a condition whose results must not be used.  Reading it does not
 * synchronise: it shows what kernels that have completed so far reported
 * (callers synchronise first for an exact answer).  hlhgat.ops.
 * check_device_errors / hlhgat.train.TrainStep raise RuntimeError on it. */
/* a BatchNorm arrival counter was found beyond its total (its workspace was
 * written by something else, or shared by concurrent launches): that launch's
 * statistics are not trusted */
#define HLHGAT_DEVERR_BN_STATE 1u
/* hlhgat_hodge_build: a row of L0 / L1 would end past the buffers the caller
 * sized (the row pointers do not describe a simple graph's Laplacians) */
#define HLHGAT_DEVERR_HODGE_SIZE 2u
int hlhgat_device_errors(unsigned* out);
int hlhgat_clear_device_errors(void);

/* ---- streams ------------------------------------------------------------ */
/* A HIP stream of the library's own on `device` (the capture, copy and side
 * streams of hlhgat.train.TrainStep / hlhgat.loader.StagedFeed / the node and
 * edge chains: never one of torch's round-robin pool streams, which two
 * unrelated users can be handed at once).  Created by the HIP runtime this
 * library is linked against -- the one torch loaded (same SONAME), so the
 * handle is valid in torch.cuda.ExternalStream.  cu_mask_words > 0: the stream
 * runs only on the CUs whose bits are set (hipExtStreamCreateWithCUMask; bit
 * c of word c/32 = CU c; the words must cover every CU of the device) -- the
 * config-3 per-sample producer's stream (hlhgat.pipeline), so the replayed
 * step keeps the other CUs.  flags: hipStreamNonBlocking (1) etc., unmasked
 * streams only; priority != 0: hipStreamCreateWithPriority (lower = higher
 * priority, hipDeviceGetStreamPriorityRange), unmasked streams only.  The reference has no streams (one implicit CUDA stream,
 * main_*.py); these are plumbing of the drop-in's own training loop. */
int hlhgat_stream_create(int device, unsigned flags, int priority, const uint32_t* cu_mask,
                         int cu_mask_words, void** out);
/* The CU mask a stream runs on (hipExtStreamGetCUMask): all ones for an
 * unmasked stream. */
int hlhgat_stream_cu_mask(void* stream, uint32_t* cu_mask, int cu_mask_words);

/* Test hook: `workgroups` workgroups of 64 threads with lds_bytes of LDS
 * each; the first `hold` of them stay resident for `usec` microseconds (time
 * bounded), the others exit at once -- a kernel that holds most CUs while
 * another stream's kernel runs (tests of the BatchNorm barrier). */
int hlhgat_test_occupy(int workgroups, int hold, int lds_bytes, unsigned usec, void* stream);

/* ---- live kernel timing ------------------------------------------------ */
#define HLHGAT_PROF_POLY 0 /* SpMM / fused polynomial step kernel */
#define HLHGAT_PROF_PROJ 1 /* MFMA projection forward */
#define HLHGAT_PROF_HODGE_NODE 2 /* factored L1, stage 1: Z = B1 X (node rows) */
#define HLHGAT_PROF_HODGE_EDGE 3 /* factored L1, stage 2: k_hodge_edge_step */
#define HLHGAT_PROF_PROJ_BWD 4 /* Linear backward: k_proj_bwd_fused (weight partials + data grad) */
#define HLHGAT_PROF_BN_FWD 5 /* BatchNorm forward: k_bn_fwd_grid / k_bn_stats + k_bn_apply */
#define HLHGAT_PROF_BN_BWD 6 /* BatchNorm backward: k_bn_bwd_reduce + k_bn_bwd_apply */
#define HLHGAT_PROF_PROJ_BN 7 /* projection + BatchNorm forward in one launch: k_proj_bn_fwd */
/* call sites of k_poly_step beside the Laplacian basis (HLHGAT_PROF_POLY):
 * the adjoint recurrence of the basis backward (hlhgat_poly_basis_bwd*), and
 * the |B1| incidence gathers of NodeEdgeInt (hlhgat_incidence_step: node
 * rows gathering edge rows, x_s2t of lib/Hodge_Cheb_Conv.py:294 and the
 * node-side adjoint of x_t2s, :295); k_edge_gather2 (edge rows gathering
 * their two node rows: x_t2s and the adjoint of x_s2t) */
#define HLHGAT_PROF_POLY_ADJ 8
#define HLHGAT_PROF_INCIDENCE 9
#define HLHGAT_PROF_GATHER2 10
#define HLHGAT_PROF_NCLASS 11
/* Enable (1) / disable (0) event timing of the given kernel class. */
int hlhgat_prof_enable(int kernel_class, int enable);
int hlhgat_prof_reset(void);
/* Synchronises the recorded events and returns launch count, summed kernel
 * milliseconds, summed algorithmic bytes and flops for the class. */
int hlhgat_prof_read(int kernel_class, int64_t* launches, double* total_ms,
                     double* total_bytes, double* total_flops);

/* ---- captured-graph introspection (runtime) ----------------------------- */
/* Introspection of a captured graph: its kernel nodes, and those whose
 * kernel name contains name_part (e.g. "ncclDevKernel": RCCL's kernels). */
int hlhgat_graph_kernel_count(void* graph, const char* name_part, int64_t* kernels,
                              int64_t* matching);

#ifdef __cplusplus
}
#endif

#endif /* HLHGAT_H_ */
