// Native data loader: PairData collation + capacity padding + the batch
// tables, as HOST code (host pointers, no stream).
//
// The reference's DataLoader collates PairData graphs every step
// (lib/Hodge_Dataset.py:40-48: node / edge indices offset by the rows of the
// graphs before them) and the training loop copies the batch to the device
// (main_zinc_HL_HGCNN_dense_int3_pyr.py:151-162).  Here ONE call turns a list
// of graph ids of a packed dataset (hlhgat_packed_graphs_t, the
// InMemoryDataset-style storage of hlhgat.hodge_dataset.PackedGraphs) into
// the padded batch the hipGraph-replayed step reads, tables included:
//   x_t / x_s, the L0 / L1 COO with offsets, the B1 edge list, y, the graph
//   sizes; the Laplacian CSRs (rowptr over edge_index[0], int32 columns), the
//   incidence CSR of |B1| and the node degrees (adj2par1 / degree,
//   lib/Hodge_Dataset.py:169-191, lib/Hodge_Cheb_Conv.py:359), the readout
//   segment offsets, and the padding of hodge_dataset.pad_batch (zero rows,
//   zero-weight self-loops spread evenly over the padding rows, B1
//   self-edges over the padding nodes, unit padding degrees).
// Every array is bitwise what hodge_dataset.collate + pad_batch build
// (tests/test_host.py), in one pass over the bytes with no Python per-graph
// work: the loader keeps up with the replayed step on one host core.
#include <cstdint>
#include <cstring>
#include <vector>

#include "common.h"

namespace {

struct Sizes {
  int64_t n_t = 0, n_s = 0, z_t = 0, z_s = 0;
};

int batch_sizes(const hlhgat_packed_graphs_t* d, const int64_t* idx, int64_t B, Sizes& s) {
  for (int64_t b = 0; b < B; ++b) {
    const int64_t g = idx[b];
    HLH_CHECK_ARG(g >= 0 && g < d->n_graphs, "collate: graph id %lld out of range [0, %lld)",
                  (long long)g, (long long)d->n_graphs);
    s.n_t += d->node_ptr[g + 1] - d->node_ptr[g];
    s.n_s += d->edge_ptr[g + 1] - d->edge_ptr[g];
    s.z_t += d->lt_ptr[g + 1] - d->lt_ptr[g];
    s.z_s += d->ls_ptr[g + 1] - d->ls_ptr[g];
  }
  return HLHGAT_OK;
}

// rows r in [n, R) each get `base` (+1 for the first `extra` of them) of the
// zero-weight padding self-loops (hodge_dataset._spread)
void pad_loops(int64_t n, int64_t R, int64_t z, int64_t Z, int64_t* row, int64_t* col,
               float* w) {
  const int64_t extra = Z - z, bins = R - n;
  if (extra <= 0 || bins <= 0) return;
  const int64_t base = extra / bins, more = extra % bins;
  int64_t p = z;
  for (int64_t r = n; r < R; ++r) {
    const int64_t k = base + (r - n < more ? 1 : 0);
    for (int64_t i = 0; i < k; ++i, ++p) {
      row[p] = r;
      col[p] = r;
      w[p] = 0.f;
    }
  }
}

// CSR of a row-sorted COO: rowptr from the row counts, int32 columns
void coo_csr(const int64_t* row, const int64_t* col, int64_t nnz, int64_t n, int32_t* rowptr,
             int32_t* ccol) {
  std::memset(rowptr, 0, sizeof(int32_t) * (size_t)(n + 1));
  for (int64_t e = 0; e < nnz; ++e) rowptr[row[e] + 1]++;
  for (int64_t r = 0; r < n; ++r) rowptr[r + 1] += rowptr[r];
  for (int64_t e = 0; e < nnz; ++e) ccol[e] = (int32_t)col[e];
}

}  // namespace

extern "C" int hlhgat_collate_sizes(const hlhgat_packed_graphs_t* d, const int64_t* idx,
                                    int64_t n_idx, int64_t* sizes) {
  HLH_CHECK_ARG(d && sizes && n_idx >= 0 && (n_idx == 0 || idx), "collate_sizes: bad arguments");
  Sizes s;
  const int rc = batch_sizes(d, idx, n_idx, s);
  if (rc) return rc;
  sizes[0] = s.n_t;
  sizes[1] = s.n_s;
  sizes[2] = s.z_t;
  sizes[3] = s.z_s;
  return HLHGAT_OK;
}

extern "C" int hlhgat_collate(const hlhgat_packed_graphs_t* d, const int64_t* idx, int64_t B,
                              hlhgat_collated_t* o) {
  HLH_CHECK_ARG(d && o && B > 0 && idx, "collate: bad arguments");
  HLH_CHECK_ARG(d->node_ptr && d->edge_ptr && d->lt_ptr && d->ls_ptr && d->x_t && d->x_s &&
                    d->lt_row && d->lt_col && d->lt_w && d->ls_row && d->ls_col && d->ls_w &&
                    d->b1_src && d->b1_dst && d->f_t > 0 && d->f_s > 0 &&
                    (d->y_dim == 0 || d->y),
                "collate: incomplete packed dataset");
  Sizes s;
  int rc = batch_sizes(d, idx, B, s);
  if (rc) return rc;
  const int64_t Rt = o->rows_t, Rs = o->rows_s, Zt = o->nnz_t, Zs = o->nnz_s;
  const bool padded = !(Rt == s.n_t && Rs == s.n_s && Zt == s.z_t && Zs == s.z_s);
  if (padded)
    HLH_CHECK_ARG(Rt > s.n_t && Rs > s.n_s && Zt >= s.z_t && Zs >= s.z_s,
                  "collate: capacities (%lld, %lld, %lld, %lld) do not hold the batch "
                  "(%lld, %lld, %lld, %lld)",
                  (long long)Rt, (long long)Rs, (long long)Zt, (long long)Zs,
                  (long long)s.n_t, (long long)s.n_s, (long long)s.z_t, (long long)s.z_s);
  HLH_CHECK_ARG(Rt < INT32_MAX && 2 * Rs < INT32_MAX && Zt < INT32_MAX && Zs < INT32_MAX,
                "collate: batch too large for int32 tables");
  HLH_CHECK_ARG(o->x_t && o->x_s && o->edge_index_t && o->edge_weight_t && o->edge_index_s &&
                    o->edge_weight_s && o->edge_index && o->num_node1 && o->num_edge1 &&
                    (d->y_dim == 0 || o->y),
                "collate: NULL output");
  const int64_t Ft = d->f_t, Fs = d->f_s;
  int64_t* eit_r = o->edge_index_t;
  int64_t* eit_c = o->edge_index_t + Zt;
  int64_t* eis_r = o->edge_index_s;
  int64_t* eis_c = o->edge_index_s + Zs;
  int64_t* b1_r = o->edge_index;
  int64_t* b1_c = o->edge_index + Rs;
  int64_t nt = 0, ns = 0, zt = 0, zs = 0;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t g = idx[b];
    const int64_t n0 = d->node_ptr[g], n1 = d->node_ptr[g + 1];
    const int64_t e0 = d->edge_ptr[g], e1 = d->edge_ptr[g + 1];
    const int64_t t0 = d->lt_ptr[g], t1 = d->lt_ptr[g + 1];
    const int64_t s0 = d->ls_ptr[g], s1 = d->ls_ptr[g + 1];
    // the packed dataset is input data: every index must lie inside its own
    // graph and each Laplacian COO must be row-sorted (coo_csr below counts
    // rows into rowptr), else no write happens
    HLH_CHECK_ARG(n1 >= n0 && e1 >= e0 && t1 >= t0 && s1 >= s0,
                  "collate: graph %lld has negative sizes", (long long)g);
    for (int64_t k = t0; k < t1; ++k)
      HLH_CHECK_ARG(d->lt_row[k] >= 0 && d->lt_row[k] < n1 - n0 && d->lt_col[k] >= 0 &&
                        d->lt_col[k] < n1 - n0 && (k == t0 || d->lt_row[k] >= d->lt_row[k - 1]),
                    "collate: graph %lld: L0 entry %lld out of range or not row-sorted",
                    (long long)g, (long long)(k - t0));
    for (int64_t k = s0; k < s1; ++k)
      HLH_CHECK_ARG(d->ls_row[k] >= 0 && d->ls_row[k] < e1 - e0 && d->ls_col[k] >= 0 &&
                        d->ls_col[k] < e1 - e0 && (k == s0 || d->ls_row[k] >= d->ls_row[k - 1]),
                    "collate: graph %lld: L1 entry %lld out of range or not row-sorted",
                    (long long)g, (long long)(k - s0));
    for (int64_t e = e0; e < e1; ++e)
      HLH_CHECK_ARG(d->b1_src[e] >= 0 && d->b1_src[e] < n1 - n0 && d->b1_dst[e] >= 0 &&
                        d->b1_dst[e] < n1 - n0,
                    "collate: graph %lld: B1 edge %lld out of range", (long long)g,
                    (long long)(e - e0));
    std::memcpy(o->x_t + nt * Ft, d->x_t + n0 * Ft, sizeof(float) * (size_t)((n1 - n0) * Ft));
    std::memcpy(o->x_s + ns * Fs, d->x_s + e0 * Fs, sizeof(float) * (size_t)((e1 - e0) * Fs));
    for (int64_t k = t0; k < t1; ++k) {  // L0 COO: node offset
      eit_r[zt + k - t0] = nt + d->lt_row[k];
      eit_c[zt + k - t0] = nt + d->lt_col[k];
    }
    std::memcpy(o->edge_weight_t + zt, d->lt_w + t0, sizeof(float) * (size_t)(t1 - t0));
    for (int64_t k = s0; k < s1; ++k) {  // L1 COO: edge offset
      eis_r[zs + k - s0] = ns + d->ls_row[k];
      eis_c[zs + k - s0] = ns + d->ls_col[k];
    }
    std::memcpy(o->edge_weight_s + zs, d->ls_w + s0, sizeof(float) * (size_t)(s1 - s0));
    for (int64_t e = e0; e < e1; ++e) {  // B1 edge list: node offset
      b1_r[ns + e - e0] = nt + d->b1_src[e];
      b1_c[ns + e - e0] = nt + d->b1_dst[e];
    }
    if (d->y_dim)
      std::memcpy(o->y + b * d->y_dim, d->y + g * d->y_dim, sizeof(float) * (size_t)d->y_dim);
    o->num_node1[b] = n1 - n0;
    o->num_edge1[b] = e1 - e0;
    nt += n1 - n0;
    ns += e1 - e0;
    zt += t1 - t0;
    zs += s1 - s0;
  }
  // padding (hodge_dataset.pad_batch): zero feature rows, zero-weight
  // self-loops spread over the padding rows, B1 self-edges over the
  // padding nodes (nt + i % (Rt - nt))
  std::memset(o->x_t + nt * Ft, 0, sizeof(float) * (size_t)((Rt - nt) * Ft));
  std::memset(o->x_s + ns * Fs, 0, sizeof(float) * (size_t)((Rs - ns) * Fs));
  pad_loops(nt, Rt, zt, Zt, eit_r, eit_c, o->edge_weight_t);
  pad_loops(ns, Rs, zs, Zs, eis_r, eis_c, o->edge_weight_s);
  for (int64_t i = 0; i < Rs - ns; ++i) {
    b1_r[ns + i] = nt + i % (Rt - nt);
    b1_c[ns + i] = nt + i % (Rt - nt);
  }
  // Laplacian CSRs (hodge_dataset.laplacian_csr)
  if (o->csr_rowptr_t && o->csr_col_t) coo_csr(eit_r, eit_c, Zt, Rt, o->csr_rowptr_t, o->csr_col_t);
  if (o->csr_rowptr_s && o->csr_col_s) coo_csr(eis_r, eis_c, Zs, Rs, o->csr_rowptr_s, o->csr_col_s);
  // incidence CSR of |B1| (hodge_dataset.incidence_csr): edge e under both of
  // its end nodes, ascending edge ids per node, a self-edge twice
  if (o->inc_rowptr && o->inc_eids) {
    int32_t* rp = o->inc_rowptr;
    std::memset(rp, 0, sizeof(int32_t) * (size_t)(Rt + 1));
    for (int64_t e = 0; e < Rs; ++e) {
      HLH_CHECK_ARG(b1_r[e] >= 0 && b1_r[e] < Rt && b1_c[e] >= 0 && b1_c[e] < Rt,
                    "collate: B1 edge %lld out of range", (long long)e);
      rp[b1_r[e] + 1]++;
      rp[b1_c[e] + 1]++;
    }
    for (int64_t r = 0; r < Rt; ++r) rp[r + 1] += rp[r];
    std::vector<int32_t> fill(rp, rp + Rt);
    for (int64_t e = 0; e < Rs; ++e) {
      o->inc_eids[fill[b1_r[e]]++] = (int32_t)e;
      o->inc_eids[fill[b1_c[e]]++] = (int32_t)e;
    }
    // degree (lib/Hodge_Cheb_Conv.py:359) and its fp32 reciprocal; padding
    // nodes get degree 1 (hodge_dataset.node_degree(valid=nt))
    if (o->deg_t && o->inv_deg_t) {
      for (int64_t r = 0; r < Rt; ++r) {
        const float dv = (padded && r >= nt) ? 1.f : (float)(rp[r + 1] - rp[r]);
        o->deg_t[r] = dv;
        o->inv_deg_t[r] = 1.f / dv;
      }
    }
  }
  // readout segment offsets (global_mean_pool, lib/Hodge_ST_Model.py:636)
  if (o->seg_ptr_t && o->seg_ptr_s) {
    o->seg_ptr_t[0] = 0;
    o->seg_ptr_s[0] = 0;
    for (int64_t b = 0; b < B; ++b) {
      o->seg_ptr_t[b + 1] = o->seg_ptr_t[b] + (int32_t)o->num_node1[b];
      o->seg_ptr_s[b + 1] = o->seg_ptr_s[b] + (int32_t)o->num_edge1[b];
    }
  }
  if (o->valid_mask_t)
    for (int64_t r = 0; r < Rt; ++r) o->valid_mask_t[r] = r < nt ? 1 : 0;
  o->n_t = nt;
  o->n_s = ns;
  return HLHGAT_OK;
}
