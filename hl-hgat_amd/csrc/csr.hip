// CSR construction for the Hodge Laplacians (L0, L1) and the incidence |B1|.
//
// The reference never builds CSR: PyG propagate gathers x[edge_index[0]] and
// scatter-adds into edge_index[1] (lib/Hodge_Cheb_Conv.py:494,502), and
// torch.sparse.mm coalesces the COO |B1| on every call
// (lib/Hodge_Cheb_Conv.py:294-295, lib/Hodge_Dataset.py:169-191).  Here the
// operator is converted once per batch into row-owned CSR so the SpMM needs no
// atomics and is deterministic.
#include "common.h"

#include <hipcub/hipcub.hpp>

using namespace hlhgat;

namespace {

constexpr int kThreads = 256;

__global__ void k_check_sorted(const int64_t* __restrict__ row,
                               const int64_t* __restrict__ col, int64_t nnz,
                               int64_t n_rows, int64_t n_cols,
                               int32_t* __restrict__ flag) {
  int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= nnz) return;
  int64_t r = row[e], c = col[e];
  bool ok = r >= 0 && r < n_rows && c >= 0 && c < n_cols;
  if (e + 1 < nnz) {
    int64_t r1 = row[e + 1], c1 = col[e + 1];
    ok = ok && (r < r1 || (r == r1 && c <= c1));
  }
  if (!ok) atomicAnd(flag, 0);
}

// rowptr[r] = first e with key(e) >= r, for r in [0, n_rows]; keys sorted.
template <typename KeyFn>
__device__ __forceinline__ int64_t lower_bound_rows(KeyFn key, int64_t nnz,
                                                    int64_t target) {
  int64_t lo = 0, hi = nnz;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (key(mid) < target)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ void k_rowptr_sorted_rows(const int64_t* __restrict__ row,
                                     int64_t nnz, int64_t n_rows,
                                     int32_t* __restrict__ rowptr) {
  int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (r > n_rows) return;
  rowptr[r] = (int32_t)lower_bound_rows([&](int64_t i) { return row[i]; }, nnz, r);
}

__global__ void k_convert_sorted(const int64_t* __restrict__ col,
                                 const float* __restrict__ w, int64_t nnz,
                                 int32_t* __restrict__ col_out,
                                 float* __restrict__ val_out) {
  int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= nnz) return;
  col_out[e] = (int32_t)col[e];
  if (val_out) val_out[e] = w ? w[e] : 1.f;
}

__global__ void k_make_keys(const int64_t* __restrict__ row,
                            const int64_t* __restrict__ col, int64_t nnz,
                            uint64_t n_cols, uint64_t* __restrict__ keys,
                            int32_t* __restrict__ idx) {
  int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= nnz) return;
  keys[e] = (uint64_t)row[e] * n_cols + (uint64_t)col[e];
  idx[e] = (int32_t)e;
}

// Incidence entries of |B1|: entry t < E is (edge_index[0][t], t), entry
// t >= E is (edge_index[1][t-E], t-E) — the same row/col lists adj2par1 builds
// (lib/Hodge_Dataset.py:184-186).
__global__ void k_make_incidence_keys(const int64_t* __restrict__ ei,
                                      int64_t n_edges,
                                      uint64_t* __restrict__ keys) {
  int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (t >= 2 * n_edges) return;
  int64_t e = t < n_edges ? t : t - n_edges;
  keys[t] = (uint64_t)ei[t] * (uint64_t)n_edges + (uint64_t)e;
}

__global__ void k_finish_sorted_keys(const uint64_t* __restrict__ keys,
                                     const int32_t* __restrict__ idx,
                                     const float* __restrict__ w, int64_t nnz,
                                     uint64_t n_cols,
                                     int32_t* __restrict__ col_out,
                                     float* __restrict__ val_out,
                                     int32_t* __restrict__ perm) {
  int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= nnz) return;
  col_out[e] = (int32_t)(keys[e] % n_cols);
  if (idx) {
    int32_t src = idx[e];
    if (val_out) val_out[e] = w ? w[src] : 1.f;
    if (perm) perm[e] = src;
  }
}

__global__ void k_rowptr_from_keys(const uint64_t* __restrict__ keys,
                                   int64_t nnz, int64_t n_rows,
                                   uint64_t n_cols,
                                   int32_t* __restrict__ rowptr) {
  int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (r > n_rows) return;
  rowptr[r] = (int32_t)lower_bound_rows(
      [&](int64_t i) { return (int64_t)(keys[i] / n_cols); }, nnz, r);
}

int bits_for(uint64_t v) {  // number of bits to represent values < v
  int b = 0;
  while (b < 64 && (v >> b) > 0) ++b;
  return b < 1 ? 1 : b;
}

size_t cub_temp_bytes(int64_t nnz) {
  size_t t_pairs = 0, t_keys = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t_pairs, (uint64_t*)nullptr,
                                           (uint64_t*)nullptr, (int32_t*)nullptr,
                                           (int32_t*)nullptr, (int)nnz, 0, 64);
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, t_keys, (uint64_t*)nullptr,
                                          (uint64_t*)nullptr, (int)nnz, 0, 64);
  return t_pairs > t_keys ? t_pairs : t_keys;
}

inline size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

struct SortWs {
  uint64_t* keys_in;
  uint64_t* keys_out;
  int32_t* idx_in;
  int32_t* idx_out;
  void* temp;
  size_t temp_bytes;
};

size_t ws_bytes(int64_t nnz) {
  size_t n = (size_t)(nnz > 0 ? nnz : 1);
  return align_up(n * 8) * 2 + align_up(n * 4) * 2 + align_up(cub_temp_bytes(n));
}

SortWs carve(void* ws, int64_t nnz) {
  size_t n = (size_t)(nnz > 0 ? nnz : 1);
  char* p = (char*)ws;
  SortWs s;
  s.keys_in = (uint64_t*)p;
  p += align_up(n * 8);
  s.keys_out = (uint64_t*)p;
  p += align_up(n * 8);
  s.idx_in = (int32_t*)p;
  p += align_up(n * 4);
  s.idx_out = (int32_t*)p;
  p += align_up(n * 4);
  s.temp = p;
  s.temp_bytes = align_up(cub_temp_bytes(n));
  return s;
}

inline unsigned grid_for(int64_t n) {
  return (unsigned)((n + kThreads - 1) / kThreads);
}

}  // namespace

using namespace hlhgat;

extern "C" size_t hlhgat_csr_workspace_bytes(int64_t nnz) { return ws_bytes(nnz); }

extern "C" int hlhgat_coo_check_sorted(const int64_t* row, const int64_t* col,
                                       int64_t nnz, int64_t n_rows,
                                       int64_t n_cols, int32_t* flag_dev,
                                       void* stream) {
  HLH_CHECK_ARG(flag_dev, "coo_check_sorted: flag is NULL");
  HLH_CHECK_ARG(nnz >= 0, "coo_check_sorted: nnz < 0");
  hipStream_t s = as_stream(stream);
  const int32_t one = 1;
  HLH_CHECK_HIP(hipMemsetD32Async((hipDeviceptr_t)flag_dev, one, 1, s));
  if (nnz == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(row && col, "coo_check_sorted: NULL index");
  k_check_sorted<<<grid_for(nnz), kThreads, 0, s>>>(row, col, nnz, n_rows,
                                                    n_cols, flag_dev);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_csr_from_sorted_coo(const int64_t* row, const int64_t* col,
                                          const float* w, int64_t nnz,
                                          int64_t n_rows, int32_t* rowptr,
                                          int32_t* col_out, float* val_out,
                                          void* stream) {
  HLH_CHECK_ARG(nnz >= 0 && nnz < (int64_t)INT32_MAX,
                "csr_from_sorted_coo: nnz=%lld out of int32 range", (long long)nnz);
  HLH_CHECK_ARG(n_rows >= 0 && n_rows < (int64_t)INT32_MAX,
                "csr_from_sorted_coo: n_rows out of range");
  HLH_CHECK_ARG(rowptr, "csr_from_sorted_coo: rowptr is NULL");
  HLH_CHECK_ARG(nnz == 0 || (row && col && col_out),
                "csr_from_sorted_coo: NULL pointer");
  hipStream_t s = as_stream(stream);
  k_rowptr_sorted_rows<<<grid_for(n_rows + 1), kThreads, 0, s>>>(row, nnz, n_rows,
                                                                 rowptr);
  HLH_CHECK_LAUNCH();
  if (nnz > 0) {
    k_convert_sorted<<<grid_for(nnz), kThreads, 0, s>>>(col, w, nnz, col_out,
                                                        val_out);
    HLH_CHECK_LAUNCH();
  }
  return HLHGAT_OK;
}

extern "C" int hlhgat_csr_from_coo(const int64_t* row, const int64_t* col,
                                   const float* w, int64_t nnz, int64_t n_rows,
                                   int64_t n_cols, int32_t* rowptr,
                                   int32_t* col_out, float* val_out,
                                   int32_t* perm, void* workspace,
                                   size_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(nnz >= 0 && nnz < (int64_t)INT32_MAX,
                "csr_from_coo: nnz=%lld out of int32 range", (long long)nnz);
  HLH_CHECK_ARG(n_rows >= 0 && n_rows < (int64_t)INT32_MAX && n_cols > 0 &&
                    n_cols < (int64_t)INT32_MAX,
                "csr_from_coo: n_rows/n_cols out of range");
  HLH_CHECK_ARG(rowptr, "csr_from_coo: rowptr is NULL");
  hipStream_t s = as_stream(stream);
  if (nnz == 0) {
    HLH_CHECK_HIP(hipMemsetAsync(rowptr, 0, sizeof(int32_t) * (n_rows + 1), s));
    return HLHGAT_OK;
  }
  HLH_CHECK_ARG(row && col && col_out, "csr_from_coo: NULL pointer");
  HLH_CHECK_ARG(workspace && workspace_bytes >= ws_bytes(nnz),
                "csr_from_coo: workspace too small (%zu < %zu)", workspace_bytes,
                ws_bytes(nnz));
  SortWs ws = carve(workspace, nnz);
  const uint64_t nc = (uint64_t)n_cols;
  k_make_keys<<<grid_for(nnz), kThreads, 0, s>>>(row, col, nnz, nc, ws.keys_in,
                                                 ws.idx_in);
  HLH_CHECK_LAUNCH();
  int end_bit = bits_for((uint64_t)n_rows * nc);
  size_t temp = ws.temp_bytes;
  HLH_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(
      ws.temp, temp, ws.keys_in, ws.keys_out, ws.idx_in, ws.idx_out, (int)nnz,
      0, end_bit, s));
  k_finish_sorted_keys<<<grid_for(nnz), kThreads, 0, s>>>(
      ws.keys_out, ws.idx_out, w, nnz, nc, col_out, val_out, perm);
  HLH_CHECK_LAUNCH();
  k_rowptr_from_keys<<<grid_for(n_rows + 1), kThreads, 0, s>>>(ws.keys_out, nnz,
                                                               n_rows, nc, rowptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_incidence_csr(const int64_t* edge_index, int64_t n_edges,
                                    int64_t n_nodes, int32_t* rowptr,
                                    int32_t* edge_ids, void* workspace,
                                    size_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(n_edges >= 0 && 2 * n_edges < (int64_t)INT32_MAX,
                "incidence_csr: n_edges out of range");
  HLH_CHECK_ARG(n_nodes >= 0 && n_nodes < (int64_t)INT32_MAX,
                "incidence_csr: n_nodes out of range");
  HLH_CHECK_ARG(rowptr, "incidence_csr: rowptr is NULL");
  hipStream_t s = as_stream(stream);
  if (n_edges == 0) {
    HLH_CHECK_HIP(hipMemsetAsync(rowptr, 0, sizeof(int32_t) * (n_nodes + 1), s));
    return HLHGAT_OK;
  }
  HLH_CHECK_ARG(edge_index && edge_ids, "incidence_csr: NULL pointer");
  const int64_t nnz = 2 * n_edges;
  HLH_CHECK_ARG(workspace && workspace_bytes >= ws_bytes(nnz),
                "incidence_csr: workspace too small (%zu < %zu)", workspace_bytes,
                ws_bytes(nnz));
  SortWs ws = carve(workspace, nnz);
  const uint64_t ne = (uint64_t)n_edges;
  k_make_incidence_keys<<<grid_for(nnz), kThreads, 0, s>>>(edge_index, n_edges,
                                                           ws.keys_in);
  HLH_CHECK_LAUNCH();
  int end_bit = bits_for((uint64_t)n_nodes * ne);
  size_t temp = ws.temp_bytes;
  HLH_CHECK_HIP(hipcub::DeviceRadixSort::SortKeys(ws.temp, temp, ws.keys_in,
                                                  ws.keys_out, (int)nnz, 0,
                                                  end_bit, s));
  k_finish_sorted_keys<<<grid_for(nnz), kThreads, 0, s>>>(
      ws.keys_out, nullptr, nullptr, nnz, ne, edge_ids, nullptr, nullptr);
  HLH_CHECK_LAUNCH();
  k_rowptr_from_keys<<<grid_for(n_nodes + 1), kThreads, 0, s>>>(
      ws.keys_out, nnz, n_nodes, ne, rowptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// ---------------------------------------------------------------------------
// Halo tiles for the LDS-staged SpMM (host side, run once per graph at
// dataset-build time like the row schedule; see hlhgat_halo_t).
// Greedy over the row schedule: a row joins the current tile unless that
// would push the tile past max_rows rows, max_nnz entries or max_halo
// distinct columns.
// ---------------------------------------------------------------------------
#include <algorithm>
#include <vector>

extern "C" int hlhgat_halo_tiles(const int32_t* rowptr, const int32_t* col, int64_t n_rows,
                                 int64_t n_cols, const int32_t* order, int32_t max_rows,
                                 int32_t max_nnz, int32_t max_halo, int32_t* tile_ptr,
                                 int32_t* halo_ptr, int32_t* halo, int32_t* srp, uint16_t* lcol,
                                 int32_t* eperm, int32_t* hdr, int64_t* n_tiles,
                                 int64_t* n_halo) {
  HLH_CHECK_ARG(n_rows >= 0 && n_cols >= 0 && n_rows < INT32_MAX && n_cols < INT32_MAX,
                "halo_tiles: bad sizes");
  HLH_CHECK_ARG(max_rows > 0 && max_nnz > 0 && max_halo > 0 && max_halo <= 65535,
                "halo_tiles: max_rows, max_nnz > 0 and 0 < max_halo <= 65535 required");
  HLH_CHECK_ARG(rowptr && tile_ptr && halo_ptr && srp && hdr && n_tiles && n_halo,
                "halo_tiles: NULL pointer");
  const int64_t nnz = n_rows ? rowptr[n_rows] : 0;
  HLH_CHECK_ARG(nnz == 0 || (col && halo && lcol && eperm), "halo_tiles: NULL pointer");
  // owner[c] = tile that holds column c in its halo; probe[c] = last probe
  std::vector<int64_t> owner((size_t)n_cols, -1), probe((size_t)n_cols, -1);
  std::vector<int32_t> cols;  // current tile's halo, insertion order
  cols.reserve((size_t)max_halo);
  int64_t t = 0, h = 0, p0 = 0, probes = 0, tile_nnz = 0;
  tile_ptr[0] = 0;
  halo_ptr[0] = 0;
  srp[0] = 0;
  auto row_at = [&](int64_t p) -> int64_t { return order ? (int64_t)order[p] : p; };
  auto close_tile = [&](int64_t p_end) {
    // halo ascending; tile-local column of every entry of the tile's rows
    std::sort(cols.begin(), cols.end());
    for (size_t i = 0; i < cols.size(); ++i) halo[h + (int64_t)i] = cols[i];
    for (int64_t p = p0; p < p_end; ++p) {
      const int64_t r = row_at(p);
      int64_t i = srp[p];
      for (int32_t e = rowptr[r]; e < rowptr[r + 1]; ++e, ++i) {
        lcol[i] = (uint16_t)(std::lower_bound(cols.begin(), cols.end(), col[e]) - cols.begin());
        eperm[i] = e;
      }
    }
    h += (int64_t)cols.size();
    ++t;
    tile_ptr[t] = (int32_t)p_end;
    halo_ptr[t] = (int32_t)h;
    cols.clear();
    p0 = p_end;
    tile_nnz = 0;
  };
  for (int64_t p = 0; p < n_rows; ++p) {
    const int64_t r = row_at(p);
    HLH_CHECK_ARG(r >= 0 && r < n_rows, "halo_tiles: order[%lld] out of range", (long long)p);
    const int64_t len = rowptr[r + 1] - rowptr[r];
    for (int pass = 0; pass < 2; ++pass) {
      // distinct columns this row would add to the current tile
      const int64_t id = probes++;
      int64_t add = 0;
      for (int32_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
        const int32_t c = col[e];
        HLH_CHECK_ARG(c >= 0 && c < n_cols, "halo_tiles: col out of range");
        if (owner[c] != t && probe[c] != id) {
          probe[c] = id;
          ++add;
        }
      }
      if ((int64_t)cols.size() + add <= max_halo && p - p0 < max_rows &&
          tile_nnz + len <= max_nnz) {
        for (int32_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
          const int32_t c = col[e];
          if (owner[c] != t) {
            owner[c] = t;
            cols.push_back(c);
          }
        }
        tile_nnz += len;
        srp[p + 1] = (int32_t)(srp[p] + len);
        break;
      }
      HLH_CHECK_ARG(p > p0 && pass == 0,
                    "halo_tiles: row %lld exceeds max_halo=%d columns or max_nnz=%d entries",
                    (long long)r, max_halo, max_nnz);
      close_tile(p);
    }
  }
  if (p0 < n_rows) close_tile(n_rows);
  for (int64_t i = 0; i < t; ++i) {  // one 32-B header per tile (a single load in the kernel)
    int32_t* q = hdr + 8 * i;
    q[0] = tile_ptr[i];
    q[1] = tile_ptr[i + 1] - tile_ptr[i];
    q[2] = halo_ptr[i];
    q[3] = halo_ptr[i + 1] - halo_ptr[i];
    q[4] = srp[tile_ptr[i]];
    q[5] = srp[tile_ptr[i + 1]] - srp[tile_ptr[i]];
    q[6] = q[7] = 0;
  }
  *n_tiles = t;
  *n_halo = h;
  return HLHGAT_OK;
}

namespace {
__global__ void k_gather_f32(const float* __restrict__ src, const int32_t* __restrict__ idx,
                             int64_t n, float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}
}  // namespace

extern "C" int hlhgat_gather_f32(const float* src, const int32_t* idx, int64_t n, float* dst,
                                 void* stream) {
  HLH_CHECK_ARG(n >= 0, "gather_f32: n < 0");
  if (n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(src && idx && dst, "gather_f32: NULL pointer");
  k_gather_f32<<<grid_for(n), kThreads, 0, as_stream(stream)>>>(src, idx, n, dst);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}
