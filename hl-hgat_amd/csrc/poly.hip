// CSR SpMM, the fused Laguerre / Chebyshev polynomial step (forward and
// adjoint), the node<->edge boundary-operator gathers and segment means.
//
// All of these are HBM/L2-bound row gathers: one group of LPR lanes owns one
// output row, each lane owns V consecutive features (float4 when the width
// allows), so a 64-float feature row is ONE coalesced 256-B access by 16 lanes
// and a wave64 serves 4 rows at once.  Rows are owned by exactly one lane
// group: no atomics, deterministic summation in CSR (= coalesced COO) order.
//
// Built with -ffp-contract=off: products and sums are rounded separately in
// the same order as the reference's CPU scatter-add / sparse.mm, so for the
// forward SpMM and Laguerre step the results are bitwise equal to the torch
// CPU restatement in oracle/ (tests check this).
#include "common.h"

using namespace hlhgat;

namespace {

struct PolyArgs {
  const int32_t* order;  // optional row schedule: slot -> row (a permutation)
  const int32_t* rowptr;
  const int32_t* col;
  const float* val;
  const float* rs;
  const float* X;
  const float* Z;
  const float* P;
  const float* Q;
  float* Y;
  int64_t ldx, ldz, ldp, ldq, ldy;
  int64_t n_rows;
  int d;
  float alpha, beta, gamma, div, p, q;
};

// Row r's CSR entries are staged LPR at a time: lane `sub` of the row group
// loads entry eb+sub's column and weight with ONE coalesced load, and the
// group broadcasts them with __shfl (ds_bpermute) while it walks the entries
// in CSR order.  The per-entry index / weight traffic thus leaves the vector
// memory pipe, which then carries only the gathered feature rows (the cost
// that bounds this kernel at TSP scale: ~20 gathered 512-B rows per output
// row).  Summation order is unchanged: acc += w_e * X[c_e] for e ascending.
__device__ __forceinline__ unsigned xcd_slot(unsigned b, unsigned nb) {
  const unsigned x = b & 7u, k = b >> 3, per = nb >> 3, extra = nb & 7u;
  return x * per + (x < extra ? x : extra) + k;
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_poly_step(PolyArgs a) {
  using vt = typename VecT<V>::type;
  // XCD-aware slots: blocks are dealt round-robin over the 8 XCDs, so block b
  // takes slot range xcd_slot(b): each XCD walks ONE contiguous range of the
  // (optionally locality-ordered) row schedule and its L2 sees the neighbours
  // of the rows it is working on.
  const int64_t slot = ((int64_t)xcd_slot(blockIdx.x, gridDim.x) * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  const bool live = slot < a.n_rows;
  const int64_t row = live ? (a.order ? (int64_t)a.order[slot] : slot) : 0;
  const int64_t rr = row;
  const int e0 = live ? a.rowptr[rr] : 0;
  const int e1 = live ? a.rowptr[rr + 1] : 0;
  const float rsv = (live && a.rs) ? a.rs[rr] : 1.f;
  const float* __restrict__ X = a.X;
  for (int f0 = 0; f0 < a.d; f0 += LPR * V) {
    const int f = f0 + sub * V;
    const bool fok = live && f < a.d;
    vt acc;
#pragma unroll
    for (int i = 0; i < V; ++i) vget(acc, i) = 0.f;
    for (int eb = e0; eb < e1; eb += LPR) {
      const int me = eb + sub;
      const int cm = me < e1 ? a.col[me] : 0;
      const float wm = me < e1 ? (a.val ? a.val[me] : 1.f) : 0.f;
      const int cnt = e1 - eb < LPR ? e1 - eb : LPR;
      int j = 0;
      for (; j + 3 < cnt; j += 4) {  // four gathers in flight per lane
        const int c0 = __shfl(cm, j, LPR), c1 = __shfl(cm, j + 1, LPR),
                  c2 = __shfl(cm, j + 2, LPR), c3 = __shfl(cm, j + 3, LPR);
        const float w0 = __shfl(wm, j, LPR), w1 = __shfl(wm, j + 1, LPR),
                    w2 = __shfl(wm, j + 2, LPR), w3 = __shfl(wm, j + 3, LPR);
        if (fok) {
          vt x0 = vload<V>(X + (int64_t)c0 * a.ldx + f);
          vt x1 = vload<V>(X + (int64_t)c1 * a.ldx + f);
          vt x2 = vload<V>(X + (int64_t)c2 * a.ldx + f);
          vt x3 = vload<V>(X + (int64_t)c3 * a.ldx + f);
#pragma unroll
          for (int i = 0; i < V; ++i) {
            float s = vget(acc, i);
            s = s + w0 * vget(x0, i);
            s = s + w1 * vget(x1, i);
            s = s + w2 * vget(x2, i);
            s = s + w3 * vget(x3, i);
            vget(acc, i) = s;
          }
        }
      }
      for (; j < cnt; ++j) {
        const int c = __shfl(cm, j, LPR);
        const float w = __shfl(wm, j, LPR);
        if (fok) {
          vt x = vload<V>(X + (int64_t)c * a.ldx + f);
#pragma unroll
          for (int i = 0; i < V; ++i) vget(acc, i) = vget(acc, i) + w * vget(x, i);
        }
      }
    }
    if (!fok) continue;
    vt out;
#pragma unroll
    for (int i = 0; i < V; ++i) vget(out, i) = a.alpha * (rsv * vget(acc, i));
    if (a.beta != 0.f) {
      vt xr = vload<V>(X + row * a.ldx + f);
#pragma unroll
      for (int i = 0; i < V; ++i) vget(out, i) = vget(out, i) + a.beta * vget(xr, i);
    }
    if (a.Z) {
      vt z = vload<V>(a.Z + row * a.ldz + f);
#pragma unroll
      for (int i = 0; i < V; ++i) vget(out, i) = vget(out, i) + a.gamma * vget(z, i);
    }
    if (a.div != 1.f) {
#pragma unroll
      for (int i = 0; i < V; ++i) vget(out, i) = vget(out, i) / a.div;
    }
    if (a.P) {
      vt pv = vload<V>(a.P + row * a.ldp + f);
#pragma unroll
      for (int i = 0; i < V; ++i) vget(out, i) = vget(out, i) + a.p * vget(pv, i);
    }
    if (a.Q) {
      vt qv = vload<V>(a.Q + row * a.ldq + f);
#pragma unroll
      for (int i = 0; i < V; ++i) vget(out, i) = vget(out, i) + a.q * vget(qv, i);
    }
    vstore<V>(a.Y + row * a.ldy + f, out);
  }
}

// out[e] = ca*(sa[i]*x[i]) + cb*(sb[j]*x[j]) (+ z[e]) (+ out[e])
struct Gather2Args {
  const int64_t* ei;
  int64_t n_edges;
  const float* x;
  int64_t ldx;
  int d;
  const float* sa;
  const float* sb;
  float ca, cb;
  const float* z;  // optional per-edge addend [n_edges][ldz]
  int64_t ldz;
  float* out;
  int64_t ldo;
  int accumulate;
};

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_edge_gather2(Gather2Args a) {
  using vt = typename VecT<V>::type;
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (e >= a.n_edges) return;
  const int64_t i = a.ei[e];
  const int64_t j = a.ei[a.n_edges + e];
  const float si = a.sa ? a.sa[i] : 1.f;
  const float sj = a.sb ? a.sb[j] : 1.f;
  for (int f = sub * V; f < a.d; f += LPR * V) {
    vt xi = vload<V>(a.x + i * a.ldx + f);
    vt xj = vload<V>(a.x + j * a.ldx + f);
    vt o;
#pragma unroll
    for (int c = 0; c < V; ++c)
      vget(o, c) = a.ca * (si * vget(xi, c)) + a.cb * (sj * vget(xj, c));
    if (a.z) {
      vt zv = vload<V>(a.z + e * a.ldz + f);
#pragma unroll
      for (int c = 0; c < V; ++c) vget(o, c) = vget(zv, c) + vget(o, c);
    }
    if (a.accumulate) {
      vt prev = vload<V>(a.out + e * a.ldo + f);
#pragma unroll
      for (int c = 0; c < V; ++c) vget(o, c) = vget(prev, c) + vget(o, c);
    }
    vstore<V>(a.out + e * a.ldo + f, o);
  }
}

// Segment mean: out[s] = (sum_{r in seg s} x[r]) / max(|seg|, 1)
// (torch_scatter.scatter_mean semantics: sum divided by clamped count).
struct SegArgs {
  const int32_t* ptr;
  const int32_t* rows;
  int64_t n_seg;
  const float* x;
  int64_t ldx;
  int d;
  float* out;
  int64_t ldo;
};

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_segment_mean_fwd(SegArgs a) {
  using vt = typename VecT<V>::type;
  const int64_t s = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (s >= a.n_seg) return;
  const int r0 = a.ptr[s], r1 = a.ptr[s + 1];
  const float cnt = (float)(r1 - r0 > 0 ? r1 - r0 : 1);
  for (int f = sub * V; f < a.d; f += LPR * V) {
    vt acc;
#pragma unroll
    for (int c = 0; c < V; ++c) vget(acc, c) = 0.f;
    for (int t = r0; t < r1; ++t) {
      const int64_t r = a.rows ? a.rows[t] : t;
      vt xv = vload<V>(a.x + r * a.ldx + f);
#pragma unroll
      for (int c = 0; c < V; ++c) vget(acc, c) = vget(acc, c) + vget(xv, c);
    }
#pragma unroll
    for (int c = 0; c < V; ++c) vget(acc, c) = vget(acc, c) / cnt;
    vstore<V>(a.out + s * a.ldo + f, acc);
  }
}

// dx[r] = dout[s] / max(|seg s|, 1) for each member r of segment s.
template <int V, int LPR>
__global__ __launch_bounds__(256) void k_segment_mean_bwd(SegArgs a) {
  using vt = typename VecT<V>::type;
  const int64_t s = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (s >= a.n_seg) return;
  const int r0 = a.ptr[s], r1 = a.ptr[s + 1];
  const float cnt = (float)(r1 - r0 > 0 ? r1 - r0 : 1);
  // here x = dout (ldx), out = dx (ldo)
  for (int f = sub * V; f < a.d; f += LPR * V) {
    vt g = vload<V>(a.x + s * a.ldx + f);
#pragma unroll
    for (int c = 0; c < V; ++c) vget(g, c) = vget(g, c) / cnt;
    for (int t = r0; t < r1; ++t) {
      const int64_t r = a.rows ? a.rows[t] : t;
      vstore<V>(a.out + r * a.ldo + f, g);
    }
  }
}

// --- host-side dispatch ------------------------------------------------------
// Widest vector width V in {4,2,1} that divides d and every row stride and
// keeps every base pointer aligned; lanes per row = next pow2 of d/V (<= 64).
int pick_vec(int64_t d, std::initializer_list<int64_t> lds,
             std::initializer_list<const void*> ptrs) {
  for (int v : {4, 2}) {
    bool ok = (d % v) == 0;
    for (int64_t ld : lds) ok = ok && (ld % v) == 0;
    for (const void* p : ptrs)
      ok = ok && (p == nullptr ||
                  (reinterpret_cast<uintptr_t>(p) % (uintptr_t)(4 * v)) == 0);
    if (ok) return v;
  }
  return 1;
}

int pick_lpr(int64_t d, int v) {
  int lanes = (int)ceil_div(d, v);
  int l = next_pow2(lanes);
  return l > 64 ? 64 : l;
}

#define HLH_DISPATCH_VL(V, L, KERNEL, GRID_ROWS, STREAM, ARGS, PROF)           \
  do {                                                                         \
    const int64_t _rows_per_block = 256 / (L);                                 \
    const unsigned _grid = (unsigned)ceil_div((GRID_ROWS), _rows_per_block);   \
    if (_grid == 0) break;                                                     \
    switch ((V) * 100 + (L)) {                                                 \
      case 101: launch(KERNEL<1, 1>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 102: launch(KERNEL<1, 2>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 104: launch(KERNEL<1, 4>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 108: launch(KERNEL<1, 8>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 116: launch(KERNEL<1, 16>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 132: launch(KERNEL<1, 32>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 164: launch(KERNEL<1, 64>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 201: launch(KERNEL<2, 1>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 202: launch(KERNEL<2, 2>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 204: launch(KERNEL<2, 4>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 208: launch(KERNEL<2, 8>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 216: launch(KERNEL<2, 16>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 232: launch(KERNEL<2, 32>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 264: launch(KERNEL<2, 64>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 401: launch(KERNEL<4, 1>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 402: launch(KERNEL<4, 2>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 404: launch(KERNEL<4, 4>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 408: launch(KERNEL<4, 8>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 416: launch(KERNEL<4, 16>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 432: launch(KERNEL<4, 32>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      case 464: launch(KERNEL<4, 64>, _grid, 256, 0, STREAM, PROF, ARGS); break; \
      default: break;                                                          \
    }                                                                          \
  } while (0)

// Algorithmic bytes of one poly-step launch: CSR streamed once
// (int32 col + fp32 val per nnz, int32 rowptr), the gathered operand counted
// once per row (X read once), every dense row operand read once, Y written.
double poly_bytes(const PolyArgs& a, int64_t nnz) {
  double b = (double)nnz * (a.val ? 8.0 : 4.0) + 4.0 * (double)(a.n_rows + 1);
  double row_bytes = 4.0 * (double)a.n_rows * a.d;
  int dense = 2;  // gathered X (read once) + Y written
  if (a.Z) dense++;
  if (a.P) dense++;
  if (a.Q) dense++;
  if (a.rs) b += 4.0 * a.n_rows;
  return b + dense * row_bytes;
}

int launch_poly(PolyArgs& a, int64_t nnz, hipStream_t s) {
  HLH_CHECK_ARG(a.n_rows >= 0 && a.n_rows < (int64_t)INT32_MAX,
                "poly_step: n_rows out of range");
  HLH_CHECK_ARG(a.d > 0, "poly_step: d must be > 0");
  HLH_CHECK_ARG(a.rowptr && (nnz == 0 || a.col) && a.X && a.Y,
                "poly_step: NULL pointer");
  HLH_CHECK_ARG(a.ldx >= a.d && a.ldy >= a.d, "poly_step: ld < d");
  HLH_CHECK_ARG(!a.Z || a.ldz >= a.d, "poly_step: ldz < d");
  HLH_CHECK_ARG(!a.P || a.ldp >= a.d, "poly_step: ldp < d");
  HLH_CHECK_ARG(!a.Q || a.ldq >= a.d, "poly_step: ldq < d");
  HLH_CHECK_ARG(a.div != 0.f, "poly_step: div == 0");
  if (a.n_rows == 0) return HLHGAT_OK;
  const int v = pick_vec(a.d, {a.ldx, a.ldy, a.Z ? a.ldz : 4, a.P ? a.ldp : 4,
                               a.Q ? a.ldq : 4},
                         {a.X, a.Y, a.Z, a.P, a.Q});
  const int l = pick_lpr(a.d, v);
  ProfScope prof(HLHGAT_PROF_POLY, s, poly_bytes(a, nnz),
                 2.0 * (double)nnz * a.d);
  HLH_DISPATCH_VL(v, l, k_poly_step, a.n_rows, s, a, &prof);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

PolyArgs make_args(const int32_t* rowptr, const int32_t* col, const float* val,
                   int64_t n, const float* X, int64_t ldx, int64_t d, float* Y,
                   int64_t ldy, const int32_t* order = nullptr) {
  PolyArgs a{};
  a.order = order;
  a.rowptr = rowptr;
  a.col = col;
  a.val = val;
  a.rs = nullptr;
  a.X = X;
  a.ldx = ldx;
  a.Y = Y;
  a.ldy = ldy;
  a.n_rows = n;
  a.d = (int)d;
  a.alpha = 1.f;
  a.beta = 0.f;
  a.gamma = 0.f;
  a.div = 1.f;
  a.p = 0.f;
  a.q = 0.f;
  return a;
}

}  // namespace

using namespace hlhgat;

extern "C" int hlhgat_spmm(const int32_t* rowptr, const int32_t* col,
                           const float* val, int64_t n_rows, int64_t nnz,
                           const int32_t* row_order, const float* X, int64_t ldx,
                           int64_t d, float* Y, int64_t ldy, void* stream) {
  PolyArgs a = make_args(rowptr, col, val, n_rows, X, ldx, d, Y, ldy, row_order);
  return launch_poly(a, nnz, as_stream(stream));
}

extern "C" int hlhgat_poly_step(const int32_t* rowptr, const int32_t* col,
                                const float* val, const float* rs,
                                int64_t n_rows, int64_t nnz,
                                const int32_t* row_order, const float* X,
                                int64_t ldx, int64_t d, const float* Z,
                                int64_t ldz, const float* P, int64_t ldp,
                                const float* Q, int64_t ldq, float alpha,
                                float beta, float gamma, float div, float p,
                                float q, float* Y, int64_t ldy, void* stream) {
  PolyArgs a = make_args(rowptr, col, val, n_rows, X, ldx, d, Y, ldy, row_order);
  a.rs = rs;
  a.Z = Z;
  a.ldz = ldz;
  a.P = P;
  a.ldp = ldp;
  a.Q = Q;
  a.ldq = ldq;
  a.alpha = alpha;
  a.beta = beta;
  a.gamma = gamma;
  a.div = div;
  a.p = p;
  a.q = q;
  return launch_poly(a, nnz, as_stream(stream));
}

extern "C" int hlhgat_poly_basis_fwd(int kind, const int32_t* rowptr,
                                     const int32_t* col, const float* val,
                                     int64_t n, int64_t nnz,
                                     const int32_t* row_order, const float* X,
                                     int64_t ldx, int64_t F, int K, float* T,
                                     void* stream) {
  HLH_CHECK_ARG(kind == HLHGAT_POLY_LAGUERRE || kind == HLHGAT_POLY_CHEB,
                "poly_basis_fwd: bad kind %d", kind);
  HLH_CHECK_ARG(K >= 1, "poly_basis_fwd: K must be > 0 (assert K > 0)");
  if (K == 1 || n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(T, "poly_basis_fwd: T is NULL");
  hipStream_t s = as_stream(stream);
  const int64_t blk = n * F;
  auto Tk = [&](int k) -> float* { return T + (int64_t)(k - 1) * blk; };
  // T_1
  {
    PolyArgs a = make_args(rowptr, col, val, n, X, ldx, F, Tk(1), F, row_order);
    if (kind == HLHGAT_POLY_LAGUERRE) {  // Tx_1 = x - L x   (:494)
      a.alpha = -1.f;
      a.beta = 1.f;
    }  // Cheb: Tx_1 = L x   (:416)
    int rc = launch_poly(a, nnz, s);
    if (rc) return rc;
  }
  for (int k = 1; k + 1 < K; ++k) {
    const float* prev = (k == 1) ? X : Tk(k - 1);
    const int64_t ldprev = (k == 1) ? ldx : F;
    PolyArgs a = make_args(rowptr, col, val, n, Tk(k), F, F, Tk(k + 1), F, row_order);
    a.Z = prev;
    a.ldz = ldprev;
    if (kind == HLHGAT_POLY_LAGUERRE) {
      // Tx_2 = (-L Tx_1 + (2k+1) Tx_1 - k Tx_0) / (k+1)   (:502,507)
      a.alpha = -1.f;
      a.beta = (float)(2 * k + 1);
      a.gamma = -(float)k;
      a.div = (float)(k + 1);
    } else {
      // Tx_2 = 2 L Tx_1 - Tx_0   (:430-432)
      a.alpha = 2.f;
      a.gamma = -1.f;
    }
    int rc = launch_poly(a, nnz, s);
    if (rc) return rc;
  }
  return HLHGAT_OK;
}

extern "C" int hlhgat_poly_basis_bwd(int kind, const int32_t* rowptr_t,
                                     const int32_t* col_t, const float* val_t,
                                     int64_t n, int64_t nnz,
                                     const int32_t* row_order, int64_t F, int K,
                                     float* G, void* stream) {
  HLH_CHECK_ARG(kind == HLHGAT_POLY_LAGUERRE || kind == HLHGAT_POLY_CHEB,
                "poly_basis_bwd: bad kind %d", kind);
  HLH_CHECK_ARG(K >= 1, "poly_basis_bwd: K must be > 0");
  if (K == 1 || n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(G, "poly_basis_bwd: G is NULL");
  hipStream_t s = as_stream(stream);
  const int64_t blk = n * F;
  auto Gk = [&](int k) -> float* { return G + (int64_t)k * blk; };
  for (int k = K - 1; k >= 1; --k) {
    PolyArgs a = make_args(rowptr_t, col_t, val_t, n, Gk(k), F, F, Gk(k - 1), F, row_order);
    a.P = Gk(k - 1);
    a.ldp = F;
    a.p = 1.f;
    if (k + 1 <= K - 1) {
      a.Q = Gk(k + 1);
      a.ldq = F;
    }
    if (kind == HLHGAT_POLY_LAGUERRE) {
      // G_{k-1} += (-L^T G_k + (2k-1) G_k)/k - k/(k+1) G_{k+1}
      a.alpha = -1.f;
      a.beta = (float)(2 * k - 1);
      a.div = (float)k;
      a.q = -(float)k / (float)(k + 1);
    } else {
      // G_{k-1} += c_k L^T G_k - G_{k+1},  c_1 = 1, c_k = 2
      a.alpha = (k == 1) ? 1.f : 2.f;
      a.q = -1.f;
    }
    int rc = launch_poly(a, nnz, s);
    if (rc) return rc;
  }
  return HLHGAT_OK;
}

extern "C" int hlhgat_edge_gather2(const int64_t* edge_index, int64_t n_edges,
                                   const float* x, int64_t ldx, int64_t d,
                                   const float* sa, const float* sb, float ca,
                                   float cb, const float* z, int64_t ldz,
                                   float* out, int64_t ldo, int accumulate,
                                   void* stream) {
  HLH_CHECK_ARG(n_edges >= 0 && d > 0 && ldx >= d && ldo >= d && (!z || ldz >= d),
                "edge_gather2: bad sizes");
  if (n_edges == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(edge_index && x && out, "edge_gather2: NULL pointer");
  Gather2Args a{edge_index, n_edges, x, ldx, (int)d, sa, sb, ca, cb, z, ldz, out, ldo,
                accumulate};
  const int v = pick_vec(d, {ldx, ldo, z ? ldz : 4}, {x, out, z});
  const int l = pick_lpr(d, v);
  hipStream_t s = as_stream(stream);
  HLH_DISPATCH_VL(v, l, k_edge_gather2, n_edges, s, a, nullptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_segment_mean_fwd(const int32_t* seg_ptr,
                                       const int32_t* seg_rows, int64_t n_seg,
                                       const float* x, int64_t ldx, int64_t d,
                                       float* out, int64_t ldo, void* stream) {
  HLH_CHECK_ARG(n_seg >= 0 && d > 0 && ldx >= d && ldo >= d,
                "segment_mean_fwd: bad sizes");
  if (n_seg == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(seg_ptr && x && out, "segment_mean_fwd: NULL pointer");
  SegArgs a{seg_ptr, seg_rows, n_seg, x, ldx, (int)d, out, ldo};
  const int v = pick_vec(d, {ldx, ldo}, {x, out});
  const int l = pick_lpr(d, v);
  hipStream_t s = as_stream(stream);
  HLH_DISPATCH_VL(v, l, k_segment_mean_fwd, n_seg, s, a, nullptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_segment_mean_bwd(const int32_t* seg_ptr,
                                       const int32_t* seg_rows, int64_t n_seg,
                                       const float* dout, int64_t ldo, int64_t d,
                                       float* dx, int64_t ldx, void* stream) {
  HLH_CHECK_ARG(n_seg >= 0 && d > 0 && ldx >= d && ldo >= d,
                "segment_mean_bwd: bad sizes");
  if (n_seg == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(seg_ptr && dout && dx, "segment_mean_bwd: NULL pointer");
  SegArgs a{seg_ptr, seg_rows, n_seg, dout, ldo, (int)d, dx, ldx};
  const int v = pick_vec(d, {ldx, ldo}, {dout, dx});
  const int l = pick_lpr(d, v);
  hipStream_t s = as_stream(stream);
  HLH_DISPATCH_VL(v, l, k_segment_mean_bwd, n_seg, s, a, nullptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}
