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

#include <cstdlib>

using namespace hlhgat;

namespace {

struct PolyArgs {
  const int32_t* order;  // optional row schedule: slot -> row (a permutation)
  const int32_t* rowptr;
  const int32_t* col;
  const float* val;
  const float* rs;
  const float* X;
  const float* B;  // operand of the beta term (NULL: X itself)
  const float* Z;
  const float* P;
  const float* Q;
  float* Y;
  int64_t ldx, ldb, ldz, ldp, ldq, ldy;
  int64_t n_rows;
  int d;
  float alpha, beta, gamma, div, p, q;
  // halo tiles (optional; lcol != NULL selects k_poly_halo, see hlhgat_halo_t)
  const int32_t* hdr;
  const int32_t* htile;
  const int32_t* hptr;
  const int32_t* hcols;
  const int32_t* srp;
  const uint16_t* lcol;
  const float* sval;
  int64_t n_tiles;
  int max_halo, max_trows, max_tnnz, halo_fs;
  int nt_store;  // streaming (non-temporal) stores of Y: keep L2 for the gathered X rows
  // Hodge-factored L1 edge step (k_hodge_edge_step): X = Z = B1 T (node rows)
  const int2* ends;     // [n_rows] (i, j) of each edge
  const float* ealpha;  // [n_rows] alpha_e = L1[e,e] / 2
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

// Row epilogue shared by k_poly_step and k_poly_halo (identical operations,
// hence identical results):  Y = (alpha*rs*acc + beta*B + gamma*Z)/div + p*P + q*Q
template <int V>
__device__ __forceinline__ void poly_epilogue(const PolyArgs& a, int64_t row, int f,
                                              typename VecT<V>::type acc, float rsv) {
  using vt = typename VecT<V>::type;
  const float* __restrict__ X = a.X;
  vt out;
#pragma unroll
  for (int i = 0; i < V; ++i) vget(out, i) = a.alpha * (rsv * vget(acc, i));
  if (a.beta != 0.f) {
    vt xr = a.B ? vload<V>(a.B + row * a.ldb + f) : vload<V>(X + row * a.ldx + f);
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
  if (a.nt_store)
    vstore_nt<V>(a.Y + row * a.ldy + f, out);
  else
    vstore<V>(a.Y + row * a.ldy + f, out);
}

// Entries j .. j+rem-1 (rem <= NB) of the row's staged chunk in ONE batch: all
// rem gathers issued before the first add, the adds in CSR order (so bitwise
// the same sums as one entry at a time).  Without it a row's last entries
// were one dependent gather each, and a ZINC row has 2-6 entries in all:
// 3-4 round trips to L2 per row instead of one.  Source lanes past the group
// wrap (__shfl width LPR); their values are never used.
template <int V, int NB, int LPR>
__device__ __forceinline__ void gather_batch(const float* __restrict__ X, int64_t ldx, int f,
                                             bool fok, int cm, float wm, int j, int rem,
                                             typename VecT<V>::type& acc) {
  using vt = typename VecT<V>::type;
  int c[NB];
  float w[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    c[u] = __shfl(cm, j + u, LPR);
    w[u] = __shfl(wm, j + u, LPR);
  }
  if (!fok) return;
  vt x[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u)
    if (u < rem) x[u] = vload<V>(X + (int64_t)c[u] * ldx + f);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    float s = vget(acc, i);
#pragma unroll
    for (int u = 0; u < NB; ++u)
      if (u < rem) s = s + w[u] * vget(x[u], i);
    vget(acc, i) = s;
  }
}

// DEPTH gathers in flight per lane (4; 8 for long rows, k_poly_step_deep).
// Loads are issued DEPTH at a time, the adds stay in CSR order (bitwise the
// same result for any DEPTH).  A staged chunk of <= 8 entries (every ZINC
// row) and the < 4 entries after the 4-batches go as one gather_batch
// (same-process A/B at the cfg2 step: +0.3-0.6 %; the L0 Laguerre step
// 5.95 -> 5.6 us in a chain, profiles/r03_l_ab_poly_batch.txt).
template <int V, int LPR, int DEPTH>
__device__ __forceinline__ void poly_step_body(const PolyArgs& a, Blk blk) {
  using vt = typename VecT<V>::type;
  // XCD-aware slots: blocks are dealt round-robin over the 8 XCDs, so block b
  // takes slot range xcd_slot(b): each XCD walks ONE contiguous range of the
  // (optionally locality-ordered) row schedule and its L2 sees the neighbours
  // of the rows it is working on.
  const int64_t slot = ((int64_t)xcd_slot(blk.x, blk.gx) * 256 + threadIdx.x) / LPR;
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
      if (cnt <= 8) {
        gather_batch<V, 8, LPR>(X, a.ldx, f, fok, cm, wm, 0, cnt, acc);
        continue;
      }
      if constexpr (DEPTH == 8) {
        for (; j + 7 < cnt; j += 8) {  // eight gathers in flight per lane
          int c[8];
          float w[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            c[u] = __shfl(cm, j + u, LPR);
            w[u] = __shfl(wm, j + u, LPR);
          }
          if (fok) {
            vt x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = vload<V>(X + (int64_t)c[u] * a.ldx + f);
#pragma unroll
            for (int i = 0; i < V; ++i) {
              float s = vget(acc, i);
#pragma unroll
              for (int u = 0; u < 8; ++u) s = s + w[u] * vget(x[u], i);
              vget(acc, i) = s;
            }
          }
        }
      }
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
      if (j < cnt) gather_batch<V, 3, LPR>(X, a.ldx, f, fok, cm, wm, j, cnt - j, acc);
    }
    if (!fok) continue;
    poly_epilogue<V>(a, row, f, acc, rsv);
  }
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_poly_step(PolyArgs a) {
  poly_step_body<V, LPR, 4>(a, blk_hw());
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_poly_step_deep(PolyArgs a) {
  poly_step_body<V, LPR, 8>(a, blk_hw());
}

// ---------------------------------------------------------------------------
// Second factor of the Hodge-factored L1 (hlhgat_hodge_factor_t):
//   acc = alpha_e (Z[j] - Z[i]) = (-alpha_e) Z[i] + alpha_e Z[j]
// (the CSR order of row e of alpha B1^T), then the same epilogue as
// k_poly_step, so a factored Laguerre / Chebyshev step applies the
// recurrence exactly as the CSR step does; the B operand carries T_k.
// One lane group per edge: the edge's two node rows are the only gathers and
// both are issued before any arithmetic (no rowptr / col hop).
// ---------------------------------------------------------------------------
template <int V, int LPR>
__global__ __launch_bounds__(256) void k_hodge_edge_step(PolyArgs a) {
  using vt = typename VecT<V>::type;
  // kEpg edges per lane group: their ends, then all 2 kEpg node-row gathers,
  // are in flight together (the kernel is a latency chain ends -> Z -> Y;
  // one edge per group left most of the HBM write bandwidth idle)
  constexpr int kEpg = 4;
  const int64_t grp = ((int64_t)xcd_slot(blockIdx.x, gridDim.x) * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  const int64_t s0 = grp * kEpg;
  if (s0 >= a.n_rows) return;  // no cross-lane operations below
  int64_t e[kEpg];
  int2 ij[kEpg];
  float al[kEpg];
#pragma unroll
  for (int u = 0; u < kEpg; ++u) {
    const int64_t sl = s0 + u < a.n_rows ? s0 + u : s0;
    e[u] = a.order ? (int64_t)a.order[sl] : sl;
  }
#pragma unroll
  for (int u = 0; u < kEpg; ++u) {
    ij[u] = a.ends[e[u]];
    al[u] = a.ealpha[e[u]];
  }
  const float* __restrict__ Z = a.X;
  for (int f = sub * V; f < a.d; f += LPR * V) {
    vt zi[kEpg], zj[kEpg];
#pragma unroll
    for (int u = 0; u < kEpg; ++u) {
      zi[u] = vload<V>(Z + (int64_t)ij[u].x * a.ldx + f);
      zj[u] = vload<V>(Z + (int64_t)ij[u].y * a.ldx + f);
    }
#pragma unroll
    for (int u = 0; u < kEpg; ++u) {
      if (s0 + u >= a.n_rows) break;
      vt acc;
#pragma unroll
      for (int c = 0; c < V; ++c) {
        float s = 0.f;
        s = s + (-al[u]) * vget(zi[u], c);
        s = s + al[u] * vget(zj[u], c);
        vget(acc, c) = s;
      }
      poly_epilogue<V>(a, e[u], f, acc, 1.f);
    }
  }
}

// ---------------------------------------------------------------------------
// LDS-staged SpMM / polynomial step over halo tiles (large Laplacians).
//
// At TSP scale (BASELINE config 5: L1 of 4 x 10k-node kNN graphs, n = 207k
// rows, ~20 entries per row) k_poly_step is bound by the L2 -> CU gather
// rate: every entry re-reads a 256-512 B feature row from L2.  Here one
// workgroup owns a halo tile (hlhgat_halo_tiles: a run of the row schedule
// whose rows reference <= max_halo distinct columns, ~5 uses per staged row in
// RCM order).  Prologue: the tile's entries (tile-local column, value; laid
// out in schedule order, so one contiguous range) and row offsets go to LDS
// with bulk coalesced loads.  Then per FS-float feature slice: the halo rows
// of X are staged in LDS (every load of the slice in flight at once), and
// each row group sums its rows' entries from LDS in CSR order.  Same per-row
// summation and epilogue as k_poly_step: bitwise equal results.  Tiles are
// dealt XCD-contiguously (xcd_slot): neighbouring tiles share much of their
// halo and hit the same L2.
// ---------------------------------------------------------------------------
constexpr int kHaloIds = 8;  // halo row ids held per lane (max_halo <= 8 * row groups)

template <int V, int LPR, int NT>
__global__ __launch_bounds__(NT) void k_poly_halo(PolyArgs a) {
  using vt = typename VecT<V>::type;
  constexpr int FS = V * LPR;    // features per staged slice
  constexpr int RG = NT / LPR;   // row groups per workgroup
  constexpr int kHaloThreads = NT;
  extern __shared__ float4 halo_lds[];
  float* img = reinterpret_cast<float*>(halo_lds);            // [max_halo][FS]
  int2* ent = reinterpret_cast<int2*>(img + (int64_t)a.max_halo * FS);  // [max_tnnz] {col, w}
  int* rp = reinterpret_cast<int*>(ent + a.max_tnnz);         // [max_trows + 1]
  const int64_t t = xcd_slot(blockIdx.x, gridDim.x);
  if (t >= a.n_tiles) return;  // whole workgroup: uniform
  const int4 h0 = reinterpret_cast<const int4*>(a.hdr)[2 * t];
  const int2 h1 = reinterpret_cast<const int2*>(a.hdr)[4 * t + 2];
  const int p0 = h0.x, nr = h0.y, hb = h0.z, nh = h0.w, e_lo = h1.x, ne = h1.y;
  const int sub = threadIdx.x % LPR, rg = threadIdx.x / LPR;
  // prologue, one burst: entries + row offsets to LDS, this lane's halo ids
  // to registers (reused by every feature slice)
  int hid[kHaloIds];
#pragma unroll
  for (int u = 0; u < kHaloIds; ++u) {
    const int hh = rg + u * RG;
    hid[u] = hh < nh ? a.hcols[hb + hh] : 0;
  }
  for (int i = threadIdx.x; i < ne; i += kHaloThreads)
    ent[i] = make_int2((int)a.lcol[e_lo + i], __float_as_int(a.sval ? a.sval[e_lo + i] : 1.f));
  for (int r = threadIdx.x; r <= nr; r += kHaloThreads) rp[r] = a.srp[p0 + r] - e_lo;
  // this row group's first row id (epilogue), loaded with the prologue burst
  const int64_t row_first =
      rg < nr ? (a.order ? (int64_t)a.order[p0 + rg] : (int64_t)(p0 + rg)) : 0;
  const float* __restrict__ X = a.X;
  for (int f0 = 0; f0 < a.d; f0 += FS) {
    const int f = f0 + sub * V;
    const bool fok = f < a.d;
    if (f0) __syncthreads();  // the previous slice's readers are done
    {
      vt v[kHaloIds];
#pragma unroll
      for (int u = 0; u < kHaloIds; ++u) {
        const int hh = rg + u * RG;
        if (hh < nh && fok) {
          v[u] = vload<V>(X + (int64_t)hid[u] * a.ldx + f);
        } else {
#pragma unroll
          for (int i = 0; i < V; ++i) vget(v[u], i) = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < kHaloIds; ++u) {
        const int hh = rg + u * RG;
        if (hh < nh) vstore<V>(img + hh * FS + sub * V, v[u]);
      }
    }
    __syncthreads();
    if (!fok) continue;
    for (int r = rg; r < nr; r += RG) {
      const int e0 = rp[r], e1 = rp[r + 1];
      vt acc;
#pragma unroll
      for (int i = 0; i < V; ++i) vget(acc, i) = 0.f;
      int e = e0;
      for (; e + 3 < e1; e += 4) {
        const int2 q0 = ent[e], q1 = ent[e + 1], q2 = ent[e + 2], q3 = ent[e + 3];
        const int c0 = q0.x, c1 = q1.x, c2 = q2.x, c3 = q3.x;
        const float w0 = __int_as_float(q0.y), w1 = __int_as_float(q1.y),
                    w2 = __int_as_float(q2.y), w3 = __int_as_float(q3.y);
        vt x0 = vload<V>(img + c0 * FS + sub * V);
        vt x1 = vload<V>(img + c1 * FS + sub * V);
        vt x2 = vload<V>(img + c2 * FS + sub * V);
        vt x3 = vload<V>(img + c3 * FS + sub * V);
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
      for (; e < e1; ++e) {
        const int2 q = ent[e];
        vt x = vload<V>(img + q.x * FS + sub * V);
        const float w = __int_as_float(q.y);
#pragma unroll
        for (int i = 0; i < V; ++i) vget(acc, i) = vget(acc, i) + w * vget(x, i);
      }
      const int64_t row =
          r == rg ? row_first : (a.order ? (int64_t)a.order[p0 + r] : (int64_t)(p0 + r));
      const float rsv = a.rs ? a.rs[row] : 1.f;
      poly_epilogue<V>(a, row, f, acc, rsv);
    }
  }
}

// longest recurrence the DEMO adjoint fold unrolls
constexpr int DEMO_MAXK = 16;

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

// The TSP readout's x_t2s = |B1^T x_t| / 2 per edge (lib/Hodge_ST_Model.py:
// 846-848: sparse.mm(par_1^T, x_t), .abs(), / 2) in one pass, and its
// backward's edge factor (g / 2) * sgn(x_j - x_i) (DivBackward, AbsBackward)
// before the B1 product: the arithmetic of the unfused ops, bit for bit.
// BWD: a.z holds g; out = the edge factor.
template <bool BWD, int V, int LPR>
__device__ __forceinline__ void edge_absdiff_body(const Gather2Args& a) {
  using vt = typename VecT<V>::type;
  const int64_t e = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (e >= a.n_edges) return;
  const int64_t i = a.ei[e];
  const int64_t j = a.ei[a.n_edges + e];
  for (int f = sub * V; f < a.d; f += LPR * V) {
    vt xi = vload<V>(a.x + i * a.ldx + f);
    vt xj = vload<V>(a.x + j * a.ldx + f);
    vt o;
    if (BWD) {
      vt g = vload<V>(a.z + e * a.ldz + f);
#pragma unroll
      for (int c = 0; c < V; ++c) {
        const float dd = -vget(xi, c) + vget(xj, c);
        const float sg = dd > 0.f ? 1.f : (dd < 0.f ? -1.f : 0.f);  // torch.sgn
        vget(o, c) = (vget(g, c) * 0.5f) * sg;
      }
    } else {
#pragma unroll
      for (int c = 0; c < V; ++c) vget(o, c) = fabsf(-vget(xi, c) + vget(xj, c)) * 0.5f;
    }
    vstore<V>(a.out + e * a.ldo + f, o);
  }
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_edge_absdiff_fwd(Gather2Args a) {
  edge_absdiff_body<false, V, LPR>(a);
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_edge_absdiff_bwd(Gather2Args a) {
  edge_absdiff_body<true, V, LPR>(a);
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
  int64_t n_rows;   // bwd, contiguous segments: rows of dx (0 = no fill)
  int64_t n_fill;   // bwd: lane groups after the segment groups that zero-fill
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
    int t = r0;
    // 8 member rows in flight, summed in member order (the sequential sum)
    for (; t + 8 <= r1; t += 8) {
      vt xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t r = a.rows ? a.rows[t + u] : t + u;
        xv[u] = vload<V>(a.x + r * a.ldx + f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int c = 0; c < V; ++c) vget(acc, c) = vget(acc, c) + vget(xv[u], c);
    }
    for (; t < r1; ++t) {
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

// dx[r] = dout[s] / max(|seg s|, 1) for each member r of segment s.  With
// contiguous segments the lane groups after the first n_seg write exact
// zeros into the rows no segment covers, [0, ptr[0]) and [ptr[n_seg], n_rows)
// (the adjoint of global_mean_pool is zero there, lib/Hodge_ST_Model.py:636):
// padding rows of a padded batch never carry uninitialised memory upstream.
template <int V, int LPR>
__global__ __launch_bounds__(256) void k_segment_mean_bwd(SegArgs a) {
  using vt = typename VecT<V>::type;
  const int64_t s = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (s >= a.n_seg) {
    const int64_t z = s - a.n_seg;
    if (z >= a.n_fill) return;
    vt zero;
#pragma unroll
    for (int c = 0; c < V; ++c) vget(zero, c) = 0.f;
    if (a.rows) {
      // listed members covering every row (hlhgat_pool_mean_bwd): the
      // trailing bucket n_seg lists the rows in no segment, zeroed here
      for (int64_t t = a.ptr[a.n_seg] + z; t < a.ptr[a.n_seg + 1]; t += a.n_fill) {
        const int64_t r = a.rows[t];
        for (int f = sub * V; f < a.d; f += LPR * V) vstore<V>(a.out + r * a.ldo + f, zero);
      }
      return;
    }
    const int64_t lo = a.ptr[0], hi = a.ptr[a.n_seg];
    for (int64_t r = z; r < a.n_rows; r += a.n_fill) {
      if (r >= lo && r < hi) {
        r = hi - 1 - ((hi - 1 - z) % a.n_fill);  // next stride point >= hi
        continue;
      }
      for (int f = sub * V; f < a.d; f += LPR * V) vstore<V>(a.out + r * a.ldo + f, zero);
    }
    return;
  }
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
// Reverse sweep of the DEMO recurrence (HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py
// :552-568) for one element:  T_1 = x - S,  T_{k+1} = (-S + (2k+1) T_k -
// k T_{k-1})/(k+1) with S = L x.  In: G_k = dLoss/dT_k (G_0 = direct dX).
// Out: block 0 = direct dX, block 1 = dS.
struct DemoArgs {
  float* G;
  int64_t blk;
  int K;
};

__global__ __launch_bounds__(256) void k_demo_adjoint_fold(DemoArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.blk) return;
  float g[DEMO_MAXK];
#pragma unroll
  for (int k = 0; k < DEMO_MAXK; ++k) g[k] = k < a.K ? a.G[k * a.blk + i] : 0.f;
  float ds = 0.f;
#pragma unroll
  for (int k = DEMO_MAXK - 1; k >= 2; --k) {  // T_k from T_{k-1}, T_{k-2}, S
    if (k >= a.K) continue;
    const float gk = g[k] / (float)k;
    g[k - 1] = g[k - 1] + (float)(2 * k - 1) * gk;
    g[k - 2] = g[k - 2] - (float)(k - 1) * gk;
    ds = ds - gk;
  }
  a.G[i] = g[0] + g[1];       // T_1 = x - S
  a.G[a.blk + i] = ds - g[1];
}

double poly_bytes(const PolyArgs& a, int64_t nnz) {
  double b = (double)nnz * (a.val ? 8.0 : 4.0) + 4.0 * (double)(a.n_rows + 1);
  double row_bytes = 4.0 * (double)a.n_rows * a.d;
  int dense = 2;  // gathered X (read once) + Y written
  if (a.B) dense++;
  if (a.Z) dense++;
  if (a.P) dense++;
  if (a.Q) dense++;
  if (a.rs) b += 4.0 * a.n_rows;
  return b + dense * row_bytes;
}

// LDS of one halo-tile workgroup: the X image (<= kHaloImgBytes) plus the
// tile's entries and row offsets; <= 64 KB keeps >= 2 workgroups per CU.
constexpr size_t kHaloImgBytes = 32 * 1024;
constexpr double kNtStoreBytes = 48.0 * 1024 * 1024;
constexpr size_t kHaloLdsBytes = 64 * 1024;

int launch_poly(PolyArgs& a, int64_t nnz, hipStream_t s, int prof_class = HLHGAT_PROF_POLY,
                double prof_bytes = -1.0) {
  HLH_CHECK_ARG(a.n_rows >= 0 && a.n_rows < (int64_t)INT32_MAX,
                "poly_step: n_rows out of range");
  HLH_CHECK_ARG(a.d > 0, "poly_step: d must be > 0");
  HLH_CHECK_ARG(a.rowptr && (nnz == 0 || a.col) && a.X && a.Y,
                "poly_step: NULL pointer");
  HLH_CHECK_ARG(a.ldx >= a.d && a.ldy >= a.d, "poly_step: ld < d");
  HLH_CHECK_ARG(!a.B || a.ldb >= a.d, "poly_step: ldb < d");
  HLH_CHECK_ARG(!a.Z || a.ldz >= a.d, "poly_step: ldz < d");
  HLH_CHECK_ARG(!a.P || a.ldp >= a.d, "poly_step: ldp < d");
  HLH_CHECK_ARG(!a.Q || a.ldq >= a.d, "poly_step: ldq < d");
  HLH_CHECK_ARG(a.div != 0.f, "poly_step: div == 0");
  if (a.n_rows == 0) return HLHGAT_OK;
  const int v = pick_vec(a.d, {a.ldx, a.ldy, a.Z ? a.ldz : 4, a.P ? a.ldp : 4,
                               a.Q ? a.ldq : 4, a.B ? a.ldb : 4},
                         {a.X, a.Y, a.Z, a.P, a.Q, a.B});
  const int l = pick_lpr(a.d, v);
  // Streaming stores of Y once Y is a sizeable fraction of the 256 MB MALL
  // (config 5: 53-106 MB per basis term): the stores then stop evicting the
  // gathered X rows; measured on the TSP L1 Laguerre step at d = 128: 164 ->
  // 116 us (profiles/r01_g_tsp_spmm.log).  Small (ZINC) operators keep
  // ordinary stores -- their consumer re-reads Y from L2 / MALL right away.
  a.nt_store = (double)a.n_rows * a.d * 4.0 >= kNtStoreBytes;
  ProfScope prof(prof_class, s, prof_bytes >= 0.0 ? prof_bytes : poly_bytes(a, nnz),
                 2.0 * (double)nnz * a.d);
  if (a.lcol && a.n_tiles > 0) {
    // slice width FS = v * lh: the widest power of two whose halo image fits
    // kHaloImgBytes (several workgroups per CU), capped by the row's lanes
    int lh = l > 16 ? 16 : l;
    while (lh > 1 && (size_t)a.max_halo * v * lh * sizeof(float) > kHaloImgBytes) lh >>= 1;
    // small tiles: 256-thread workgroups (more of them per CU); else 1024
    const int nt = a.max_trows * lh <= 128 ? 128 : (a.max_trows * lh <= 256 ? 256 : 1024);
    const bool ids_fit = a.max_halo <= kHaloIds * (nt / lh) && a.max_trows * lh <= 1024 * 8;
    const size_t img = (size_t)a.max_halo * v * lh * sizeof(float);
    const size_t shmem = img + (size_t)a.max_tnnz * sizeof(int2) +
                         (size_t)(a.max_trows + 1) * sizeof(int) + 16;
    if (shmem <= kHaloLdsBytes && ids_fit) {
      a.halo_fs = v * lh;
      const unsigned grid = (unsigned)a.n_tiles;
      switch (v * 100 + lh) {
#define HLH_HALO_CASE(VV, LL) \
  case VV * 100 + LL:                                                                   \
    if (nt == 128)                                                                      \
      launch(k_poly_halo<VV, LL, 128>, grid, 128, (uint32_t)shmem, s, &prof, a);        \
    else if (nt == 256)                                                                 \
      launch(k_poly_halo<VV, LL, 256>, grid, 256, (uint32_t)shmem, s, &prof, a);        \
    else                                                                                \
      launch(k_poly_halo<VV, LL, 1024>, grid, 1024, (uint32_t)shmem, s, &prof, a);      \
    break;
        HLH_HALO_CASE(1, 1) HLH_HALO_CASE(1, 2) HLH_HALO_CASE(1, 4) HLH_HALO_CASE(1, 8)
        HLH_HALO_CASE(1, 16) HLH_HALO_CASE(2, 1) HLH_HALO_CASE(2, 2) HLH_HALO_CASE(2, 4)
        HLH_HALO_CASE(2, 8) HLH_HALO_CASE(2, 16) HLH_HALO_CASE(4, 1) HLH_HALO_CASE(4, 2)
        HLH_HALO_CASE(4, 4) HLH_HALO_CASE(4, 8) HLH_HALO_CASE(4, 16)
#undef HLH_HALO_CASE
        default: break;
      }
      HLH_CHECK_LAUNCH();
      return HLHGAT_OK;
    }
  }
  // long rows (>= 12 entries on average: high-degree L1 such as the DEMO brain
  // skeleton's 152 per row) keep 8 gathers in flight per lane
  if (a.n_rows > 0 && nnz >= 12 * a.n_rows && l >= 8)
    HLH_DISPATCH_VL(v, l, k_poly_step_deep, a.n_rows, s, a, &prof);
  else
    HLH_DISPATCH_VL(v, l, k_poly_step, a.n_rows, s, a, &prof);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

PolyArgs make_args(const int32_t* rowptr, const int32_t* col, const float* val,
                   int64_t n, const float* X, int64_t ldx, int64_t d, float* Y,
                   int64_t ldy, const int32_t* order = nullptr,
                   const hlhgat_halo_t* halo = nullptr) {
  PolyArgs a{};
  a.order = order;
  if (halo && halo->lcol && halo->srp && halo->hdr && halo->n_tiles > 0) {
    a.hdr = halo->hdr;
    a.htile = halo->tile_ptr;
    a.hptr = halo->halo_ptr;
    a.hcols = halo->halo;
    a.srp = halo->srp;
    a.lcol = halo->lcol;
    a.sval = halo->sval;
    a.n_tiles = halo->n_tiles;
    a.max_halo = halo->max_halo;
    a.max_trows = halo->max_rows;
    a.max_tnnz = halo->max_nnz;
  }
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

// One application of the Hodge-factored L1 inside a poly step `a` (built as
// for the CSR path: a.X = the SpMM operand, epilogue fields set):
//   stage 1: work = B1 a.X            (k_poly_step over the signed incidence)
//   stage 2: a.Y = epilogue(alpha B1^T work)   (k_hodge_edge_step)
// The beta term keeps reading the ORIGINAL operand (a.B), as the CSR step
// reads X.
int launch_factored(PolyArgs a, const hlhgat_hodge_factor_t& f, float* work, hipStream_t s) {
  HLH_CHECK_ARG(f.node_rowptr && f.ends && f.alpha && work && a.n_rows == f.n_edges &&
                    (f.n_edges == 0 || (f.node_edge && f.node_sign)),
                "hodge factor: incomplete descriptor or row count %lld != n_edges %lld",
                (long long)a.n_rows, (long long)f.n_edges);
  HLH_CHECK_ARG(!a.rs, "hodge factor: row scale not supported");
  if (a.n_rows == 0) return HLHGAT_OK;
  if (a.beta != 0.f && !a.B) {
    a.B = a.X;
    a.ldb = a.ldx;
  }
  {
    PolyArgs b = make_args(f.node_rowptr, f.node_edge, f.node_sign, f.n_nodes, a.X, a.ldx, a.d,
                           work, a.d, f.node_order);
    // own algorithmic bytes: incidence CSR, the E edge rows of X read once, Z written
    const double b1 = 16.0 * (double)f.n_edges + 4.0 * (double)(f.n_nodes + 1) +
                      4.0 * (double)(f.n_edges + f.n_nodes) * a.d;
    int rc = launch_poly(b, 2 * f.n_edges, s, HLHGAT_PROF_HODGE_NODE, b1);
    if (rc) return rc;
  }
  a.X = work;
  a.ldx = a.d;
  a.order = f.edge_order;
  a.ends = reinterpret_cast<const int2*>(f.ends);
  a.ealpha = f.alpha;
  a.lcol = nullptr;
  a.n_tiles = 0;
  const int v = pick_vec(a.d, {a.ldx, a.ldy, a.Z ? a.ldz : 4, a.P ? a.ldp : 4, a.Q ? a.ldq : 4,
                               a.B ? a.ldb : 4},
                         {a.X, a.Y, a.Z, a.P, a.Q, a.B});
  const int l = pick_lpr(a.d, v);
  a.nt_store = (double)a.n_rows * a.d * 4.0 >= kNtStoreBytes;
  // own algorithmic bytes: ends + alpha, Z read once, Y and the dense epilogue operands
  int dense = 1 + (a.beta != 0.f) + (a.Z != nullptr) + (a.P != nullptr) + (a.Q != nullptr);
  ProfScope prof(HLHGAT_PROF_HODGE_EDGE, s,
                 12.0 * (double)a.n_rows + 4.0 * (double)(f.n_nodes + dense * a.n_rows) * a.d,
                 4.0 * (double)a.n_rows * a.d);
  HLH_DISPATCH_VL(v, l, k_hodge_edge_step, ceil_div(a.n_rows, (int64_t)4), s, a, &prof);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// Runs one poly step on the CSR operator, or factored when fac != NULL.
struct StepRunner {
  int64_t nnz;
  const hlhgat_hodge_factor_t* fac;
  float* work;
  hipStream_t s;
  int prof_class = HLHGAT_PROF_POLY;  // the adjoint recurrence: HLHGAT_PROF_POLY_ADJ
  int operator()(PolyArgs& a) const {
    return fac ? launch_factored(a, *fac, work, s) : launch_poly(a, nnz, s, prof_class);
  }
};

}  // namespace

using namespace hlhgat;

extern "C" int hlhgat_spmm(const int32_t* rowptr, const int32_t* col,
                           const float* val, int64_t n_rows, int64_t nnz,
                           const int32_t* row_order, const hlhgat_halo_t* halo,
                           const float* X, int64_t ldx,
                           int64_t d, float* Y, int64_t ldy, void* stream) {
  PolyArgs a = make_args(rowptr, col, val, n_rows, X, ldx, d, Y, ldy, row_order, halo);
  return launch_poly(a, nnz, as_stream(stream));
}

extern "C" int hlhgat_poly_step(const int32_t* rowptr, const int32_t* col,
                                const float* val, const float* rs,
                                int64_t n_rows, int64_t nnz,
                                const int32_t* row_order, const hlhgat_halo_t* halo,
                                const float* X,
                                int64_t ldx, int64_t d, const float* Z,
                                int64_t ldz, const float* P, int64_t ldp,
                                const float* Q, int64_t ldq, float alpha,
                                float beta, float gamma, float div, float p,
                                float q, float* Y, int64_t ldy, void* stream) {
  PolyArgs a = make_args(rowptr, col, val, n_rows, X, ldx, d, Y, ldy, row_order, halo);
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

extern "C" int hlhgat_incidence_step(const int32_t* rowptr, const int32_t* col,
                                     const float* val, const float* rs, int64_t n_rows,
                                     int64_t nnz, int64_t n_src, const float* X, int64_t ldx,
                                     int64_t d, const float* Z, int64_t ldz, float alpha,
                                     float gamma, float* Y, int64_t ldy, void* stream) {
  HLH_CHECK_ARG(n_src >= 0, "incidence_step: n_src < 0");
  PolyArgs a = make_args(rowptr, col, val, n_rows, X, ldx, d, Y, ldy);
  a.rs = rs;
  a.Z = Z;
  a.ldz = ldz;
  a.alpha = alpha;
  a.gamma = gamma;
  a.div = 1.f;
  // algorithmic bytes: the incidence CSR once, the n_src gathered rows once,
  // Y written, Z / rs read once
  const double bytes = (double)nnz * (val ? 8.0 : 4.0) + 4.0 * (double)(n_rows + 1) +
                       4.0 * (double)n_src * d + 4.0 * (double)n_rows * d * (Z ? 2.0 : 1.0) +
                       (rs ? 4.0 * (double)n_rows : 0.0);
  return launch_poly(a, nnz, as_stream(stream), HLHGAT_PROF_INCIDENCE, bytes);
}

namespace {
int basis_fwd_core(int kind, const int32_t* rowptr, const int32_t* col, const float* val,
                   int64_t n, int64_t nnz, const int32_t* row_order, const hlhgat_halo_t* halo,
                   const float* X, int64_t ldx, int64_t F, int K, float* T,
                   const hlhgat_hodge_factor_t* fac, float* work, void* stream) {
  HLH_CHECK_ARG(kind == HLHGAT_POLY_LAGUERRE || kind == HLHGAT_POLY_CHEB ||
                    kind == HLHGAT_POLY_LAGUERRE_DEMO,
                "poly_basis_fwd: bad kind %d", kind);
  HLH_CHECK_ARG(K >= 1, "poly_basis_fwd: K must be > 0 (assert K > 0)");
  if (K == 1 || n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(T, "poly_basis_fwd: T is NULL");
  hipStream_t s = as_stream(stream);
  const StepRunner run{nnz, fac, work, s};
  const int64_t blk = n * F;
  auto Tk = [&](int k) -> float* { return T + (int64_t)(k - 1) * blk; };
  // T_1
  {
    PolyArgs a = make_args(rowptr, col, val, n, X, ldx, F, Tk(1), F, row_order, halo);
    if (kind != HLHGAT_POLY_CHEB) {  // Tx_1 = x - L x   (:494; DEMO :554)
      a.alpha = -1.f;
      a.beta = 1.f;
    }  // Cheb: Tx_1 = L x   (:416)
    int rc = run(a);
    if (rc) return rc;
  }
  for (int k = 1; k + 1 < K; ++k) {
    const float* prev = (k == 1) ? X : Tk(k - 1);
    const int64_t ldprev = (k == 1) ? ldx : F;
    PolyArgs a = make_args(rowptr, col, val, n, Tk(k), F, F, Tk(k + 1), F, row_order, halo);
    a.Z = prev;
    a.ldz = ldprev;
    if (kind == HLHGAT_POLY_LAGUERRE_DEMO) {
      // DEMO fork: Tx_2 = (-L x + (2k+1) Tx_1 - k Tx_0) / (k+1) -- the SpMM
      // operand is the layer INPUT x at every k
      // (HL-HGAT-DEMO/lib/Hodge_Cheb_Conv.py:561,566)
      a.X = X;
      a.ldx = ldx;
      a.B = Tk(k);
      a.ldb = F;
      a.alpha = -1.f;
      a.beta = (float)(2 * k + 1);
      a.gamma = -(float)k;
      a.div = (float)(k + 1);
    } else if (kind == HLHGAT_POLY_LAGUERRE) {
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
    int rc = run(a);
    if (rc) return rc;
  }
  return HLHGAT_OK;
}

int basis_bwd_core(int kind, const int32_t* rowptr_t, const int32_t* col_t,
                   const float* val_t, int64_t n, int64_t nnz, const int32_t* row_order,
                   const hlhgat_halo_t* halo, int64_t F, int K, float* G,
                   const hlhgat_hodge_factor_t* fac, float* work, void* stream) {
  HLH_CHECK_ARG(kind == HLHGAT_POLY_LAGUERRE || kind == HLHGAT_POLY_CHEB ||
                    kind == HLHGAT_POLY_LAGUERRE_DEMO,
                "poly_basis_bwd: bad kind %d", kind);
  HLH_CHECK_ARG(K >= 1, "poly_basis_bwd: K must be > 0");
  if (K == 1 || n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(G, "poly_basis_bwd: G is NULL");
  hipStream_t s = as_stream(stream);
  const StepRunner run{nnz, fac, work, s, HLHGAT_PROF_POLY_ADJ};
  const int64_t blk = n * F;
  auto Gk = [&](int k) -> float* { return G + (int64_t)k * blk; };
  if (kind == HLHGAT_POLY_LAGUERRE_DEMO) {
    // Every T_k (k >= 1) depends on x through S = L x and the recurrence:
    // one elementwise reverse sweep folds G_K-1..G_1 into dS (block 1) and
    // the direct part of dX (block 0), then dX += L^T dS.
    HLH_CHECK_ARG(K <= DEMO_MAXK, "poly_basis_bwd: DEMO recurrence needs K <= %d", DEMO_MAXK);
    DemoArgs d{G, n * F, K};
    launch(k_demo_adjoint_fold, dim3((unsigned)ceil_div(n * F, (int64_t)256)), dim3(256), 0, s,
           nullptr, d);
    HLH_CHECK_LAUNCH();
    PolyArgs a = make_args(rowptr_t, col_t, val_t, n, Gk(1), F, F, Gk(0), F, row_order, halo);
    a.P = Gk(0);
    a.ldp = F;
    a.p = 1.f;
    return run(a);
  }
  for (int k = K - 1; k >= 1; --k) {
    PolyArgs a = make_args(rowptr_t, col_t, val_t, n, Gk(k), F, F, Gk(k - 1), F, row_order, halo);
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
    int rc = run(a);
    if (rc) return rc;
  }
  return HLHGAT_OK;
}

}  // namespace

extern "C" int hlhgat_poly_basis_fwd(int kind, const int32_t* rowptr, const int32_t* col,
                                     const float* val, int64_t n, int64_t nnz,
                                     const int32_t* row_order, const hlhgat_halo_t* halo,
                                     const float* X, int64_t ldx, int64_t F, int K, float* T,
                                     void* stream) {
  return basis_fwd_core(kind, rowptr, col, val, n, nnz, row_order, halo, X, ldx, F, K, T,
                        nullptr, nullptr, stream);
}

extern "C" int hlhgat_poly_basis_bwd(int kind, const int32_t* rowptr_t, const int32_t* col_t,
                                     const float* val_t, int64_t n, int64_t nnz,
                                     const int32_t* row_order, const hlhgat_halo_t* halo,
                                     int64_t F, int K, float* G, void* stream) {
  return basis_bwd_core(kind, rowptr_t, col_t, val_t, n, nnz, row_order, halo, F, K, G,
                        nullptr, nullptr, stream);
}

extern "C" int64_t hlhgat_hodge_factor_work_floats(int64_t n_nodes, int64_t F) {
  return n_nodes > 0 && F > 0 ? n_nodes * F : 1;
}

extern "C" int hlhgat_hodge_spmm(const hlhgat_hodge_factor_t* f, const float* X, int64_t ldx,
                                 int64_t d, float* Y, int64_t ldy, float* work, void* stream) {
  HLH_CHECK_ARG(f, "hodge_spmm: NULL factor");
  HLH_CHECK_ARG(d > 0 && ldx >= d && ldy >= d && X && Y, "hodge_spmm: bad operands");
  PolyArgs a = make_args(nullptr, nullptr, nullptr, f->n_edges, X, ldx, d, Y, ldy);
  return launch_factored(a, *f, work, as_stream(stream));
}

extern "C" int hlhgat_hodge_poly_step(const hlhgat_hodge_factor_t* f, const float* X,
                                      int64_t ldx, int64_t d, const float* Z, int64_t ldz,
                                      const float* P, int64_t ldp, const float* Q, int64_t ldq,
                                      float alpha, float beta, float gamma, float div, float p,
                                      float q, float* Y, int64_t ldy, float* work, void* stream) {
  HLH_CHECK_ARG(f, "hodge_poly_step: NULL factor");
  HLH_CHECK_ARG(d > 0 && ldx >= d && ldy >= d && X && Y && (!Z || ldz >= d) &&
                    (!P || ldp >= d) && (!Q || ldq >= d) && div != 0.f,
                "hodge_poly_step: bad operands");
  PolyArgs a = make_args(nullptr, nullptr, nullptr, f->n_edges, X, ldx, d, Y, ldy);
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
  return launch_factored(a, *f, work, as_stream(stream));
}

extern "C" int hlhgat_poly_basis_fwd_factored(int kind, const hlhgat_hodge_factor_t* f,
                                              const float* X, int64_t ldx, int64_t F, int K,
                                              float* T, float* work, void* stream) {
  HLH_CHECK_ARG(f, "poly_basis_fwd_factored: NULL factor");
  return basis_fwd_core(kind, nullptr, nullptr, nullptr, f->n_edges, 0, nullptr, nullptr, X, ldx,
                        F, K, T, f, work, stream);
}

extern "C" int hlhgat_poly_basis_bwd_factored(int kind, const hlhgat_hodge_factor_t* f,
                                              int64_t F, int K, float* G, float* work,
                                              void* stream) {
  HLH_CHECK_ARG(f, "poly_basis_bwd_factored: NULL factor");
  return basis_bwd_core(kind, nullptr, nullptr, nullptr, f->n_edges, 0, nullptr, nullptr, F, K,
                        G, f, work, stream);
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
  // algorithmic bytes: the edge list, the two gathered rows per
  // edge, the out rows written (and read when accumulating), z and the scales
  const double gb = 16.0 * (double)n_edges +
                    4.0 * (double)n_edges * d * (2.0 + 1.0 + (accumulate ? 1.0 : 0.0) +
                                                 (z ? 1.0 : 0.0)) +
                    ((sa ? 4.0 : 0.0) + (sb ? 4.0 : 0.0)) * (double)n_edges;
  ProfScope prof(HLHGAT_PROF_GATHER2, s, gb, 4.0 * (double)n_edges * d);
  HLH_DISPATCH_VL(v, l, k_edge_gather2, n_edges, s, a, &prof);
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
  SegArgs a{seg_ptr, seg_rows, n_seg, x, ldx, (int)d, out, ldo, 0, 0};
  const int v = pick_vec(d, {ldx, ldo}, {x, out});
  const int l = pick_lpr(d, v);
  hipStream_t s = as_stream(stream);
  HLH_DISPATCH_VL(v, l, k_segment_mean_fwd, n_seg, s, a, nullptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_edge_absdiff(const int64_t* edge_index, int64_t n_edges, const float* x,
                                   int64_t ldx, int64_t d, const float* g, int64_t ldg,
                                   float* out, int64_t ldo, void* stream) {
  HLH_CHECK_ARG(n_edges >= 0 && d > 0 && ldx >= d && ldo >= d && (!g || ldg >= d),
                "edge_absdiff: bad sizes");
  if (n_edges == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(edge_index && x && out, "edge_absdiff: NULL pointer");
  Gather2Args a{edge_index, n_edges, x, ldx, (int)d, nullptr, nullptr, -1.f, 1.f, g,
                g ? ldg : 0, out, ldo, 0};
  const int v = pick_vec(d, {ldx, ldo, g ? ldg : 4}, {x, out, g});
  const int l = pick_lpr(d, v);
  hipStream_t s = as_stream(stream);
  if (g)
    HLH_DISPATCH_VL(v, l, k_edge_absdiff_bwd, n_edges, s, a, nullptr);
  else
    HLH_DISPATCH_VL(v, l, k_edge_absdiff_fwd, n_edges, s, a, nullptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_pool_mean_bwd(const int32_t* seg_ptr, const int32_t* seg_rows,
                                    int64_t n_seg, const float* dout, int64_t ldo, int64_t d,
                                    float* dx, int64_t ldx, int64_t n_rows, void* stream) {
  HLH_CHECK_ARG(n_seg >= 0 && d > 0 && ldx >= d && ldo >= d && n_rows >= 0,
                "pool_mean_bwd: bad sizes");
  if (n_rows == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(seg_ptr && seg_rows && dx && (n_seg == 0 || dout),
                "pool_mean_bwd: NULL pointer");
  // lane groups after the segment groups stride over the zero bucket
  const int64_t n_fill = n_rows < 1024 ? n_rows : 1024;
  SegArgs a{seg_ptr, seg_rows, n_seg, dout, ldo, (int)d, dx, ldx, n_rows, n_fill};
  const int v = pick_vec(d, {ldx, ldo}, {dout, dx});
  const int l = pick_lpr(d, v);
  hipStream_t s = as_stream(stream);
  HLH_DISPATCH_VL(v, l, k_segment_mean_bwd, n_seg + n_fill, s, a, nullptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_segment_mean_bwd(const int32_t* seg_ptr,
                                       const int32_t* seg_rows, int64_t n_seg,
                                       const float* dout, int64_t ldo, int64_t d,
                                       float* dx, int64_t ldx, int64_t n_rows,
                                       void* stream) {
  HLH_CHECK_ARG(n_seg >= 0 && d > 0 && ldx >= d && ldo >= d && n_rows >= 0,
                "segment_mean_bwd: bad sizes");
  // listed members (scatter_mean): the caller zero-fills dx; no fill here
  const int64_t n_fill = seg_rows ? 0 : (n_rows < 1024 ? n_rows : 1024);
  if (n_seg == 0 && n_fill == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(seg_ptr && dx && (n_seg == 0 || dout), "segment_mean_bwd: NULL pointer");
  SegArgs a{seg_ptr, seg_rows, n_seg, dout, ldo, (int)d, dx, ldx, n_rows, n_fill};
  const int v = pick_vec(d, {ldx, ldo}, {dout, dx});
  const int l = pick_lpr(d, v);
  hipStream_t s = as_stream(stream);
  HLH_DISPATCH_VL(v, l, k_segment_mean_bwd, n_seg + n_fill, s, a, nullptr);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}
