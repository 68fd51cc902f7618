// Dense per-simplex projections on the fp32 matrix cores of gfx950.
//
// HodgeLaguerreConv computes out = sum_k lins[k](T_k) + bias
// (lib/Hodge_Cheb_Conv.py:487,497,509,512-513) and NodeEdgeInt computes
// Linear(cat[a, b]) (lib/Hodge_Cheb_Conv.py:307-308).  Both are one GEMM whose
// reduction axis is split over several operand blocks A_b (the basis terms
// T_k, or the two halves of the concatenation), so neither the K separate
// GEMMs + adds nor the torch.cat are materialised.
//
// MFMA: v_mfma_f32_16x16x4_f32 (exact f32 fma chain; 32-cycle issue).  Lane
// l = 16*q + i supplies A[i][k=q] and B[k=q][i]; the four MFMAs of a 16-wide
// k chunk use k = k0 + 4q + j (j = 0..3), which lets every lane fetch its four
// k values of a row with ONE 16-byte load (A and W are both k-contiguous).
// Accumulator register r of lane l holds C[4q + r][i].
//
// Shapes here are skinny (N = d_out <= 256, M = simplices up to millions), so
// the kernels stream A straight into registers (each row read once, W served
// from L1/L2), 4 waves per workgroup stacked along M.
#include "gemm_core.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>

using namespace hlhgat;

namespace {

template <bool VEC>
__device__ __forceinline__ void load_k4(const float* __restrict__ p, int kk,
                                        int kb, bool valid, float (&o)[4]) {
  if (VEC) {
    if (valid && kk < kb) {
      float4 v = *reinterpret_cast<const float4*>(p + kk);
      o[0] = v.x;
      o[1] = v.y;
      o[2] = v.z;
      o[3] = v.w;
    } else {
      o[0] = o[1] = o[2] = o[3] = 0.f;
    }
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = (valid && kk + t < kb) ? p[kk + t] : 0.f;
  }
}

template <int TM, int TN, bool VEC>
__global__ __launch_bounds__(256) void k_proj_fwd(FwdArgs a) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, i = lane & 15;
  const int64_t m_base = ((int64_t)blockIdx.x * 4 + wave) * (TM * 16);
  const int n_base = blockIdx.y * (TN * 16);
  if (m_base >= a.M) return;

  floatx4 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int b = 0; b < a.nb; ++b) {
    const int kb = a.kb[b];
    const float* arow[TM];
    bool aval[TM];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
      const int64_t row = m_base + tm * 16 + i;
      aval[tm] = row < a.M;
      arow[tm] = a.A[b] + (aval[tm] ? row : 0) * a.lda[b];
    }
    const float* wrow[TN];
    bool wval[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int col = n_base + tn * 16 + i;
      wval[tn] = col < a.N;
      wrow[tn] = a.W[b] + (int64_t)(wval[tn] ? col : 0) * a.ldw[b];
    }
    float af[TM][4], bf[TN][4];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) load_k4<VEC>(arow[tm], 4 * q, kb, aval[tm], af[tm]);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) load_k4<VEC>(wrow[tn], 4 * q, kb, wval[tn], bf[tn]);
    for (int k0 = 0; k0 < kb; k0 += 16) {
      // prefetch the next 16-wide chunk while this one feeds the MFMAs
      float an[TM][4], bn[TN][4];
      const int kn = k0 + 16 + 4 * q;
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) load_k4<VEC>(arow[tm], kn, kb, aval[tm], an[tm]);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) load_k4<VEC>(wrow[tn], kn, kb, wval[tn], bn[tn]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = mfma16(af[tm][j], bf[tn][j], acc[tm][tn]);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int t = 0; t < 4; ++t) af[tm][t] = an[tm][t];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int t = 0; t < 4; ++t) bf[tn][t] = bn[tn][t];
    }
  }

#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = n_base + tn * 16 + i;
    if (col >= a.N) continue;
    const float bv = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m_base + tm * 16 + 4 * q + r;
        if (row >= a.M) continue;
        float v = acc[tm][tn][r];
        if (a.bias) v = v + bv;
        float* dst = a.C + row * a.ldc + col;
        *dst = a.accumulate ? *dst + v : v;
      }
    }
  }
}

template <int TN>
__device__ __forceinline__ void proj_fwd_lds_body(const FwdArgs& a, Blk blk,
                                                  float (*wl)[TN * 16][KCP]) {
  const int wave = threadIdx.x >> 6;
  const int64_t m_base = ((int64_t)blk.x * 4 + wave) * 16;
  const int n_base = blk.y * (TN * 16);
  floatx4 acc[TN];
  proj_fwd_lds_mainloop<TN>(a, (int)blk.x, (int)blk.y, wl, acc);

  // every wave is past the loop's last barrier: wl is free for the epilogue
  float* scratch = &wl[0][0][0] + wave * 16 * (TN * 16 + 4);
  const int ncols = a.N - n_base < TN * 16 ? a.N - n_base : TN * 16;
  const bool vec_ok = (a.N % 4) == 0 && (a.ldc % 4) == 0 &&
                      (reinterpret_cast<uintptr_t>(a.C) & 15) == 0;
  store_tile_rows<TN>(acc, scratch, m_base, a.M, a.C + n_base, a.ldc, ncols,
                      a.bias ? a.bias + n_base : nullptr, a.accumulate, vec_ok);
}

// XCD-aware order (a.xcd_map): workgroups are dealt round-robin over the 8
// XCDs, so linear id L goes to XCD L % 8; w = that XCD's (L / 8)-th item of
// ONE contiguous range of the (row block, column tile) items, column tile
// fastest: the gridDim.y column tiles of a row block run at about the same
// time on one XCD and read its A rows from HBM once (the others hit that
// XCD's L2).  With blockIdx.x fastest, a row block's A rows were read once
// per column tile, far apart in time (config 5's N = 256 Linears: 4x A).
__device__ __forceinline__ Blk fwd_item(const FwdArgs& a) {
  if (!a.xcd_map || gridDim.y == 1) return blk_hw();
  const unsigned total = gridDim.x * gridDim.y;
  const unsigned L = blockIdx.x + blockIdx.y * gridDim.x;
  const unsigned x = L & 7u, k = L >> 3, per = total >> 3, extra = total & 7u;
  const unsigned w = x * per + (x < extra ? x : extra) + k;
  return Blk{w / gridDim.y, w % gridDim.y, gridDim.x, gridDim.y};
}

template <int TN>
__global__ __launch_bounds__(256) void k_proj_fwd_lds(FwdArgs a) {
  __shared__ float wl[2][TN * 16][KCP];
  proj_fwd_lds_body<TN>(a, fwd_item(a), wl);
}

// ---------------------------------------------------------------------------
// data gradient: dA_b = dC W_b   (reduction over N)
// ---------------------------------------------------------------------------
struct BwdDataArgs {
  int nb;
  int N;
  int64_t M;
  const float* G;
  int64_t ldg;
  const float* W[MAXB];
  float* O[MAXB];
  int64_t ldw[MAXB];
  int64_t ldo[MAXB];
  int kb[MAXB];
  int tile_start[MAXB + 1];
  int accumulate;
};

template <int TM, int TN, bool VEC>
__global__ __launch_bounds__(256) void k_proj_bwd_data(BwdDataArgs a) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, i = lane & 15;
  const int64_t m_base = ((int64_t)blockIdx.x * 4 + wave) * (TM * 16);
  if (m_base >= a.M) return;
  int b = 0;
  while (b + 1 < a.nb && (int)blockIdx.y >= a.tile_start[b + 1]) ++b;
  const int kb = a.kb[b];
  const int c_base = ((int)blockIdx.y - a.tile_start[b]) * (TN * 16);
  const float* __restrict__ W = a.W[b];
  const int64_t ldw = a.ldw[b];

  floatx4 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};

  const float* grow[TM];
  bool gval[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int64_t row = m_base + tm * 16 + i;
    gval[tm] = row < a.M;
    grow[tm] = a.G + (gval[tm] ? row : 0) * a.ldg;
  }
  int cols[TN];
  bool cval[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    cols[tn] = c_base + tn * 16 + i;
    cval[tn] = cols[tn] < kb;
  }
  for (int r0 = 0; r0 < a.N; r0 += 16) {
    const int kk = r0 + 4 * q;
    float af[TM][4], bf[TN][4];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) load_k4<VEC>(grow[tm], kk, a.N, gval[tm], af[tm]);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[tn][j] = (cval[tn] && kk + j < a.N) ? W[(int64_t)(kk + j) * ldw + cols[tn]] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = mfma16(af[tm][j], bf[tn][j], acc[tm][tn]);
  }
  float* __restrict__ O = a.O[b];
  const int64_t ldo = a.ldo[b];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    if (!cval[tn]) continue;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m_base + tm * 16 + 4 * q + r;
        if (row >= a.M) continue;
        float* dst = O + row * ldo + cols[tn];
        const float v = acc[tm][tn][r];
        *dst = a.accumulate ? *dst + v : v;
      }
    }
  }
}

// Vector path of the data gradient: W_b[n0:n0+64][c_tile] is staged in LDS
// TRANSPOSED (wl[c][n], rows padded) so each lane's B fragment (4 consecutive
// n of one column) is one ds_read_b128; dC rows stream into registers one
// 64-wide n chunk ahead.
template <int TN>
__device__ __forceinline__ void bwd_data_lds_body(const BwdDataArgs& a, int bx, int by,
                                                  float (*wl)[TN * 16][KCP]) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, i = lane & 15;
  const int64_t m_base = ((int64_t)bx * 4 + wave) * 16;
  int b = 0;
  while (b + 1 < a.nb && by >= a.tile_start[b + 1]) ++b;
  const int kb = a.kb[b];
  const int c_base = (by - a.tile_start[b]) * (TN * 16);
  const float* __restrict__ W = a.W[b];
  const int64_t ldw = a.ldw[b];
  const int64_t row = m_base + i;
  const bool gval = row < a.M;
  const float* grow = a.G + (gval ? row : 0) * a.ldg;
  auto load_g = [&](int n0, float4 (&o)[4]) { load_a_chunk(grow, gval, n0, a.N, q, o); };


  // staging: TN*16 columns x 64 n = TN*256 float4 over 256 threads; thread
  // loads W[n][c4*4 .. +3] (a half-wave covers 32 consecutive n of one c4)
  // and scatters the 4 floats into the transposed, swizzled tile
  // (conflict-free ds_write_b32: the 32 lanes hit 32 distinct banks)
  auto load_w = [&](int n0, float4 (&st)[TN]) {
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int idx = threadIdx.x + 256 * u;
      const int nl = idx & 63, c4 = idx >> 6;
      const int n = n0 + nl, c = c_base + 4 * c4;
      if (n < a.N && c < kb)
        st[u] = *reinterpret_cast<const float4*>(W + (int64_t)n * ldw + c);
      else
        st[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_w = [&](float (*lds)[KCP], const float4 (&st)[TN]) {
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int idx = threadIdx.x + 256 * u;
      const int nl = idx & 63, c4 = idx >> 6;
      const int r0 = 4 * c4;
      lds[r0 + 0][4 * wswz(r0 + 0, nl >> 2) + (nl & 3)] = st[u].x;
      lds[r0 + 1][4 * wswz(r0 + 1, nl >> 2) + (nl & 3)] = st[u].y;
      lds[r0 + 2][4 * wswz(r0 + 2, nl >> 2) + (nl & 3)] = st[u].z;
      lds[r0 + 3][4 * wswz(r0 + 3, nl >> 2) + (nl & 3)] = st[u].w;
    }
  };

  floatx4 acc[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) acc[tn] = floatx4{0.f, 0.f, 0.f, 0.f};
  float4 wst[TN], gc[4];
  load_w(0, wst);
  load_g(0, gc);
  store_w(wl[0], wst);
  __syncthreads();
  int buf = 0;
  for (int n0 = 0; n0 < a.N; n0 += KC) {
    const bool has_next = n0 + KC < a.N;
    float4 gn[4];
    if (has_next) {
      load_w(n0 + KC, wst);
      load_g(n0 + KC, gn);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float4 bf[TN];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        bf[tn] = *reinterpret_cast<const float4*>(&wl[buf][tn * 16 + i][4 * wswz(i, 4 * s + q)]);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        acc[tn] = mfma16(gc[s].x, bf[tn].x, acc[tn]);
        acc[tn] = mfma16(gc[s].y, bf[tn].y, acc[tn]);
        acc[tn] = mfma16(gc[s].z, bf[tn].z, acc[tn]);
        acc[tn] = mfma16(gc[s].w, bf[tn].w, acc[tn]);
      }
    }
    if (has_next) {
      store_w(wl[buf ^ 1], wst);
#pragma unroll
      for (int s = 0; s < 4; ++s) gc[s] = gn[s];
    }
    __syncthreads();
    buf ^= 1;
  }
  float* scratch = &wl[0][0][0] + wave * 16 * (TN * 16 + 4);
  const int ncols = kb - c_base < TN * 16 ? kb - c_base : TN * 16;
  const bool vec_ok = (a.ldo[b] % 4) == 0 && (reinterpret_cast<uintptr_t>(a.O[b]) & 15) == 0;
  store_tile_rows<TN>(acc, scratch, m_base, a.M, a.O[b] + c_base, a.ldo[b], ncols, nullptr,
                      a.accumulate, vec_ok);
}

// Data gradient, one workgroup per 64-row block covering EVERY column tile of
// every block (N <= 64: the workgroup's whole dC chunk stays in registers), so
// dC is read once per row block instead of once per column tile; the W tiles
// go through two LDS buffers (the next one loaded while the current one feeds
// the MFMAs) and the epilogue has its own scratch.  Per element the same MFMA
// sequence as bwd_data_lds_body: bitwise the same dA.
template <int TN>
__device__ __forceinline__ void bwd_data_rows_body(const BwdDataArgs& a, int bx, float* lds) {
  float (*wl)[TN * 16][KCP] = reinterpret_cast<float (*)[TN * 16][KCP]>(lds);
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, i = lane & 15;
  float* scratch = lds + 2 * TN * 16 * KCP + wave * 16 * (TN * 16 + 4);
  const int64_t m_base = ((int64_t)bx * 4 + wave) * 16;
  const int64_t row = m_base + i;
  const bool gval = row < a.M;
  float4 gc[4];
  load_a_chunk(a.G + (gval ? row : 0) * a.ldg, gval, 0, a.N, q, gc);
  const int ntiles = a.tile_start[a.nb];
  auto tile_of = [&](int t, int& b, int& c_base) {
    b = 0;
    while (b + 1 < a.nb && t >= a.tile_start[b + 1]) ++b;
    c_base = (t - a.tile_start[b]) * (TN * 16);
  };
  auto load_w = [&](int t, float4 (&st)[TN]) {  // as bwd_data_lds_body's staging
    int b, c_base;
    tile_of(t, b, c_base);
    const float* __restrict__ W = a.W[b];
    const int64_t ldw = a.ldw[b];
    const int kb = a.kb[b];
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int idx = threadIdx.x + 256 * u;
      const int nl = idx & 63, c4 = idx >> 6;
      const int c = c_base + 4 * c4;
      st[u] = (nl < a.N && c < kb) ? *reinterpret_cast<const float4*>(W + (int64_t)nl * ldw + c)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_w = [&](float (*dst)[KCP], const float4 (&st)[TN]) {
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int idx = threadIdx.x + 256 * u;
      const int nl = idx & 63, c4 = idx >> 6;
      const int r0 = 4 * c4;
      dst[r0 + 0][4 * wswz(r0 + 0, nl >> 2) + (nl & 3)] = st[u].x;
      dst[r0 + 1][4 * wswz(r0 + 1, nl >> 2) + (nl & 3)] = st[u].y;
      dst[r0 + 2][4 * wswz(r0 + 2, nl >> 2) + (nl & 3)] = st[u].z;
      dst[r0 + 3][4 * wswz(r0 + 3, nl >> 2) + (nl & 3)] = st[u].w;
    }
  };
  float4 wst[TN];
  load_w(0, wst);
  store_w(wl[0], wst);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const bool has_next = t + 1 < ntiles;
    if (has_next) load_w(t + 1, wst);
    floatx4 acc[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[tn] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float4 bf[TN];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        bf[tn] = *reinterpret_cast<const float4*>(&wl[buf][tn * 16 + i][4 * wswz(i, 4 * s + q)]);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        acc[tn] = mfma16(gc[s].x, bf[tn].x, acc[tn]);
        acc[tn] = mfma16(gc[s].y, bf[tn].y, acc[tn]);
        acc[tn] = mfma16(gc[s].z, bf[tn].z, acc[tn]);
        acc[tn] = mfma16(gc[s].w, bf[tn].w, acc[tn]);
      }
    }
    int b, c_base;
    tile_of(t, b, c_base);
    const int ncols = a.kb[b] - c_base < TN * 16 ? a.kb[b] - c_base : TN * 16;
    const bool vec_ok = (a.ldo[b] % 4) == 0 && (reinterpret_cast<uintptr_t>(a.O[b]) & 15) == 0;
    store_tile_rows<TN>(acc, scratch, m_base, a.M, a.O[b] + c_base, a.ldo[b], ncols, nullptr,
                        a.accumulate, vec_ok);
    if (has_next) store_w(wl[buf ^ 1], wst);
    __syncthreads();
  }
}

template <int TN>
__global__ __launch_bounds__(256) void k_proj_bwd_data_lds(BwdDataArgs a) {
  __shared__ float wl[2][TN * 16][KCP];
  bwd_data_lds_body<TN>(a, (int)blockIdx.x, (int)blockIdx.y, wl);
}

// ---------------------------------------------------------------------------
// weight gradient: dW_b = dC^T A_b  (reduction over M, split over workgroups)
// Each workgroup owns one (64 n x 64 k) output tile of one block and one slice
// of M; its 4 waves take interleaved 16-row chunks of the slice and are summed
// through LDS in wave order; slices are summed in order by k_reduce_splits.
// The bias gradient (column sums of dC) rides along in the k_base == 0 tiles
// of block 0.
// ---------------------------------------------------------------------------
constexpr int WT_TM = 4;  // 64 rows of n per tile
constexpr int WT_TN = 4;  // 64 cols of k per tile
constexpr int WT_ROWS = WT_TM * 16;
constexpr int WT_COLS = WT_TN * 16;

struct BwdWeightArgs {
  int nb;
  int N;
  int64_t M;
  const float* G;
  int64_t ldg;
  const float* A[MAXB];
  int64_t lda[MAXB];
  int kb[MAXB];
  int tile_start[MAXB + 1];
  int64_t part_off[MAXB];
  int64_t bias_off;  // -1: no bias gradient
  int64_t part_stride;
  float* part;
  int64_t rows_per_split;
  int tiles_n;
  int xcd_map;  // remap (tile, split) so each XCD walks one contiguous range of them
};

__global__ __launch_bounds__(256) void k_proj_bwd_weight(BwdWeightArgs a) {
  __shared__ float red[4][WT_TM * WT_TN * 4][64];
  __shared__ float bred[4][WT_TM][64];
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, i = lane & 15;
  int b = 0;
  while (b + 1 < a.nb && (int)blockIdx.y >= a.tile_start[b + 1]) ++b;
  const int t = (int)blockIdx.y - a.tile_start[b];
  const int n_base = (t % a.tiles_n) * WT_ROWS;
  const int k_base = (t / a.tiles_n) * WT_COLS;
  const int kb = a.kb[b];
  const float* __restrict__ A = a.A[b];
  const int64_t lda = a.lda[b];
  const bool do_bias = a.bias_off >= 0 && b == 0 && k_base == 0;

  const int64_t m_lo = (int64_t)blockIdx.z * a.rows_per_split;
  int64_t m_hi = m_lo + a.rows_per_split;
  if (m_hi > a.M) m_hi = a.M;

  floatx4 acc[WT_TM][WT_TN];
#pragma unroll
  for (int tm = 0; tm < WT_TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < WT_TN; ++tn) acc[tm][tn] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum[WT_TM];
#pragma unroll
  for (int tm = 0; tm < WT_TM; ++tm) bsum[tm] = 0.f;

  int ncol[WT_TM];
  bool nval[WT_TM];
#pragma unroll
  for (int tm = 0; tm < WT_TM; ++tm) {
    ncol[tm] = n_base + tm * 16 + i;
    nval[tm] = ncol[tm] < a.N;
  }
  int kcol[WT_TN];
  bool kval[WT_TN];
#pragma unroll
  for (int tn = 0; tn < WT_TN; ++tn) {
    kcol[tn] = k_base + tn * 16 + i;
    kval[tn] = kcol[tn] < kb;
  }

  // operands of one 16-row chunk: lane (q, i) holds rows m0 + 4q + j (j=0..3)
  auto load_chunk = [&](int64_t m0, float (&af)[WT_TM][4], float (&bf)[WT_TN][4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + 4 * q + j;
      const bool mv = m < m_hi;
      const float* grow = a.G + (mv ? m : 0) * a.ldg;
      const float* arow = A + (mv ? m : 0) * lda;
#pragma unroll
      for (int tm = 0; tm < WT_TM; ++tm) af[tm][j] = (mv && nval[tm]) ? grow[ncol[tm]] : 0.f;
#pragma unroll
      for (int tn = 0; tn < WT_TN; ++tn) bf[tn][j] = (mv && kval[tn]) ? arow[kcol[tn]] : 0.f;
    }
  };
  float af[WT_TM][4], bf[WT_TN][4];
  int64_t m0 = m_lo + wave * 16;
  if (m0 < m_hi) load_chunk(m0, af, bf);
  for (; m0 < m_hi; m0 += 64) {
    float an[WT_TM][4], bn[WT_TN][4];
    const bool has_next = m0 + 64 < m_hi;
    if (has_next) load_chunk(m0 + 64, an, bn);  // prefetch the next chunk
    if (do_bias) {
#pragma unroll
      for (int tm = 0; tm < WT_TM; ++tm)
        bsum[tm] = bsum[tm] + ((af[tm][0] + af[tm][1]) + (af[tm][2] + af[tm][3]));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tm = 0; tm < WT_TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < WT_TN; ++tn)
          acc[tm][tn] = mfma16(af[tm][j], bf[tn][j], acc[tm][tn]);
    if (has_next) {
#pragma unroll
      for (int tm = 0; tm < WT_TM; ++tm)
#pragma unroll
        for (int j = 0; j < 4; ++j) af[tm][j] = an[tm][j];
#pragma unroll
      for (int tn = 0; tn < WT_TN; ++tn)
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[tn][j] = bn[tn][j];
    }
  }

  // cross-wave reduction (fixed order: wave 0 + 1 + 2 + 3)
#pragma unroll
  for (int tm = 0; tm < WT_TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < WT_TN; ++tn)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][(tm * WT_TN + tn) * 4 + r][lane] = acc[tm][tn][r];
  if (do_bias) {
#pragma unroll
    for (int tm = 0; tm < WT_TM; ++tm) bred[wave][tm][lane] = bsum[tm];
  }
  __syncthreads();
  float* slab = a.part + (int64_t)blockIdx.z * a.part_stride;
  // every thread finalises 16 of the 4096 tile entries
  for (int idx = threadIdx.x; idx < WT_TM * WT_TN * 4 * 64; idx += 256) {
    const int ln = idx & 63;
    const int reg = idx >> 6;  // (tm*WT_TN + tn)*4 + r
    const int r = reg & 3;
    const int tn = (reg >> 2) % WT_TN;
    const int tm = (reg >> 2) / WT_TN;
    const float v = ((red[0][reg][ln] + red[1][reg][ln]) + red[2][reg][ln]) + red[3][reg][ln];
    const int n = n_base + tm * 16 + 4 * (ln >> 4) + r;
    const int k = k_base + tn * 16 + (ln & 15);
    if (n < a.N && k < kb) slab[a.part_off[b] + (int64_t)n * kb + k] = v;
  }
  if (do_bias && threadIdx.x < WT_ROWS) {
    const int tm = threadIdx.x >> 4;
    const int ii = threadIdx.x & 15;
    // lanes ii, ii+16, ii+32, ii+48 of each wave hold partial sums of column
    // n_base + tm*16 + ii
    float v = 0.f;
    for (int w = 0; w < 4; ++w)
      for (int qq = 0; qq < 4; ++qq) v = v + bred[w][tm][qq * 16 + ii];
    const int n = n_base + tm * 16 + ii;
    if (n < a.N) slab[a.bias_off + n] = v;
  }
}

// Weight gradient, vector path (all operands 16-B aligned, widths % 4 == 0):
// a workgroup owns a 64(n) x 64(k) tile and one M-slice; 32-row chunks of dC
// and A_b are staged in LDS with coalesced float4 loads (double buffered) and
// each wave accumulates one 32x32 quadrant with v_mfma_f32_32x32x2_f32:
// lane l supplies dC[m0 + (l>>5)][n = 32wn + (l&31)] and
// A_b[m0 + (l>>5)][k = 32wk + (l&31)] — row-contiguous ds_read_b32, no bank
// conflicts, and no cross-wave reduction.  Partials go to the split slab.
typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int WR = 32;  // rows per staged chunk
constexpr int WDEPTH = 2;  // staged chunks in flight per workgroup (register ring; 4 measured no faster at the ZINC shapes and costs the fused kernel occupancy)

// XCD-aware work order: workgroups are dealt round-robin over the 8 XCDs, so
// (tile, split) item w = xcd_slot(linear id) puts consecutive items -- the
// n-tiles sharing an A chunk, the k-tiles sharing a dC chunk of one split --
// on ONE XCD at about the same time: their shared chunks hit that XCD's L2
__device__ __forceinline__ void weight_item(unsigned L, unsigned Y, unsigned total, int& by,
                                            int& bz) {
  const unsigned x = L & 7u, k = L >> 3, per = total >> 3, extra = total & 7u;
  const unsigned w = x * per + (x < extra ? x : extra) + k;
  by = (int)(w % Y);
  bz = (int)(w / Y);
}

__device__ __forceinline__ void bwd_weight32_body(const BwdWeightArgs& a, int by, int bz,
                                                  float (*gl)[WR][64], float (*al)[WR][64]) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wn = wave >> 1, wk = wave & 1;
  int b = 0;
  while (b + 1 < a.nb && by >= a.tile_start[b + 1]) ++b;
  const int t = by - a.tile_start[b];
  const int n_base = (t % a.tiles_n) * 64;
  const int k_base = (t / a.tiles_n) * 64;
  const int kb = a.kb[b];
  const float* __restrict__ A = a.A[b];
  const int64_t lda = a.lda[b];
  const bool do_bias = a.bias_off >= 0 && b == 0 && k_base == 0;
  const int64_t m_lo = (int64_t)bz * a.rows_per_split;
  int64_t m_hi = m_lo + a.rows_per_split;
  if (m_hi > a.M) m_hi = a.M;

  // staging: each tile is 32 rows x 16 float4; thread -> (row = tid/16 + 16u, c4 = tid%16)
  const int sr = threadIdx.x >> 4, sc = (threadIdx.x & 15) * 4;
  auto load = [&](int64_t m0, float4 (&g)[2], float4 (&x)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t m = m0 + sr + 16 * u;
      const bool mv = m < m_hi;
      const int n = n_base + sc, k = k_base + sc;
      g[u] = (mv && n < a.N) ? *reinterpret_cast<const float4*>(a.G + m * a.ldg + n)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
      x[u] = (mv && k < kb) ? *reinterpret_cast<const float4*>(A + m * lda + k)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store = [&](int buf, const float4 (&g)[2], const float4 (&x)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      *reinterpret_cast<float4*>(&gl[buf][sr + 16 * u][sc]) = g[u];
      *reinterpret_cast<float4*>(&al[buf][sr + 16 * u][sc]) = x[u];
    }
  };

  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float bsum = 0.f;
  const int rl = lane >> 5, cl = lane & 31;
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < WR / 2; ++kk) {
      const float av = gl[buf][2 * kk + rl][32 * wn + cl];
      const float bv = al[buf][2 * kk + rl][32 * wk + cl];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
      bsum = bsum + av;
    }
  };
  // WDEPTH chunks in flight in a register ring while one is consumed from
  // LDS: a slice of a few chunks costs about one memory round trip, not one
  // per chunk.  Chunk c goes register slot c % WDEPTH -> LDS buffer c & 1;
  // the one barrier per chunk also orders the buffer reuse (chunk c+2 is
  // stored after every wave passed chunk c+1's barrier, i.e. finished c).
  float4 gr[WDEPTH][2], xr[WDEPTH][2];
  const int64_t nchunk = m_hi > m_lo ? (m_hi - m_lo + WR - 1) / WR : 0;
  // Two-level fp32 accumulation: the MFMA accumulator chains at most
  // kFlushChunks chunks (256 rows), then is added into `outer` and restarted.
  // A split of 4096 rows (configs 3 / 5) otherwise sums 2048 MFMA steps in
  // one chain -- twice the rounding error of the fp32 CPU GEMM, which blocks
  // its reduction (the config-5 gradient gate).  Splits of at
  // most kFlushChunks chunks (config 2) never flush: the same bits as before.
  constexpr int kFlushChunks = 8;
  floatx16 outer;
#pragma unroll
  for (int r = 0; r < 16; ++r) outer[r] = 0.f;
  float bouter = 0.f;
  bool flushed = false;
#pragma unroll
  for (int j = 0; j < WDEPTH; ++j)
    if (j < nchunk) load(m_lo + j * WR, gr[j], xr[j]);
  for (int64_t c0 = 0; c0 < nchunk; c0 += WDEPTH) {
#pragma unroll
    for (int j = 0; j < WDEPTH; ++j) {
      const int64_t c = c0 + j;
      if (c >= nchunk) break;
      const int buf = (int)(c & 1);
      store(buf, gr[j], xr[j]);
      __syncthreads();
      if (c + WDEPTH < nchunk) load(m_lo + (c + WDEPTH) * WR, gr[j], xr[j]);
      compute(buf);
      if ((c + 1) % kFlushChunks == 0 && c + 1 < nchunk) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          outer[r] = outer[r] + acc[r];
          acc[r] = 0.f;
        }
        bouter = bouter + bsum;
        bsum = 0.f;
        flushed = true;
      }
    }
  }
  if (flushed) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = outer[r] + acc[r];
    bsum = bouter + bsum;
  }

  float* slab = a.part + (int64_t)bz * a.part_stride + a.part_off[b];
  const int k = k_base + 32 * wk + cl;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = n_base + 32 * wn + (r & 3) + 8 * (r >> 2) + 4 * rl;
    if (n < a.N && k < kb) slab[(int64_t)n * kb + k] = acc[r];
  }
  if (do_bias && wk == 0) {
    // lanes l and l+32 hold partial column sums of n = n_base + 32wn + (l&31)
    const float tot = bsum + __shfl_xor(bsum, 32, 64);
    const int n = n_base + 32 * wn + cl;
    if (rl == 0 && n < a.N)
      a.part[(int64_t)bz * a.part_stride + a.bias_off + n] = tot;
  }
}

__global__ __launch_bounds__(256) void k_proj_bwd_weight32(BwdWeightArgs a) {
  __shared__ float gl[2][WR][64];
  __shared__ float al[2][WR][64];
  int by = (int)blockIdx.y, bz = (int)blockIdx.z;
  if (a.xcd_map)
    weight_item(blockIdx.y + blockIdx.z * gridDim.y, gridDim.y, gridDim.y * gridDim.z, by, bz);
  bwd_weight32_body(a, by, bz, gl, al);
}

}  // namespace
#include "proj_big.h"
namespace {

struct ReduceArgs {
  int nb;
  int N;
  int splits;
  const float* part;
  int64_t part_stride;
  int64_t part_off[MAXB];
  int kb[MAXB];
  float* dW[MAXB];
  int64_t lddw[MAXB];
  int64_t elem_start[MAXB + 1];
  int64_t bias_off;
  float* dbias;
  int accumulate;
};

// 64 consecutive output elements per workgroup; the 4 waves sum interleaved
// subsets of the splits (coalesced 256-B reads per split), then combine in
// fixed order through LDS -> deterministic and fully parallel.
__device__ __forceinline__ void reduce_splits_body(const ReduceArgs& a, Blk blk) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t e = (int64_t)blk.x * 64 + lane;
  const int64_t total = a.elem_start[a.nb] + (a.bias_off >= 0 ? a.N : 0);
  int64_t src = -1;
  float* dst = nullptr;
  if (e < total) {
    if (e >= a.elem_start[a.nb]) {
      const int64_t n = e - a.elem_start[a.nb];
      src = a.bias_off + n;
      dst = a.dbias + n;
    } else {
      int b = 0;
      while (b + 1 < a.nb && e >= a.elem_start[b + 1]) ++b;
      const int64_t loc = e - a.elem_start[b];
      const int64_t n = loc / a.kb[b];
      const int64_t k = loc % a.kb[b];
      src = a.part_off[b] + loc;
      dst = a.dW[b] + n * a.lddw[b] + k;
    }
  }
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (src >= 0) {
    // splits grp, grp+4, ... in batches of 16 independent loads (a 120-split
    // plan is two round trips per wave)
    for (int sp0 = grp; sp0 < a.splits; sp0 += 64) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int sp = sp0 + 4 * u;
        v[u] = sp < a.splits ? a.part[(int64_t)sp * a.part_stride + src] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) s[u & 3] = s[u & 3] + v[u];
    }
  }
  red[grp][lane] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (grp == 0 && dst) {
    const float v = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    *dst = a.accumulate ? *dst + v : v;
  }
}

__global__ __launch_bounds__(256) void k_reduce_splits(ReduceArgs a) {
  reduce_splits_body(a, blk_hw());
}

// ---------------------------------------------------------------------------
// Linear backward with the weight-gradient partials and the data gradient in
// ONE launch: workgroups [0, n_w) are the weight gradient's (tile, split)
// items (bwd_weight32_body), workgroups [n_w, ...) the data gradient's tiles
// (bwd_data_lds_body); k_reduce_splits follows.  The same results, bit for
// bit, as k_proj_bwd_weight32 -> k_reduce_splits -> k_proj_bwd_data_lds with
// one dependent launch fewer.  (Reducing the splits in-kernel by the last
// arriving split of a tile was measured 37 % slower at the ZINC step: one
// workgroup then reads the tile's ~100 split partials alone.)
// ---------------------------------------------------------------------------
struct BwdFusedArgs {
  BwdWeightArgs w;
  BwdDataArgs d;
  int n_w;     // weight workgroups: tiles_total * splits
  int n_wpad;  // n_w rounded up to a multiple of 8 (the data items start on XCD 0)
  int d_gx;    // data-gradient grid x
  int n_d;     // data workgroups: d_gx * column tiles
  int d_xcd;   // XCD-aware data order: the column tiles of one row block on one XCD
  int n_red;   // trailing workgroups: a deferred split reduction of an EARLIER launch
  ReduceArgs red;
};

template <int TND, bool ROWS>
__device__ __forceinline__ void proj_bwd_fused_body(const BwdFusedArgs& a, Blk blk, float* lds) {
  const int L = (int)blk.x;
  if (L >= a.n_wpad + a.n_d) {
    const int l = L - a.n_wpad - a.n_d;
    if (l < a.n_red) reduce_splits_body(a.red, Blk{(unsigned)l, 0u, (unsigned)a.n_red, 1u});
    return;
  }
  if (ROWS && L >= a.n_wpad) {  // one workgroup per row block, every column tile
    bwd_data_rows_body<TND>(a.d, L - a.n_wpad, lds);
    return;
  }
  if (L >= a.n_wpad) {
    const int l = L - a.n_wpad;
    int bx, by;
    if (a.d_xcd) {
      // w = xcd_slot(l): consecutive w on one XCD; w -> (column tile fastest,
      // row block): a row block's dC rows are fetched into one XCD's L2 once
      // for all its column tiles
      const int tiles = a.n_d / a.d_gx;
      int wy, wz;
      weight_item((unsigned)l, 1u, (unsigned)a.n_d, wy, wz);
      by = wz % tiles;
      bx = wz / tiles;
      (void)wy;
    } else {
      bx = l % a.d_gx;
      by = l / a.d_gx;
    }
    bwd_data_lds_body<TND>(a.d, bx, by, reinterpret_cast<float (*)[TND * 16][KCP]>(lds));
    return;
  }
  if (L >= a.n_w) return;  // alignment padding
  const int Y = a.w.tile_start[a.w.nb];
  int by = L % Y, bz = L / Y;
  if (a.w.xcd_map) weight_item((unsigned)L, (unsigned)Y, (unsigned)a.n_w, by, bz);
  bwd_weight32_body(a.w, by, bz, reinterpret_cast<float (*)[WR][64]>(lds),
                    reinterpret_cast<float (*)[WR][64]>(lds + 2 * WR * 64));
}

template <int TND, bool ROWS>
__global__ __launch_bounds__(256) void k_proj_bwd_fused(BwdFusedArgs a) {
  // ROWS: two W buffers + the epilogue scratch (bwd_data_rows_body)
  constexpr int kW = 2 * WR * 64 * 2;
  constexpr int kD = ROWS ? 2 * TND * 16 * KCP + 4 * 16 * (TND * 16 + 4) : 2 * TND * 16 * KCP;
  __shared__ __attribute__((aligned(16))) float lds[kW > kD ? kW : kD];
  proj_bwd_fused_body<TND, ROWS>(a, blk_hw(), lds);
}

// A/B hook (hlhgat_set_proj_bwd_rows): row-block data-gradient workgroups
bool& proj_bwd_rows_flag() {
  static bool v = true;
  return v;
}

// --- planning ------------------------------------------------------------------
struct WeightPlan {
  int big;      // 0: the 64 x 64 items (bwd_weight32_body); else a BigCfg id
  int tile_n;   // tile rows (n) and columns (k) of one item
  int tile_k;
  int tiles_n;
  int tiles_total;
  int splits;
  int64_t rows_per_split;
  int64_t part_stride;
  int64_t part_off[MAXB];
  int64_t bias_off;
  int tile_start[MAXB + 1];
};

// --- the large-tile family (proj_big.h): when and which tile ------------------
// HLHGAT_GEMM_BIG: 0 (default) = never, -1 = by shape (the rules below),
// 1 = every vector-aligned shape (A/B and tests); hlhgat_set_gemm_big
// overrides it at run time.
std::atomic<int> g_big_mode{-2};  // -2: not read yet
std::atomic<int64_t> g_big_min_m{-1};
int big_mode() {
  int v = g_big_mode.load(std::memory_order_relaxed);
  if (v == -2) {
    // default 0: in the measured training steps (configs 3 and 5, where the
    // node and edge chains share the GPU) the large tiles lost 1-2 ms per
    // step although they win shape by shape in isolation
    const char* e = std::getenv("HLHGAT_GEMM_BIG");
    v = e ? std::atoi(e) : 0;
    int expect = -2;
    g_big_mode.compare_exchange_strong(expect, v);
    v = g_big_mode.load(std::memory_order_relaxed);
  }
  return v;
}
int64_t big_min_m() {
  int64_t v = g_big_min_m.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("HLHGAT_GEMM_BIG_MIN_M");
    // default above the fused projection + BatchNorm range (<= 512 row blocks)
    v = e ? (int64_t)std::atoll(e) : (int64_t)32769;
    int64_t expect = -1;
    g_big_min_m.compare_exchange_strong(expect, v);
    v = g_big_min_m.load(std::memory_order_relaxed);
  }
  return v;
}
// HLHGAT_LOG_PROJ=1: one stderr line per projection call (shape census)
bool log_proj() {
  static const bool v = [] {
    const char* e = std::getenv("HLHGAT_LOG_PROJ");
    return e && e[0] == '1';
  }();
  return v;
}
void log_call(const char* what, int64_t M, int64_t N, int nb, const int64_t* kb,
              const int64_t* ld) {
  if (!log_proj()) return;
  char buf[512];
  int o = snprintf(buf, sizeof(buf), "[hlhgat proj] %s M=%lld N=%lld kb=", what, (long long)M,
                   (long long)N);
  for (int b = 0; b < nb && o < 400; ++b)
    o += snprintf(buf + o, sizeof(buf) - o, "%s%lld", b ? "," : "", (long long)kb[b]);
  if (ld && o < 400) {
    o += snprintf(buf + o, sizeof(buf) - o, " ld=");
    for (int b = 0; b < nb && o < 480; ++b)
      o += snprintf(buf + o, sizeof(buf) - o, "%s%lld", b ? "," : "", (long long)ld[b]);
  }
  fprintf(stderr, "%s\n", buf);
}

// Per operation, by shape (mode -1), from the census-weighted A/B of the
// config-5 step (tools/kbench_census.py, profiles/r05_kcensus_*.log): the
// large tiles win where a launch fills the chip several times over and the
// reduction is long enough to amortise the 128 x 128 staging prologue.
// HLHGAT_GEMM_BIG_OPS: which operations may take the large tiles in mode -1
// ("f" forward, "d" data gradient, "w" weight gradient; default all)
unsigned big_ops() {
  static const unsigned v = [] {
    const char* e = std::getenv("HLHGAT_GEMM_BIG_OPS");
    if (!e) return 7u;
    unsigned m = 0;
    for (const char* c = e; *c; ++c) m |= *c == 'f' ? 1u : *c == 'd' ? 2u : *c == 'w' ? 4u : 0u;
    return m;
  }();
  return v;
}

bool big_mode_decides(int64_t M, bool& out) {
  const int m = big_mode();
  if (m == 0) { out = false; return true; }
  if (m == 1) { out = M > 0; return true; }
  if (M < big_min_m()) { out = false; return true; }
  return false;
}
// forward C = A W^T: N output columns, ktot reduction
bool big_fwd_ok(int64_t M, int64_t N, int64_t ktot) {
  bool v;
  if (big_mode_decides(M, v)) return v;
  if (!(big_ops() & 1u)) return false;
  return M >= 2 * big_min_m() && N >= 128 && ktot >= 224;
}
// data gradient dA = dC W: reduction N, ktot output columns
bool big_data_ok(int64_t M, int64_t N, int64_t ktot) {
  bool v;
  if (big_mode_decides(M, v)) return v;
  if (!(big_ops() & 2u)) return false;
  if (N <= 32) return true;
  return M >= 2 * big_min_m() && (N >= 256 || (N >= 128 && ktot >= 352));
}
// weight gradient dW = dC^T A: N rows, ktot columns, reduction M
bool big_weight_ok(int64_t M, int64_t N, int64_t ktot) {
  bool v;
  if (big_mode_decides(M, v)) return v;
  if (!(big_ops() & 4u)) return false;
  return M >= 2 * big_min_m() || (N >= 128 && ktot >= 288);
}

// weight-gradient workgroups the 64 x 64 plan aims for (HLHGAT_WSPLIT_TARGET)
int64_t wsplit_target() {
  static const int64_t v = [] {
    const char* e = std::getenv("HLHGAT_WSPLIT_TARGET");
    const int64_t t = e ? (int64_t)std::atoll(e) : 240;
    return t < 1 ? (int64_t)1 : t;
  }();
  return v;
}

// rounds of two workgroups per CU the large-tile weight gradient is planned
// for (HLHGAT_BIG_W_ROUNDS; shorter items balance better beside the other
// chain's kernels, at the cost of a larger split slab)
int64_t big_w_rounds() {
  static const int64_t v = [] {
    const char* e = std::getenv("HLHGAT_BIG_W_ROUNDS");
    const int64_t r = e ? (int64_t)std::atoll(e) : 4;
    return r < 1 ? (int64_t)1 : r;
  }();
  return v;
}

// compute units of the current device (cached; 256 on MI355X)
int device_cus() {
  static std::atomic<int> cache[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 256;
  int v = cache[dev].load(std::memory_order_relaxed);
  if (v <= 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    cache[dev].store(cus, std::memory_order_relaxed);
    v = cus;
  }
  return v;
}

// tile configurations <WM, WN, TBM, TBN> (4 waves; tile (WM TBM 32) x (WN TBN 32))
enum BigCfg { kBig128x128 = 1, kBig256x64, kBig256x32, kBig128x64, kBig64x128, kBig64x64,
              kBig32x128 };
inline void big_dims(int cfg, int& rows, int& cols) {
  switch (cfg) {
    case kBig128x128: rows = 128; cols = 128; return;
    case kBig256x64: rows = 256; cols = 64; return;
    case kBig256x32: rows = 256; cols = 32; return;
    case kBig128x64: rows = 128; cols = 64; return;
    case kBig64x128: rows = 64; cols = 128; return;
    case kBig64x64: rows = 64; cols = 64; return;
    default: rows = 32; cols = 128; return;
  }
}
// forward: rows = M, cols = N
int big_fwd_cfg(int64_t N) { return N > 64 ? kBig128x128 : (N > 32 ? kBig256x64 : kBig256x32); }
// data gradient: rows = M, cols = the narrowest block's columns
int big_data_cfg(int64_t min_kb) {
  return min_kb >= 128 ? kBig128x128 : (min_kb > 32 ? kBig256x64 : kBig256x32);
}
// weight gradient: rows = N, cols = the narrowest block's columns
int big_weight_cfg(int64_t N, int64_t min_kb) {
  if (N > 64) return min_kb >= 128 ? kBig128x128 : kBig128x64;
  if (N > 32) return min_kb >= 128 ? kBig64x128 : kBig64x64;
  return kBig32x128;
}

WeightPlan plan_weight(int nb, const int64_t* kb, int64_t M, int64_t N,
                       bool with_bias, bool use_big = false) {
  WeightPlan p{};
  int64_t min_kb = kb[0];
  for (int b = 1; b < nb; ++b) min_kb = std::min<int64_t>(min_kb, kb[b]);
  p.big = use_big ? big_weight_cfg(N, min_kb) : 0;
  if (p.big) big_dims(p.big, p.tile_n, p.tile_k);
  else {
    p.tile_n = WT_ROWS;
    p.tile_k = WT_COLS;
  }
  p.tiles_n = (int)ceil_div(N, p.tile_n);
  int64_t off = 0;
  p.tile_start[0] = 0;
  for (int b = 0; b < nb; ++b) {
    p.part_off[b] = off;
    off += N * kb[b];
    p.tile_start[b + 1] = p.tile_start[b] + p.tiles_n * (int)ceil_div(kb[b], p.tile_k);
  }
  p.bias_off = with_bias ? off : -1;
  if (with_bias) off += N;
  p.part_stride = off;
  p.tiles_total = p.tile_start[nb];
  if (p.big) {
    // at most one round of two workgroups per CU over (tile, split) items (a
    // 513th item costs a whole second round: measured 1.2-1.3x at the
    // config-5 shapes), every split >= 512 rows (16 stages: the staging
    // prologue stays small against the MFMAs)
    const int64_t tiles = p.tiles_total > 0 ? p.tiles_total : 1;
    int64_t splits = std::max<int64_t>(1, (big_w_rounds() * 2 * (int64_t)device_cus()) / tiles);
    splits = std::min<int64_t>(splits, std::max<int64_t>(1, M / 512));
    if (splits < 1) splits = 1;
    int64_t rps = ceil_div(M > 0 ? M : 1, splits);
    rps = ceil_div(rps, BKC) * BKC;
    p.rows_per_split = rps;
    p.splits = (int)ceil_div(M > 0 ? M : 1, rps);
    return p;
  }
  // aim for ~240 workgroups, each slice >= 128 rows: balances MFMA
  // parallelism against the split-slab traffic the reduce re-reads, beside
  // the fused launch's data-gradient items (384 before round 5; same-box A/B
  // of the config-2 step, profiles/r05/ab_cfg2_wsplit_target.txt: 180 2.72-2.73,
  // 240 2.686-2.688, 360 2.694-2.709, 540 2.73-2.74 ms).
  const int64_t tiles = p.tiles_total > 0 ? p.tiles_total : 1;
  int64_t splits = ceil_div(wsplit_target(), tiles);
  // large M (config 3 / 5 heads, 1e5+ rows): up to ~1536 workgroups as long
  // as every slice keeps >= 4096 rows (the slab stays small against A);
  // measured 13-22 % faster on the TSP / CIFAR NEInt and conv shapes
  // (tools/kbench.py --big, profiles/r01_h_wsplit.log), ZINC shapes unchanged
  const int64_t big = std::min<int64_t>(ceil_div(1536, tiles), M / 4096);
  if (big > splits) splits = big;
  int64_t max_splits = ceil_div(M, 128);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int64_t rps = ceil_div(M, splits);
  rps = ceil_div(rps, 64) * 64;
  if (rps < 64) rps = 64;
  p.rows_per_split = rps;
  p.splits = (int)ceil_div(M > 0 ? M : 1, rps);
  return p;
}

void launch_fwd_big(int cfg, unsigned nblk, hipStream_t s, const ProfScope* prof,
                    const FwdArgs& a) {
  if (cfg == kBig128x128) launch(k_proj_fwd_big<2, 2, 2, 2>, dim3(nblk), dim3(256), 0, s, prof, a);
  else if (cfg == kBig256x64) launch(k_proj_fwd_big<4, 1, 2, 2>, dim3(nblk), dim3(256), 0, s, prof, a);
  else launch(k_proj_fwd_big<4, 1, 2, 1>, dim3(nblk), dim3(256), 0, s, prof, a);
}

void launch_data_big(int cfg, unsigned nblk, hipStream_t s, const ProfScope* prof,
                     const BwdDataArgs& a) {
  if (cfg == kBig128x128)
    launch(k_proj_bwd_data_big<2, 2, 2, 2>, dim3(nblk), dim3(256), 0, s, prof, a);
  else if (cfg == kBig256x64)
    launch(k_proj_bwd_data_big<4, 1, 2, 2>, dim3(nblk), dim3(256), 0, s, prof, a);
  else
    launch(k_proj_bwd_data_big<4, 1, 2, 1>, dim3(nblk), dim3(256), 0, s, prof, a);
}

void launch_weight_big(int cfg, unsigned nblk, hipStream_t s, const ProfScope* prof,
                       const BwdWeightArgs& a) {
  switch (cfg) {
    case kBig128x128:
      launch(k_proj_bwd_weight_big<2, 2, 2, 2>, dim3(nblk), dim3(256), 0, s, prof, a);
      break;
    case kBig128x64:
      launch(k_proj_bwd_weight_big<4, 1, 1, 2>, dim3(nblk), dim3(256), 0, s, prof, a);
      break;
    case kBig64x128:
      launch(k_proj_bwd_weight_big<2, 2, 1, 2>, dim3(nblk), dim3(256), 0, s, prof, a);
      break;
    case kBig64x64:
      launch(k_proj_bwd_weight_big<2, 2, 1, 1>, dim3(nblk), dim3(256), 0, s, prof, a);
      break;
    default:
      launch(k_proj_bwd_weight_big<1, 4, 1, 1>, dim3(nblk), dim3(256), 0, s, prof, a);
  }
}

// The large-tile data gradient of all blocks: one launch (a.tile_start and the
// grid in units of the configuration's column tile).  Returns the grid size.
int64_t data_big_setup(BwdDataArgs& a, int& cfg) {
  int64_t min_kb = a.kb[0];
  for (int b = 1; b < a.nb; ++b) min_kb = std::min<int64_t>(min_kb, a.kb[b]);
  cfg = big_data_cfg(min_kb);
  int rows, cols;
  big_dims(cfg, rows, cols);
  a.tile_start[0] = 0;
  for (int b = 0; b < a.nb; ++b)
    a.tile_start[b + 1] = a.tile_start[b] + (int)ceil_div(a.kb[b], cols);
  return ceil_div(a.M, rows) * a.tile_start[a.nb];
}

// XCD-aware work orders of the weight gradient's items and of the fused
// backward's data-gradient workgroups (results are identical in any order)
constexpr int weight_xcd_map() { return 1; }
constexpr int data_xcd_map() { return 1; }

// Data-gradient tiles of 64 columns (TN 4) where the size rule picks more
// than one 16-column tile: each staged dC row block serves 64 output columns
// (+1.3 % at the ZINC step against 32-column tiles, same-box A/B)
constexpr int bwd_tnd() { return 4; }

bool vec_ok(const float* p, int64_t ld, int64_t kb) {
  return aligned16(p) && (ld % 4) == 0 && (kb % 4) == 0;
}

// 16-column tiles per wave of the forward: enough waves to cover the 1024
// SIMDs several times over (measured at the HL-HGAT shapes, tools/kbench.py):
// small M -> 1, K <= 256 -> 2 (re-reading A from L2 is cheap), long K -> 4
int fwd_tn(int64_t M, int64_t N, int64_t ktot) {
  // (64-column tiles from K = 0 measured equal at the ZINC step, round 2)
  int tn = ceil_div(M, 16) * ceil_div(N, 16) < 4096 ? 1 : (ktot >= 256 ? 4 : 2);
  if (N <= 16) tn = 1;
  else if (N <= 32 && tn > 2) tn = 2;
  return tn;
}

}  // namespace

using namespace hlhgat;

// HLHGAT_FWD_XCD=0: k_proj_fwd_lds in blockIdx.x-fastest order (A/B)
int fwd_xcd_map() {
  static const int v = [] {
    const char* e = std::getenv("HLHGAT_FWD_XCD");
    return (e && std::atoi(e) == 0) ? 0 : 1;
  }();
  return v;
}

extern "C" int hlhgat_proj_fwd(int nblocks, const float* const* A,
                               const int64_t* lda, const float* const* W,
                               const int64_t* ldw, const int64_t* kb, int64_t M,
                               int64_t N, const float* bias, float* C,
                               int64_t ldc, int accumulate, void* stream) {
  HLH_CHECK_ARG(nblocks >= 1 && nblocks <= MAXB, "proj_fwd: nblocks=%d", nblocks);
  HLH_CHECK_ARG(M >= 0 && N > 0 && N < (1 << 30) && ldc >= N,
                "proj_fwd: bad M/N/ldc");
  HLH_CHECK_ARG(C, "proj_fwd: C is NULL");
  FwdArgs a{};
  a.nb = nblocks;
  a.M = M;
  a.N = (int)N;
  a.bias = bias;
  a.C = C;
  a.ldc = ldc;
  a.accumulate = accumulate;
  bool vec = true;
  double flops = 0;
  for (int b = 0; b < nblocks; ++b) {
    HLH_CHECK_ARG(A[b] && W[b] && kb[b] > 0 && lda[b] >= kb[b] && ldw[b] >= kb[b],
                  "proj_fwd: bad block %d", b);
    a.A[b] = A[b];
    a.W[b] = W[b];
    a.lda[b] = lda[b];
    a.ldw[b] = ldw[b];
    a.kb[b] = (int)kb[b];
    vec = vec && vec_ok(A[b], lda[b], kb[b]) && vec_ok(W[b], ldw[b], kb[b]);
    flops += 2.0 * (double)M * (double)N * (double)kb[b];
  }
  if (M == 0) return HLHGAT_OK;
  log_call("fwd", M, N, nblocks, kb, lda);
  hipStream_t s = as_stream(stream);
  // 16-column tiles per wave: enough waves to cover the 1024 SIMDs several
  // times over (measured at the HL-HGAT shapes, tools/kbench.py): small M ->
  // 1, K <= 256 -> 2 (re-reading A from L2 is cheap), long K -> 4
  int64_t ktot = 0;
  for (int b = 0; b < nblocks; ++b) ktot += kb[b];
  const int tn = fwd_tn(M, N, ktot);
  const int tm = M >= 262144 ? 2 : 1;
  dim3 grid((unsigned)ceil_div(M, 4 * tm * 16), (unsigned)ceil_div(N, tn * 16));
  double bytes = 4.0 * (double)M * N;
  for (int b = 0; b < nblocks; ++b) bytes += 4.0 * (double)M * kb[b] + 4.0 * N * kb[b];
  ProfScope prof(HLHGAT_PROF_PROJ, s, bytes, flops);
  if (vec && big_fwd_ok(M, N, ktot)) {
    const int cfg = big_fwd_cfg(N);
    int rows, cols;
    big_dims(cfg, rows, cols);
    const int64_t nblk = ceil_div(M, rows) * ceil_div(N, cols);
    HLH_CHECK_ARG(nblk < (int64_t)INT32_MAX, "proj_fwd: grid too large");
    launch_fwd_big(cfg, (unsigned)nblk, s, &prof, a);
    HLH_CHECK_LAUNCH();
    return HLHGAT_OK;
  }
  if (vec) {
    dim3 g((unsigned)ceil_div(M, 64), (unsigned)ceil_div(N, tn * 16));
    // large slabs only (configs 3 / 5: 1.4e5-2e5 rows); the config-2 shapes
    // (2.3e4 rows, their A in L2 anyway) keep the blockIdx order
    a.xcd_map = M >= 65536 ? fwd_xcd_map() : 0;
    if (tn == 1)
      launch(k_proj_fwd_lds<1>, g, 256, 0, s, &prof, a);
    else if (tn == 2)
      launch(k_proj_fwd_lds<2>, g, 256, 0, s, &prof, a);
    else
      launch(k_proj_fwd_lds<4>, g, 256, 0, s, &prof, a);
  } else if (tm == 1 && tn == 1) {
    launch(k_proj_fwd<1, 1, false>, grid, 256, 0, s, &prof, a);
  } else if (tm == 1 && tn == 2) {
    launch(k_proj_fwd<1, 2, false>, grid, 256, 0, s, &prof, a);
  } else if (tm == 1) {
    launch(k_proj_fwd<1, 4, false>, grid, 256, 0, s, &prof, a);
  } else if (tn == 1) {
    launch(k_proj_fwd<2, 1, false>, grid, 256, 0, s, &prof, a);
  } else if (tn == 2) {
    launch(k_proj_fwd<2, 2, false>, grid, 256, 0, s, &prof, a);
  } else {
    launch(k_proj_fwd<2, 4, false>, grid, 256, 0, s, &prof, a);
  }
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_proj_bwd_data(int nblocks, const float* dC, int64_t lddc,
                                    const float* const* W, const int64_t* ldw,
                                    const int64_t* kb, int64_t M, int64_t N,
                                    float* const* dA, const int64_t* ldda,
                                    int accumulate, void* stream) {
  HLH_CHECK_ARG(nblocks >= 1 && nblocks <= MAXB, "proj_bwd_data: nblocks=%d",
                nblocks);
  HLH_CHECK_ARG(M >= 0 && N > 0 && lddc >= N && dC, "proj_bwd_data: bad dC");
  BwdDataArgs a{};
  a.nb = nblocks;
  a.M = M;
  a.N = (int)N;
  a.G = dC;
  a.ldg = lddc;
  a.accumulate = accumulate;
  const int TN = 4;
  int64_t ktot = 0;
  for (int b = 0; b < nblocks; ++b) ktot += kb[b];
  int tnd = ceil_div(M, 16) * ceil_div(ktot, 16) < 4096 ? 1 : 2;  // see proj_fwd
  if (tnd == 2 && bwd_tnd() == 4) tnd = TN;
  a.tile_start[0] = 0;
  for (int b = 0; b < nblocks; ++b) {
    HLH_CHECK_ARG(W[b] && dA[b] && kb[b] > 0 && ldw[b] >= kb[b] && ldda[b] >= kb[b],
                  "proj_bwd_data: bad block %d", b);
    a.W[b] = W[b];
    a.O[b] = dA[b];
    a.ldw[b] = ldw[b];
    a.ldo[b] = ldda[b];
    a.kb[b] = (int)kb[b];
    a.tile_start[b + 1] = a.tile_start[b] + (int)ceil_div(kb[b], tnd * 16);
  }
  if (M == 0) return HLHGAT_OK;
  bool vec = aligned16(dC) && (lddc % 4) == 0 && (N % 4) == 0;
  for (int b = 0; b < nblocks; ++b)
    vec = vec && aligned16(W[b]) && (ldw[b] % 4) == 0 && (kb[b] % 4) == 0;
  hipStream_t s = as_stream(stream);
  if (vec && big_data_ok(M, N, ktot)) {
    int cfg;
    const int64_t nblk = data_big_setup(a, cfg);
    HLH_CHECK_ARG(nblk < (int64_t)INT32_MAX, "proj_bwd_data: grid too large");
    launch_data_big(cfg, (unsigned)nblk, s, nullptr, a);
    HLH_CHECK_LAUNCH();
    return HLHGAT_OK;
  }
  dim3 grid((unsigned)ceil_div(M, 4 * 16), (unsigned)a.tile_start[nblocks]);
  if (vec)
  {
    if (tnd == 1)
      launch(k_proj_bwd_data_lds<1>, dim3(grid), dim3(256), 0, s, nullptr, a);
    else if (tnd == 2)
      launch(k_proj_bwd_data_lds<2>, dim3(grid), dim3(256), 0, s, nullptr, a);
    else
      launch(k_proj_bwd_data_lds<TN>, dim3(grid), dim3(256), 0, s, nullptr, a);
  }
  else
  {
    if (tnd == 1)
      launch(k_proj_bwd_data<1, 1, false>, dim3(grid), dim3(256), 0, s, nullptr, a);
    else if (tnd == 2)
      launch(k_proj_bwd_data<1, 2, false>, dim3(grid), dim3(256), 0, s, nullptr, a);
    else
      launch(k_proj_bwd_data<1, TN, false>, dim3(grid), dim3(256), 0, s, nullptr, a);
  }
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int64_t hlhgat_proj_bwd_weight_workspace_floats(int nblocks,
                                                           const int64_t* kb,
                                                           int64_t M, int64_t N,
                                                           int with_bias) {
  if (nblocks < 1 || nblocks > MAXB || N <= 0 || M < 0) return 0;
  // the larger of the two plans: the path is chosen by shape AND alignment
  const WeightPlan p = plan_weight(nblocks, kb, M, N, with_bias != 0, false);
  const WeightPlan q = plan_weight(nblocks, kb, M, N, with_bias != 0, true);
  return std::max((int64_t)p.splits * p.part_stride, (int64_t)q.splits * q.part_stride);
}

extern "C" int hlhgat_proj_bwd_weight(int nblocks, const float* dC, int64_t lddc,
                                      const float* const* A, const int64_t* lda,
                                      const int64_t* kb, int64_t M, int64_t N,
                                      float* const* dW, const int64_t* lddw,
                                      float* dbias, int accumulate,
                                      float* workspace, int64_t workspace_floats,
                                      void* stream) {
  HLH_CHECK_ARG(nblocks >= 1 && nblocks <= MAXB, "proj_bwd_weight: nblocks=%d",
                nblocks);
  HLH_CHECK_ARG(M >= 0 && N > 0 && lddc >= N && dC, "proj_bwd_weight: bad dC");
  bool vec = aligned16(dC) && (lddc % 4) == 0 && (N % 4) == 0;
  int64_t ktot_w = 0;
  for (int b = 0; b < nblocks; ++b) {
    vec = vec && A[b] && aligned16(A[b]) && (lda[b] % 4) == 0 && (kb[b] % 4) == 0;
    ktot_w += kb[b];
  }
  WeightPlan p = plan_weight(nblocks, kb, M, N, dbias != nullptr,
                             vec && big_weight_ok(M, N, ktot_w));
  HLH_CHECK_ARG(workspace && workspace_floats >= (int64_t)p.splits * p.part_stride,
                "proj_bwd_weight: workspace too small");
  BwdWeightArgs a{};
  a.nb = nblocks;
  a.M = M;
  a.N = (int)N;
  a.G = dC;
  a.ldg = lddc;
  ReduceArgs r{};
  r.nb = nblocks;
  r.N = (int)N;
  r.elem_start[0] = 0;
  for (int b = 0; b < nblocks; ++b) {
    HLH_CHECK_ARG(A[b] && dW[b] && kb[b] > 0 && lda[b] >= kb[b] && lddw[b] >= kb[b],
                  "proj_bwd_weight: bad block %d", b);
    a.A[b] = A[b];
    a.lda[b] = lda[b];
    a.kb[b] = (int)kb[b];
    a.tile_start[b] = p.tile_start[b];
    a.part_off[b] = p.part_off[b];
    r.part_off[b] = p.part_off[b];
    r.kb[b] = (int)kb[b];
    r.dW[b] = dW[b];
    r.lddw[b] = lddw[b];
    r.elem_start[b + 1] = r.elem_start[b] + N * kb[b];
  }
  a.tile_start[nblocks] = p.tile_start[nblocks];
  a.bias_off = p.bias_off;
  a.part_stride = p.part_stride;
  a.part = workspace;
  a.rows_per_split = p.rows_per_split;
  a.tiles_n = p.tiles_n;
  a.xcd_map = weight_xcd_map();
  hipStream_t s = as_stream(stream);
  if (M == 0) {
    // no rows: gradient contribution is zero
    if (!accumulate) {
      for (int b = 0; b < nblocks; ++b)
        for (int64_t n = 0; n < N; ++n)
          HLH_CHECK_HIP(hipMemsetAsync(dW[b] + n * lddw[b], 0, sizeof(float) * kb[b], s));
      if (dbias) HLH_CHECK_HIP(hipMemsetAsync(dbias, 0, sizeof(float) * N, s));
    }
    return HLHGAT_OK;
  }
  dim3 grid(1, (unsigned)p.tiles_total, (unsigned)p.splits);
  if (p.big)
    launch_weight_big(p.big, (unsigned)(p.tiles_total * p.splits), s, nullptr, a);
  else if (vec)
    launch(k_proj_bwd_weight32, dim3(grid), dim3(256), 0, s, nullptr, a);
  else
    launch(k_proj_bwd_weight, dim3(grid), dim3(256), 0, s, nullptr, a);
  HLH_CHECK_LAUNCH();
  r.splits = p.splits;
  r.part = workspace;
  r.part_stride = p.part_stride;
  r.bias_off = p.bias_off;
  r.dbias = dbias;
  r.accumulate = accumulate;
  const int64_t total = r.elem_start[nblocks] + (dbias ? N : 0);
  launch(k_reduce_splits, dim3((unsigned)ceil_div(total, 64)), dim3(256), 0, s, nullptr, r);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

namespace {
static_assert(sizeof(ReduceArgs) + sizeof(int64_t) <= sizeof(hlhgat_reduce_desc_t),
              "hlhgat_reduce_desc_t too small");

int64_t reduce_blocks(const ReduceArgs& r) {
  const int64_t total = r.elem_start[r.nb] + (r.bias_off >= 0 ? r.N : 0);
  return ceil_div(total, 64);
}

int run_reduce(const ReduceArgs& r, hipStream_t s) {
  launch(k_reduce_splits, dim3((unsigned)reduce_blocks(r)), dim3(256), 0, s, nullptr, r);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

constexpr int64_t kDescMagic = 0x686c6872656431LL;  // "hlhred1"

// The large-tile backward (proj_big.h): an earlier launch's deferred split
// reduction first (if any), the weight-gradient partials, the data gradient,
// then this launch's split reduction (or its descriptor, deferred).  Three
// launches instead of the fused one: at these shapes each runs 100s of us.
int proj_bwd_big(bool big_w, bool big_d, int64_t M, int64_t N, const float* dC, int64_t lddc,
                 int nb_w,
                 const float* const* A, const int64_t* lda, const int64_t* kb_w,
                 float* const* dW, const int64_t* lddw, float* dbias, int nb_d,
                 const float* const* W, const int64_t* ldw, const int64_t* kb_d,
                 float* const* dA, const int64_t* ldda, int accumulate_d, float* workspace,
                 int64_t workspace_floats, void* stream, const ReduceArgs* prev,
                 hlhgat_reduce_desc_t* defer_out, int* deferred) {
  hipStream_t s = as_stream(stream);
  if (prev) {
    const int rc = run_reduce(*prev, s);
    if (rc != HLHGAT_OK) return rc;
  }
  ReduceArgs r{};
  if (nb_w > 0) {
    const WeightPlan p = plan_weight(nb_w, kb_w, M, N, dbias != nullptr, big_w);
    HLH_CHECK_ARG(workspace && workspace_floats >= (int64_t)p.splits * p.part_stride,
                  "proj_bwd: workspace too small");
    BwdWeightArgs a{};
    a.nb = nb_w;
    a.M = M;
    a.N = (int)N;
    a.G = dC;
    a.ldg = lddc;
    r.nb = nb_w;
    r.N = (int)N;
    r.elem_start[0] = 0;
    double flops = 0, bytes = 4.0 * (double)M * N;
    for (int b = 0; b < nb_w; ++b) {
      HLH_CHECK_ARG(A[b] && dW[b] && kb_w[b] > 0 && lda[b] >= kb_w[b] && lddw[b] >= kb_w[b],
                    "proj_bwd: bad weight block %d", b);
      a.A[b] = A[b];
      a.lda[b] = lda[b];
      a.kb[b] = (int)kb_w[b];
      a.tile_start[b] = p.tile_start[b];
      a.part_off[b] = p.part_off[b];
      r.part_off[b] = p.part_off[b];
      r.kb[b] = (int)kb_w[b];
      r.dW[b] = dW[b];
      r.lddw[b] = lddw[b];
      r.elem_start[b + 1] = r.elem_start[b] + N * kb_w[b];
      flops += 2.0 * (double)M * N * kb_w[b];
      bytes += 4.0 * (double)M * kb_w[b];
    }
    a.tile_start[nb_w] = p.tile_start[nb_w];
    a.bias_off = p.bias_off;
    a.part_stride = p.part_stride;
    a.part = workspace;
    a.rows_per_split = p.rows_per_split;
    a.tiles_n = p.tiles_n;
    a.xcd_map = p.big ? 1 : weight_xcd_map();
    bytes += 4.0 * (double)p.splits * p.part_stride;
    const int64_t nblk = (int64_t)p.tiles_total * p.splits;
    HLH_CHECK_ARG(nblk < (int64_t)INT32_MAX, "proj_bwd: grid too large");
    ProfScope prof(HLHGAT_PROF_PROJ_BWD, s, bytes, flops);
    if (p.big)
      launch_weight_big(p.big, (unsigned)nblk, s, &prof, a);
    else  // the 64 x 64 items (the same bits as the fused small launch's)
      launch(k_proj_bwd_weight32, dim3(1, (unsigned)p.tiles_total, (unsigned)p.splits), dim3(256),
             0, s, &prof, a);
    HLH_CHECK_LAUNCH();
    r.splits = p.splits;
    r.part = workspace;
    r.part_stride = p.part_stride;
    r.bias_off = p.bias_off;
    r.dbias = dbias;
    r.accumulate = 0;
  }
  if (nb_d > 0 && !big_d) {
    const int rc = hlhgat_proj_bwd_data(nb_d, dC, lddc, W, ldw, kb_d, M, N, dA, ldda,
                                        accumulate_d, stream);
    if (rc != HLHGAT_OK) return rc;
  } else if (nb_d > 0) {
    BwdDataArgs d{};
    d.nb = nb_d;
    d.M = M;
    d.N = (int)N;
    d.G = dC;
    d.ldg = lddc;
    d.accumulate = accumulate_d;
    double flops = 0, bytes = 4.0 * (double)M * N;
    for (int b = 0; b < nb_d; ++b) {
      HLH_CHECK_ARG(W[b] && dA[b] && kb_d[b] > 0 && ldw[b] >= kb_d[b] && ldda[b] >= kb_d[b],
                    "proj_bwd: bad data block %d", b);
      d.W[b] = W[b];
      d.O[b] = dA[b];
      d.ldw[b] = ldw[b];
      d.ldo[b] = ldda[b];
      d.kb[b] = (int)kb_d[b];
      flops += 2.0 * (double)M * N * kb_d[b];
      bytes += 4.0 * (double)M * kb_d[b] + 4.0 * N * kb_d[b];
    }
    int cfg;
    const int64_t nblk = data_big_setup(d, cfg);
    HLH_CHECK_ARG(nblk < (int64_t)INT32_MAX, "proj_bwd: grid too large");
    ProfScope prof(HLHGAT_PROF_PROJ_BWD, s, bytes, flops);
    launch_data_big(cfg, (unsigned)nblk, s, &prof, d);
    HLH_CHECK_LAUNCH();
  }
  if (nb_w == 0) return HLHGAT_OK;
  if (defer_out) {
    memset(defer_out, 0, sizeof(*defer_out));
    defer_out->words[0] = kDescMagic;
    memcpy(&defer_out->words[1], &r, sizeof(r));
    if (deferred) *deferred = 1;
    return HLHGAT_OK;
  }
  return run_reduce(r, s);
}

int proj_bwd_impl(int64_t M, int64_t N, const float* dC, int64_t lddc, int nb_w, const float* const* A, const int64_t* lda,
                  const int64_t* kb_w, float* const* dW, const int64_t* lddw, float* dbias,
                  int nb_d, const float* const* W, const int64_t* ldw, const int64_t* kb_d,
                  float* const* dA, const int64_t* ldda, int accumulate_d, float* workspace,
                  int64_t workspace_floats, void* stream,
                  const hlhgat_reduce_desc_t* merge = nullptr,
                  hlhgat_reduce_desc_t* defer_out = nullptr, int* deferred = nullptr) {
  if (deferred) *deferred = 0;
  const ReduceArgs* prev = nullptr;
  if (merge) {
    HLH_CHECK_ARG(merge->words[0] == kDescMagic, "proj_bwd: merge is not a reduce descriptor");
    prev = reinterpret_cast<const ReduceArgs*>(&merge->words[1]);
  }
  HLH_CHECK_ARG(nb_w >= 0 && nb_w <= MAXB && nb_d >= 0 && nb_d <= MAXB,
                "proj_bwd: nb_w=%d nb_d=%d", nb_w, nb_d);
  HLH_CHECK_ARG(M >= 0 && N > 0 && lddc >= N && dC, "proj_bwd: bad dC");
  const bool want_w = nb_w > 0, want_d = nb_d > 0;
  // weight-only calls (a Linear whose input needs no gradient) take the same
  // launch with no data items, so they can merge / defer split reductions too
  bool fuse = want_w && M > 0 && aligned16(dC) && (lddc % 4) == 0 && (N % 4) == 0;
  WeightPlan p{};
  if (want_w) {
    p = plan_weight(nb_w, kb_w, M, N, dbias != nullptr);
    HLH_CHECK_ARG(workspace && workspace_floats >= (int64_t)p.splits * p.part_stride,
                  "proj_bwd: workspace too small");
    for (int b = 0; b < nb_w && fuse; ++b) fuse = vec_ok(A[b], lda[b], kb_w[b]);
  }
  for (int b = 0; b < nb_d && fuse; ++b) fuse = vec_ok(W[b], ldw[b], kb_d[b]);
  if (prev && !fuse) {  // run the merged reduction on its own first
    const int rc = run_reduce(*prev, as_stream(stream));
    if (rc != HLHGAT_OK) return rc;
    prev = nullptr;
  }
  if (!fuse) {  // the separate launches (any alignment, M == 0, one side only)
    if (want_w) {
      const int rc = hlhgat_proj_bwd_weight(nb_w, dC, lddc, A, lda, kb_w, M, N, dW, lddw, dbias,
                                            0, workspace, workspace_floats, stream);
      if (rc != HLHGAT_OK) return rc;
    }
    if (want_d) return hlhgat_proj_bwd_data(nb_d, dC, lddc, W, ldw, kb_d, M, N, dA, ldda,
                                            accumulate_d, stream);
    return HLHGAT_OK;
  }
  int64_t ktot_w = 0, ktot_d = 0;
  for (int b = 0; b < nb_w; ++b) ktot_w += kb_w[b];
  for (int b = 0; b < nb_d; ++b) ktot_d += kb_d[b];
  log_call("bwd_w", M, N, nb_w, kb_w, lda);
  log_call("bwd_d", M, N, nb_d, kb_d, nullptr);
  const bool big_w = want_w && big_weight_ok(M, N, ktot_w);
  const bool big_d = want_d && big_data_ok(M, N, ktot_d);
  if (big_w || big_d)
    return proj_bwd_big(big_w, big_d, M, N, dC, lddc, nb_w, A, lda, kb_w, dW, lddw, dbias, nb_d, W, ldw, kb_d,
                        dA, ldda, accumulate_d, workspace, workspace_floats, stream, prev,
                        defer_out, deferred);
  BwdFusedArgs f{};
  BwdWeightArgs& a = f.w;
  ReduceArgs r{};
  r.nb = nb_w;
  r.N = (int)N;
  r.elem_start[0] = 0;
  a.nb = nb_w;
  a.M = M;
  a.N = (int)N;
  a.G = dC;
  a.ldg = lddc;
  for (int b = 0; b < nb_w; ++b) {
    HLH_CHECK_ARG(A[b] && dW[b] && kb_w[b] > 0 && lda[b] >= kb_w[b] && lddw[b] >= kb_w[b],
                  "proj_bwd: bad weight block %d", b);
    a.A[b] = A[b];
    a.lda[b] = lda[b];
    a.kb[b] = (int)kb_w[b];
    a.tile_start[b] = p.tile_start[b];
    a.part_off[b] = p.part_off[b];
    r.part_off[b] = p.part_off[b];
    r.kb[b] = (int)kb_w[b];
    r.dW[b] = dW[b];
    r.lddw[b] = lddw[b];
    r.elem_start[b + 1] = r.elem_start[b] + N * kb_w[b];
  }
  a.tile_start[nb_w] = p.tile_start[nb_w];
  a.bias_off = p.bias_off;
  a.part_stride = p.part_stride;
  a.part = workspace;
  a.rows_per_split = p.rows_per_split;
  a.tiles_n = p.tiles_n;
  a.xcd_map = weight_xcd_map();
  f.n_w = p.tiles_total * p.splits;

  BwdDataArgs& d = f.d;
  d.nb = nb_d;
  d.M = M;
  d.N = (int)N;
  d.G = dC;
  d.ldg = lddc;
  d.accumulate = accumulate_d;
  int64_t ktot = 0;
  for (int b = 0; b < nb_d; ++b) ktot += kb_d[b];
  int tnd = ceil_div(M, 16) * ceil_div(ktot, 16) < 4096 ? 1 : 2;  // as hlhgat_proj_bwd_data
  if (tnd == 2 && bwd_tnd() == 4) tnd = 4;
  d.tile_start[0] = 0;
  for (int b = 0; b < nb_d; ++b) {
    HLH_CHECK_ARG(W[b] && dA[b] && kb_d[b] > 0 && ldw[b] >= kb_d[b] && ldda[b] >= kb_d[b],
                  "proj_bwd: bad data block %d", b);
    d.W[b] = W[b];
    d.O[b] = dA[b];
    d.ldw[b] = ldw[b];
    d.ldo[b] = ldda[b];
    d.kb[b] = (int)kb_d[b];
    d.tile_start[b + 1] = d.tile_start[b] + (int)ceil_div(kb_d[b], tnd * 16);
  }
  f.d_gx = (int)ceil_div(M, 4 * 16);
  f.n_wpad = (f.n_w + 7) & ~7;
  // N <= 64 (one dC chunk): one data workgroup per row block for every column
  // tile (dC read once); else one per (row block, column tile)
  bool vec_d = aligned16(dC) && lddc % 4 == 0;
  for (int b = 0; b < nb_d; ++b)
    vec_d = vec_d && aligned16(W[b]) && ldw[b] % 4 == 0 && kb_d[b] % 4 == 0;
  const bool rows = proj_bwd_rows_flag() && tnd == 4 && N <= KC && vec_d;
  f.n_d = rows ? f.d_gx : f.d_gx * d.tile_start[nb_d];
  f.d_xcd = data_xcd_map();
  if (prev) {
    // (merging it only where it adds no round of workgroups -- an extra
    // launch otherwise -- measured 0.7-1.5 % slower at config 2, round 5)
    f.red = *prev;
    f.n_red = (int)reduce_blocks(*prev);
  }
  const int64_t n_blocks = (int64_t)f.n_wpad + (int64_t)f.n_d + (int64_t)f.n_red;
  HLH_CHECK_ARG(n_blocks < (int64_t)INT32_MAX, "proj_bwd: grid too large");
  hipStream_t s = as_stream(stream);
  // algorithmic flops of the launch: weight gradient 2 M N sum(kb_w) + data
  // gradient 2 M N sum(kb_d); bytes: dC once, each A_b and dA_b once, the W
  // blocks, the split slab written once
  double flops = 0, bytes = 4.0 * (double)M * N;
  for (int b = 0; b < nb_w; ++b) {
    flops += 2.0 * (double)M * N * kb_w[b];
    bytes += 4.0 * (double)M * kb_w[b];
  }
  for (int b = 0; b < nb_d; ++b) {
    flops += 2.0 * (double)M * N * kb_d[b];
    bytes += 4.0 * (double)M * kb_d[b] + 4.0 * N * kb_d[b];
  }
  bytes += 4.0 * (double)p.splits * p.part_stride;
  ProfScope prof(HLHGAT_PROF_PROJ_BWD, s, bytes, flops);
  if (rows)
    launch(k_proj_bwd_fused<4, true>, dim3((unsigned)n_blocks), dim3(256), 0, s, &prof, f);
  else if (tnd == 1)
    launch(k_proj_bwd_fused<1, false>, dim3((unsigned)n_blocks), dim3(256), 0, s, &prof, f);
  else if (tnd == 2)
    launch(k_proj_bwd_fused<2, false>, dim3((unsigned)n_blocks), dim3(256), 0, s, &prof, f);
  else
    launch(k_proj_bwd_fused<4, false>, dim3((unsigned)n_blocks), dim3(256), 0, s, &prof, f);
  HLH_CHECK_LAUNCH();
  r.splits = p.splits;
  r.part = workspace;
  r.part_stride = p.part_stride;
  r.bias_off = p.bias_off;
  r.dbias = dbias;
  r.accumulate = 0;
  if (defer_out) {
    memset(defer_out, 0, sizeof(*defer_out));
    defer_out->words[0] = kDescMagic;
    memcpy(&defer_out->words[1], &r, sizeof(r));
    if (deferred) *deferred = 1;
    return HLHGAT_OK;
  }
  return run_reduce(r, s);
}
}  // namespace

extern "C" int hlhgat_proj_bwd_defer(int64_t M, int64_t N, const float* dC, int64_t lddc,
                                     int nb_w, const float* const* A, const int64_t* lda,
                                     const int64_t* kb_w, float* const* dW, const int64_t* lddw,
                                     float* dbias, int nb_d, const float* const* W,
                                     const int64_t* ldw, const int64_t* kb_d, float* const* dA,
                                     const int64_t* ldda, int accumulate_d, float* workspace,
                                     int64_t workspace_floats, const hlhgat_reduce_desc_t* merge,
                                     hlhgat_reduce_desc_t* defer_out, int* deferred,
                                     void* stream) {
  return proj_bwd_impl(M, N, dC, lddc, nb_w, A, lda, kb_w, dW, lddw, dbias, nb_d, W, ldw, kb_d,
                       dA, ldda, accumulate_d, workspace, workspace_floats, stream, merge,
                       defer_out, deferred);
}

extern "C" int hlhgat_reduce_run(const hlhgat_reduce_desc_t* desc, void* stream) {
  HLH_CHECK_ARG(desc && desc->words[0] == kDescMagic, "reduce_run: not a reduce descriptor");
  return run_reduce(*reinterpret_cast<const ReduceArgs*>(&desc->words[1]), as_stream(stream));
}

extern "C" int hlhgat_proj_bwd(int64_t M, int64_t N, const float* dC, int64_t lddc,
                               int nb_w, const float* const* A, const int64_t* lda,
                               const int64_t* kb_w, float* const* dW, const int64_t* lddw,
                               float* dbias, int nb_d, const float* const* W,
                               const int64_t* ldw, const int64_t* kb_d, float* const* dA,
                               const int64_t* ldda, int accumulate_d, float* workspace,
                               int64_t workspace_floats, void* stream) {
  return proj_bwd_impl(M, N, dC, lddc, nb_w, A, lda, kb_w, dW, lddw, dbias,
                       nb_d, W, ldw, kb_d, dA, ldda, accumulate_d, workspace, workspace_floats,
                       stream);
}

extern "C" int hlhgat_set_gemm_big(int mode, int64_t min_m) {
  HLH_CHECK_ARG(mode >= -1 && mode <= 1, "set_gemm_big: mode must be -1, 0 or 1");
  g_big_mode.store(mode);
  if (min_m > 0) g_big_min_m.store(min_m);
  return HLHGAT_OK;
}

extern "C" int hlhgat_set_proj_bwd_rows(int on) {
  proj_bwd_rows_flag() = on != 0;
  return HLHGAT_OK;
}
