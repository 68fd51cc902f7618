// Shared device code of the fp32 MFMA projection forward (proj.hip) and the
// fused projection + BatchNorm forward (bn.hip): operand staging, the
// LDS-staged main loop and the row-store epilogue.  Everything here has
// internal linkage (anonymous namespace): each including file gets its own copy.
#pragma once
#include "common.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int MAXB = HLHGAT_MAX_BLOCKS;

__device__ __forceinline__ floatx4 mfma16(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// forward: C = sum_b A_b W_b^T + bias
// ---------------------------------------------------------------------------
struct FwdArgs {
  int nb;
  int N;
  int64_t M;
  const float* A[MAXB];
  const float* W[MAXB];
  int64_t lda[MAXB];
  int64_t ldw[MAXB];
  int kb[MAXB];
  const float* bias;
  float* C;
  int64_t ldc;
  int accumulate;
  int xcd_map;  // k_proj_fwd_lds: the column tiles of one row block on one XCD
};

// ---------------------------------------------------------------------------
// forward, LDS-staged weights (vector path: every kb % 4 == 0, 16-B aligned)
//
// Workgroup = 4 waves x 16 rows = 64 rows, TN*16 output columns.  The weight
// chunk W_b[n_tile][k0:k0+64] is loaded ONCE per workgroup into LDS (double
// buffered, rows padded to 68 floats so the 16 rows a ds_read_b128 lane group
// touches fall in 16 distinct 16-B bank slots) and shared by the 4 waves;
// each lane streams its A row chunk straight into registers one chunk ahead.
// ---------------------------------------------------------------------------
constexpr int KC = 64;
// LDS row pitch of a staged W chunk: 64 floats, with the 16-B slots of row r
// XOR-swizzled by r & 15 (slot k/4 of row r lives at slot (k/4) ^ (r & 15)).
// A ds_read_b128 lane group of the main loop (lanes (q, i) reading row
// tn*16 + i, slot 4s + q) then touches 16 distinct slots and a ds_write_b128
// group of 8 lanes 8 distinct bank quads: both conflict-free
// (MI355X_MICROARCH.md §LDS), where the former 68-float padding left the
// reads 2-way conflicted (SQ_LDS_BANK_CONFLICT ~0.4 of the LDS cycles).
constexpr int KCP = KC;
__device__ __forceinline__ int wswz(int row, int slot) { return slot ^ (row & 15); }

template <int TN>
struct WStage {
  float4 v[TN];
};

// cooperative load of W rows [n_base, n_base+TN*16) x k [k0, k0+64) of block b
template <int TN>
__device__ __forceinline__ void load_w_chunk(const FwdArgs& a, int b, int k0, int n_base,
                                             WStage<TN>& st) {
  const float* W = a.W[b];
  const int kb = a.kb[b];
  const int64_t ldw = a.ldw[b];
#pragma unroll
  for (int u = 0; u < TN; ++u) {
    const int idx = threadIdx.x + 256 * u;  // TN*16 rows x 16 float4
    const int r = idx >> 4, c4 = idx & 15;
    const int n = n_base + r, k = k0 + 4 * c4;
    if (n < a.N && k < kb)
      st.v[u] = *reinterpret_cast<const float4*>(W + (int64_t)n * ldw + k);
    else
      st.v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int TN>
__device__ __forceinline__ void store_w_chunk(float (*lds)[KCP], const WStage<TN>& st) {
#pragma unroll
  for (int u = 0; u < TN; ++u) {
    const int idx = threadIdx.x + 256 * u;
    const int r = idx >> 4, c4 = idx & 15;
    *reinterpret_cast<float4*>(&lds[r][4 * wswz(r, c4)]) = st.v[u];
  }
}

__device__ __forceinline__ void load_a_chunk(const float* arow, bool valid, int k0, int kb,
                                             int q, float4 (&o)[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = k0 + 16 * s + 4 * q;
    if (valid && k < kb)
      o[s] = *reinterpret_cast<const float4*>(arow + k);
    else
      o[s] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Epilogue through LDS: a wave's 16 x (TN*16) accumulator tile (lane (q,i)
// holds rows 4q..4q+3 of column i) is transposed in a per-wave LDS scratch
// (pitch TN*16+4: the 64 lanes' writes hit 64 distinct banks) and written
// back as whole-row float4 stores (each store instruction covers 4 full
// 64-column rows) instead of 4-byte column-strided stores.
template <int TN>
__device__ __forceinline__ void store_tile_rows(const floatx4 (&acc)[TN], float* scratch,
                                                int64_t row0, int64_t M, float* dst0,
                                                int64_t ld, int ncols, const float* bias,
                                                int accumulate, bool vec_ok) {
  constexpr int CT = TN * 16, P = CT + 4;
  const int lane = threadIdx.x & 63, q = lane >> 4, i = lane & 15;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int col = tn * 16 + i;
    const float bv = (bias && col < ncols) ? bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = acc[tn][r];
      if (bias) v = v + bv;
      scratch[(4 * q + r) * P + col] = v;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (vec_ok) {
#pragma unroll
    for (int u = 0; u < TN; ++u) {
      const int idx = lane + 64 * u;
      const int r = idx / (CT / 4), c4 = idx % (CT / 4);
      const int64_t row = row0 + r;
      if (row < M && 4 * c4 < ncols) {
        float4 v = *reinterpret_cast<const float4*>(&scratch[r * P + 4 * c4]);
        float4* d = reinterpret_cast<float4*>(dst0 + row * ld + 4 * c4);
        if (accumulate) {
          const float4 o = *d;
          v.x = o.x + v.x;
          v.y = o.y + v.y;
          v.z = o.z + v.z;
          v.w = o.w + v.w;
        }
        *d = v;
      }
    }
  } else {
    for (int idx = lane; idx < 16 * CT; idx += 64) {
      const int r = idx / CT, c = idx % CT;
      const int64_t row = row0 + r;
      if (row < M && c < ncols) {
        float* d = dst0 + row * ld + c;
        const float v = scratch[r * P + c];
        *d = accumulate ? *d + v : v;
      }
    }
  }
}

// The forward main loop: on return acc[tn] of lane (q, i) holds
// C[m_base + 4q + r][n_base + tn*16 + i] (r = 0..3, no bias) for wave rows
// m_base = (bx * 4 + wave) * 16, n_base = by * TN * 16; every wave is past
// the loop's last barrier, so wl is free for an epilogue.
template <int TN>
__device__ __forceinline__ void proj_fwd_lds_mainloop(const FwdArgs& a, int bx, int by,
                                                      float (*wl)[TN * 16][KCP],
                                                      floatx4 (&acc)[TN]) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int q = lane >> 4, i = lane & 15;
  const int64_t m_base = ((int64_t)bx * 4 + wave) * 16;
  const int n_base = by * (TN * 16);
  const int64_t row = m_base + i;
  const bool aval = row < a.M;

#pragma unroll
  for (int tn = 0; tn < TN; ++tn) acc[tn] = floatx4{0.f, 0.f, 0.f, 0.f};

  int b = 0, k0 = 0;
  WStage<TN> wst;
  float4 ac[4];
  load_w_chunk<TN>(a, b, k0, n_base, wst);
  load_a_chunk(a.A[b] + (aval ? row : 0) * a.lda[b], aval, k0, a.kb[b], q, ac);
  store_w_chunk<TN>(wl[0], wst);
  __syncthreads();
  int buf = 0;
  while (b < a.nb) {
    int nbk = b, nk = k0 + KC;
    if (nk >= a.kb[b]) {
      nbk = b + 1;
      nk = 0;
    }
    const bool has_next = nbk < a.nb;
    float4 an[4];
    if (has_next) {
      load_w_chunk<TN>(a, nbk, nk, n_base, wst);
      load_a_chunk(a.A[nbk] + (aval ? row : 0) * a.lda[nbk], aval, nk, a.kb[nbk], q, an);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float4 bf[TN];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        bf[tn] = *reinterpret_cast<const float4*>(&wl[buf][tn * 16 + i][4 * wswz(i, 4 * s + q)]);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        acc[tn] = mfma16(ac[s].x, bf[tn].x, acc[tn]);
        acc[tn] = mfma16(ac[s].y, bf[tn].y, acc[tn]);
        acc[tn] = mfma16(ac[s].z, bf[tn].z, acc[tn]);
        acc[tn] = mfma16(ac[s].w, bf[tn].w, acc[tn]);
      }
    }
    if (has_next) {
      store_w_chunk<TN>(wl[buf ^ 1], wst);
#pragma unroll
      for (int s = 0; s < 4; ++s) ac[s] = an[s];
    }
    __syncthreads();
    buf ^= 1;
    b = nbk;
    k0 = nk;
  }
}

}  // namespace
