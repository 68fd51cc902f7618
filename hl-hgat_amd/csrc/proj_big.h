// Large-tile fp32 MFMA kernels of the projections, for the config 3-5 shapes
// (M = 1e4..2e5 simplices, N = 32..256, reduction widths up to ~1900): the
// forward C = sum_b A_b W_b^T (+ bias), the data gradient dA_b = dC W_b and
// the split weight gradient dW_b = dC^T A_b (partials into the split slab that
// k_reduce_splits sums).  Included by proj.hip after the argument structs.
//
// Why a second family: the 64x64-tile kernels above keep one 32x32 (or four
// 16x16) accumulators per wave and were measured at ~10 % of the fp32 MFMA
// peak on the TSP head (profiles/r05d_cfg5_step_kernels.txt: k_proj_bwd_fused
// 606 us per launch, 54 % of the config-5 step).  Here:
//   * a workgroup tile is up to 128 x 128 (4 waves, each a 64 x 64 block of
//     2 x 2 v_mfma_f32_32x32x2_f32 accumulators: 4 MFMAs per operand pair
//     read, every operand reused twice from registers);
//   * operands are staged through LDS 32 reduction steps at a time, double
//     buffered, with the next stage's global loads in flight during the MFMAs
//     and one barrier per stage;
//   * reduction-contiguous operands (A and W in the forward, dC in the data
//     gradient) are read with ONE ds_read_b128 per 4 MFMA steps: lane half h
//     of a 32x32x2 MFMA takes reduction index 16 h + s at step s (the order of
//     the sum inside a stage is permuted, which fp32 allows; every path that
//     is compared bitwise uses the same kernel).  LDS rows are 32 floats with
//     the 16-B slots XOR-swizzled by (row >> 1) & 7: a ds_read_b128 lane group
//     (16 distinct rows mod 16) then touches 16 distinct 4-bank groups and a
//     ds_write_b128 group of 8 lanes one contiguous 128-B row: conflict-free
//     (MI355X_MICROARCH.md, LDS table);
//   * the other operands (W_b in the data gradient, dC and A_b in the weight
//     gradient) vary along the reduction by row: lane li reads column li of
//     four consecutive rows with ds_read_b32 (32 consecutive floats per lane
//     group: conflict-free).
// 32x32x2 MFMA layout: lane l supplies A[i = l % 32][k = l / 32] and
// B[k = l / 32][j = l % 32]; accumulator register r of lane l holds
// D[(r & 3) + 8 (r >> 2) + 4 (l / 32)][l % 32].
#pragma once

namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BKC = 32;  // reduction steps per LDS stage

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// 16-B slot of a 32-float LDS row (see the header)
__device__ __forceinline__ int bslot(int row, int slot) { return slot ^ ((row >> 1) & 7); }

// ---------------------------------------------------------------------------
// staging helpers: ROWS x 32 floats of a row-major matrix (k contiguous), one
// float4 per thread and pass (thread t: row t / 8 + 32 u, slot t % 8)
// ---------------------------------------------------------------------------
template <int ROWS>
struct KStage {
  float4 v[ROWS / 32];
};

template <int ROWS>
__device__ __forceinline__ void kstage_load(KStage<ROWS>& st, const float* __restrict__ P,
                                            int64_t ld, int64_t row0, int64_t nrows, int k0,
                                            int kb) {
  const int r0 = threadIdx.x >> 3, k = k0 + 4 * (threadIdx.x & 7);
#pragma unroll
  for (int u = 0; u < ROWS / 32; ++u) {
    const int64_t row = row0 + r0 + 32 * u;
    st.v[u] = (row < nrows && k < kb) ? *reinterpret_cast<const float4*>(P + row * ld + k)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int ROWS>
__device__ __forceinline__ void kstage_store(float (*lds)[BKC], const KStage<ROWS>& st) {
  const int r0 = threadIdx.x >> 3, c4 = threadIdx.x & 7;
#pragma unroll
  for (int u = 0; u < ROWS / 32; ++u) {
    const int r = r0 + 32 * u;
    *reinterpret_cast<float4*>(&lds[r][4 * bslot(r, c4)]) = st.v[u];
  }
}

// 32 rows (reduction index) x COLS floats of a row-major matrix, stored
// unswizzled: thread t covers float4 (t % (COLS / 4)) of row t / (COLS / 4) + ...
template <int COLS>
struct RStage {
  float4 v[COLS / 32];
};

template <int COLS>
__device__ __forceinline__ void rstage_load(RStage<COLS>& st, const float* __restrict__ P,
                                            int64_t ld, int64_t row0, int64_t nrows, int c0,
                                            int ncols) {
  constexpr int C4 = COLS / 4;
#pragma unroll
  for (int u = 0; u < COLS / 32; ++u) {
    const int idx = threadIdx.x + 256 * u;
    const int r = idx / C4, c = c0 + 4 * (idx % C4);
    const int64_t row = row0 + r;
    st.v[u] = (row < nrows && c < ncols) ? *reinterpret_cast<const float4*>(P + row * ld + c)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int COLS>
__device__ __forceinline__ void rstage_store(float (*lds)[COLS], const RStage<COLS>& st) {
  constexpr int C4 = COLS / 4;
#pragma unroll
  for (int u = 0; u < COLS / 32; ++u) {
    const int idx = threadIdx.x + 256 * u;
    *reinterpret_cast<float4*>(&lds[idx / C4][4 * (idx % C4)]) = st.v[u];
  }
}

// one stage of MFMAs with both operands k-contiguous in swizzled LDS rows.
// The operand registers are double-buffered: group t + 1's ds_reads are issued
// before group t's 4 TBM TBN MFMAs, so their latency hides behind the MFMAs
// (with one set, the compiler issued each group's reads after the previous
// group's MFMAs and waited on them: an exposed LDS round trip per group).
template <int TBM, int TBN>
__device__ __forceinline__ void mma_kk(const float (*as)[BKC], const float (*bs)[BKC], int arow0,
                                       int brow0, floatx16 (&acc)[TBM][TBN]) {
  const int lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  float4 av[2][TBM], bv[2][TBN];
  auto fetch = [&](int t, int slot) {
#pragma unroll
    for (int bm = 0; bm < TBM; ++bm) {
      const int r = arow0 + 32 * bm + li;
      av[slot][bm] = *reinterpret_cast<const float4*>(&as[r][4 * bslot(r, 4 * lh + t)]);
    }
#pragma unroll
    for (int bn = 0; bn < TBN; ++bn) {
      const int r = brow0 + 32 * bn + li;
      bv[slot][bn] = *reinterpret_cast<const float4*>(&bs[r][4 * bslot(r, 4 * lh + t)]);
    }
  };
  fetch(0, 0);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int cur = t & 1;
    if (t + 1 < 4) fetch(t + 1, cur ^ 1);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int bm = 0; bm < TBM; ++bm)
#pragma unroll
        for (int bn = 0; bn < TBN; ++bn)
          acc[bm][bn] = mfma32(av[cur][bm][e], bv[cur][bn][e], acc[bm][bn]);
  }
}

template <int TBM, int TBN>
__device__ __forceinline__ void zero_acc(floatx16 (&acc)[TBM][TBN]) {
#pragma unroll
  for (int bm = 0; bm < TBM; ++bm)
#pragma unroll
    for (int bn = 0; bn < TBN; ++bn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[bm][bn][r] = 0.f;
}

constexpr int kBigFlush = 8;  // stages (256 products) per inner accumulation chain

template <int TBM, int TBN>
__device__ __forceinline__ void flush_acc(floatx16 (&acc)[TBM][TBN],
                                          floatx16 (&outer)[TBM][TBN]) {
#pragma unroll
  for (int bm = 0; bm < TBM; ++bm)
#pragma unroll
    for (int bn = 0; bn < TBN; ++bn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        outer[bm][bn][r] = outer[bm][bn][r] + acc[bm][bn][r];
        acc[bm][bn][r] = 0.f;
      }
}

// Epilogue through LDS (the main loop's buffers, free after its last
// barrier): every wave writes its accumulators (+ `outer`) into the tile
// (ds_write_b32, 32 consecutive columns per lane group: conflict-free), then
// the workgroup writes whole rows with float4 stores -- and float4 loads where
// it accumulates -- instead of 4-byte stores, one per accumulator register,
// into rows ld apart (the dense-slab outputs and gradient sinks, ld = the slab
// width, accumulate = 1).  bias (per column) is added on the way.
template <int WM, int WN, int TBM, int TBN>
__device__ __forceinline__ void store_tile_lds(const floatx16 (&acc)[TBM][TBN],
                                               const floatx16 (&outer)[TBM][TBN], bool with_outer,
                                               float* lds, float* dst, int64_t ld, int64_t row0,
                                               int64_t rows, int col0, int cols,
                                               const float* bias, int accumulate) {
  constexpr int BM = WM * TBM * 32, BN = WN * TBN * 32, C4 = BN / 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WM, wn = wave / WM, li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int bm = 0; bm < TBM; ++bm)
#pragma unroll
    for (int bn = 0; bn < TBN; ++bn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (wm * TBM + bm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int cc = (wn * TBN + bn) * 32 + li;
        lds[rr * BN + cc] = with_outer ? outer[bm][bn][r] + acc[bm][bn][r] : acc[bm][bn][r];
      }
  __syncthreads();
  const bool vec = (reinterpret_cast<uintptr_t>(dst) & 15) == 0 && (ld & 3) == 0 &&
                   (cols & 3) == 0 && (col0 & 3) == 0 &&
                   (!bias || (reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  for (int idx = threadIdx.x; idx < BM * C4; idx += 256) {
    const int r = idx / C4, c = 4 * (idx % C4);
    const int64_t row = row0 + r;
    const int col = col0 + c;
    if (row >= rows || col >= cols) continue;
    float4 v = *reinterpret_cast<const float4*>(&lds[r * BN + c]);
    float* d = dst + row * ld + col;
    if (vec) {
      if (bias) {
        const float4 bv = *reinterpret_cast<const float4*>(bias + col);
        v.x = v.x + bv.x;
        v.y = v.y + bv.y;
        v.z = v.z + bv.z;
        v.w = v.w + bv.w;
      }
      if (accumulate) {
        const float4 o = *reinterpret_cast<const float4*>(d);
        v.x = o.x + v.x;
        v.y = o.y + v.y;
        v.z = o.z + v.z;
        v.w = o.w + v.w;
      }
      *reinterpret_cast<float4*>(d) = v;
    } else {
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (col + j >= cols) break;
        float x = vv[j];
        if (bias) x = x + bias[col + j];
        d[j] = accumulate ? d[j] + x : x;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// forward: C[M][N] (+)= sum_b A_b[M][kb] W_b[N][kb]^T + bias
// Workgroup tile (WM * TBM * 32) x (WN * TBN * 32); grid = row blocks x
// column tiles (column tile fastest: the tiles of one row block share A).
// ---------------------------------------------------------------------------
template <int WM, int WN, int TBM, int TBN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_proj_fwd_big(FwdArgs a) {
  constexpr int BM = WM * TBM * 32, BN = WN * TBN * 32;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(2 * (BM + BN) * BKC >= BM * BN, "the epilogue tile fits the stage buffers");
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * BKC];
  float (*As)[BM][BKC] = reinterpret_cast<float (*)[BM][BKC]>(smem);
  float (*Bs)[BN][BKC] = reinterpret_cast<float (*)[BN][BKC]>(smem + 2 * BM * BKC);
  const int wave = threadIdx.x >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int ntile = (a.N + BN - 1) / BN;
  const int64_t m0 = (int64_t)(blockIdx.x / ntile) * BM;
  const int n0 = (int)(blockIdx.x % ntile) * BN;
  // two-level accumulation over the reduction (as the weight gradient's):
  // the MFMA chains restart every kBigFlush stages (256 products) into
  // `outer`, so a 1856-wide NodeEdgeInt Linear is not one 1856-long fp32 chain
  floatx16 acc[TBM][TBN], outer[TBM][TBN];
  zero_acc(acc);
  zero_acc(outer);
  int stage = 0;
  KStage<BM> sa;
  KStage<BN> sb;
  int b = 0, k0 = 0;
  kstage_load<BM>(sa, a.A[0], a.lda[0], m0, a.M, 0, a.kb[0]);
  kstage_load<BN>(sb, a.W[0], a.ldw[0], n0, a.N, 0, a.kb[0]);
  kstage_store<BM>(As[0], sa);
  kstage_store<BN>(Bs[0], sb);
  __syncthreads();
  int buf = 0;
  for (;;) {
    int nbk = b, nk = k0 + BKC;
    if (nk >= a.kb[b]) {
      nbk = b + 1;
      nk = 0;
    }
    const bool more = nbk < a.nb;
    if (more) {
      kstage_load<BM>(sa, a.A[nbk], a.lda[nbk], m0, a.M, nk, a.kb[nbk]);
      kstage_load<BN>(sb, a.W[nbk], a.ldw[nbk], n0, a.N, nk, a.kb[nbk]);
    }
    mma_kk<TBM, TBN>(As[buf], Bs[buf], wm * TBM * 32, wn * TBN * 32, acc);
    if (++stage % kBigFlush == 0 && more) flush_acc(acc, outer);
    if (more) {
      kstage_store<BM>(As[buf ^ 1], sa);
      kstage_store<BN>(Bs[buf ^ 1], sb);
    }
    __syncthreads();
    if (!more) break;
    buf ^= 1;
    b = nbk;
    k0 = nk;
  }
  store_tile_lds<WM, WN, TBM, TBN>(acc, outer, true, smem, a.C, a.ldc, m0, a.M, n0, a.N, a.bias,
                                   a.accumulate);
}

// ---------------------------------------------------------------------------
// data gradient: dA_b[M][kb] (+)= dC[M][N] W_b[N][kb]
// Tile (WM * TBM * 32) rows x (WN * TBN * 32) columns of one block's dA_b;
// grid = row blocks x column tiles of all blocks (a.tile_start in units of
// this tile width).  dC is k-contiguous (swizzled rows), W_b is staged as
// 32 reduction rows x the tile's columns.
// ---------------------------------------------------------------------------
template <int WM, int WN, int TBM, int TBN>
__global__ __launch_bounds__(256) void k_proj_bwd_data_big(BwdDataArgs a) {
  constexpr int BM = WM * TBM * 32, BC = WN * TBN * 32;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(2 * (BM + BC) * BKC >= BM * BC, "the epilogue tile fits the stage buffers");
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BC) * BKC];
  float (*Gs)[BM][BKC] = reinterpret_cast<float (*)[BM][BKC]>(smem);
  float (*Ws)[BKC][BC] = reinterpret_cast<float (*)[BKC][BC]>(smem + 2 * BM * BKC);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WM, wn = wave / WM;
  const int li = lane & 31, lh = lane >> 5;
  const int ctiles = a.tile_start[a.nb];
  const int64_t m0 = (int64_t)(blockIdx.x / ctiles) * BM;
  const int ct = (int)(blockIdx.x % ctiles);
  int b = 0;
  while (b + 1 < a.nb && ct >= a.tile_start[b + 1]) ++b;
  const int kb = a.kb[b];
  const int c0 = (ct - a.tile_start[b]) * BC;
  const float* __restrict__ W = a.W[b];
  const int64_t ldw = a.ldw[b];
  floatx16 acc[TBM][TBN];
  zero_acc(acc);
  KStage<BM> sg;
  RStage<BC> sw;
  kstage_load<BM>(sg, a.G, a.ldg, m0, a.M, 0, a.N);
  rstage_load<BC>(sw, W, ldw, 0, a.N, c0, kb);
  kstage_store<BM>(Gs[0], sg);
  rstage_store<BC>(Ws[0], sw);
  __syncthreads();
  int buf = 0;
  for (int n0 = 0; n0 < a.N; n0 += BKC) {
    const bool more = n0 + BKC < a.N;
    if (more) {
      kstage_load<BM>(sg, a.G, a.ldg, m0, a.M, n0 + BKC, a.N);
      rstage_load<BC>(sw, W, ldw, n0 + BKC, a.N, c0, kb);
    }
    {  // operand registers double-buffered across the 4 groups (see mma_kk)
      float4 av[2][TBM];
      float bv[2][TBN][4];
      auto fetch = [&](int t, int slot) {
#pragma unroll
        for (int bm = 0; bm < TBM; ++bm) {
          const int r = (wm * TBM + bm) * 32 + li;
          av[slot][bm] = *reinterpret_cast<const float4*>(&Gs[buf][r][4 * bslot(r, 4 * lh + t)]);
        }
#pragma unroll
        for (int bn = 0; bn < TBN; ++bn)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            bv[slot][bn][e] = Ws[buf][16 * lh + 4 * t + e][(wn * TBN + bn) * 32 + li];
      };
      fetch(0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int cur = t & 1;
        if (t + 1 < 4) fetch(t + 1, cur ^ 1);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int bm = 0; bm < TBM; ++bm)
#pragma unroll
            for (int bn = 0; bn < TBN; ++bn)
              acc[bm][bn] = mfma32(av[cur][bm][e], bv[cur][bn][e], acc[bm][bn]);
      }
    }
    if (more) {
      kstage_store<BM>(Gs[buf ^ 1], sg);
      rstage_store<BC>(Ws[buf ^ 1], sw);
    }
    __syncthreads();
    buf ^= 1;
  }
  store_tile_lds<WM, WN, TBM, TBN>(acc, acc, false, smem, a.O[b], a.ldo[b], m0, a.M, c0, kb,
                                   nullptr, a.accumulate);
}

// ---------------------------------------------------------------------------
// weight gradient partials: slab[split][n][k] = sum over the split's rows m of
// dC[m][n] A_b[m][k]; bias partials = column sums of dC (block 0, first k
// tile).  Tile (WM * TBM * 32) n x (WN * TBN * 32) k; items (tile, split)
// dealt XCD-aware (weight_item).  Two-level accumulation as
// bwd_weight32_body: the MFMA chains restart every kBigFlush stages.
// ---------------------------------------------------------------------------
template <int WM, int WN, int TBM, int TBN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_proj_bwd_weight_big(BwdWeightArgs a) {
  constexpr int BNT = WM * TBM * 32, BC = WN * TBN * 32;
  static_assert(WM * WN == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) float Gs[2][BKC][BNT];
  __shared__ __attribute__((aligned(16))) float Xs[2][BKC][BC];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wm = wave % WM, wn = wave / WM;
  const int li = lane & 31, lh = lane >> 5;
  const int Y = a.tile_start[a.nb];
  int by, bz;
  weight_item(blockIdx.x, (unsigned)Y, gridDim.x, by, bz);
  int b = 0;
  while (b + 1 < a.nb && by >= a.tile_start[b + 1]) ++b;
  const int t = by - a.tile_start[b];
  const int n0 = (t % a.tiles_n) * BNT;
  const int c0 = (t / a.tiles_n) * BC;
  const int kb = a.kb[b];
  const float* __restrict__ A = a.A[b];
  const int64_t lda = a.lda[b];
  const bool do_bias = a.bias_off >= 0 && b == 0 && c0 == 0 && wn == 0;
  const int64_t m_lo = (int64_t)bz * a.rows_per_split;
  int64_t m_hi = m_lo + a.rows_per_split;
  if (m_hi > a.M) m_hi = a.M;
  const int nst = m_hi > m_lo ? (int)((m_hi - m_lo + BKC - 1) / BKC) : 0;

  floatx16 acc[TBM][TBN], outer[TBM][TBN];
  zero_acc(acc);
  zero_acc(outer);
  float bsum[TBM], bouter[TBM];
#pragma unroll
  for (int bm = 0; bm < TBM; ++bm) bsum[bm] = bouter[bm] = 0.f;
  RStage<BNT> sg;
  RStage<BC> sx;
  if (nst > 0) {
    rstage_load<BNT>(sg, a.G, a.ldg, m_lo, m_hi, n0, a.N);
    rstage_load<BC>(sx, A, lda, m_lo, m_hi, c0, kb);
    rstage_store<BNT>(Gs[0], sg);
    rstage_store<BC>(Xs[0], sx);
  }
  __syncthreads();
  int buf = 0;
  for (int s = 0; s < nst; ++s) {
    const bool more = s + 1 < nst;
    if (more) {
      const int64_t mn = m_lo + (int64_t)(s + 1) * BKC;
      rstage_load<BNT>(sg, a.G, a.ldg, mn, m_hi, n0, a.N);
      rstage_load<BC>(sx, A, lda, mn, m_hi, c0, kb);
    }
    {  // operand registers double-buffered across the 4 groups (see mma_kk)
      float av[2][TBM][4], bv[2][TBN][4];
      auto fetch = [&](int q, int slot) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = 16 * lh + 4 * q + e;
#pragma unroll
          for (int bm = 0; bm < TBM; ++bm)
            av[slot][bm][e] = Gs[buf][m][(wm * TBM + bm) * 32 + li];
#pragma unroll
          for (int bn = 0; bn < TBN; ++bn)
            bv[slot][bn][e] = Xs[buf][m][(wn * TBN + bn) * 32 + li];
        }
      };
      fetch(0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int cur = q & 1;
        if (q + 1 < 4) fetch(q + 1, cur ^ 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#pragma unroll
          for (int bm = 0; bm < TBM; ++bm) {
#pragma unroll
            for (int bn = 0; bn < TBN; ++bn)
              acc[bm][bn] = mfma32(av[cur][bm][e], bv[cur][bn][e], acc[bm][bn]);
            if (do_bias) bsum[bm] = bsum[bm] + av[cur][bm][e];
          }
        }
      }
    }
    if ((s + 1) % kBigFlush == 0 && more) {
#pragma unroll
      for (int bm = 0; bm < TBM; ++bm) {
#pragma unroll
        for (int bn = 0; bn < TBN; ++bn)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            outer[bm][bn][r] = outer[bm][bn][r] + acc[bm][bn][r];
            acc[bm][bn][r] = 0.f;
          }
        bouter[bm] = bouter[bm] + bsum[bm];
        bsum[bm] = 0.f;
      }
    }
    if (more) {
      rstage_store<BNT>(Gs[buf ^ 1], sg);
      rstage_store<BC>(Xs[buf ^ 1], sx);
    }
    __syncthreads();
    buf ^= 1;
  }
  float* slab = a.part + (int64_t)bz * a.part_stride + a.part_off[b];
#pragma unroll
  for (int bm = 0; bm < TBM; ++bm)
#pragma unroll
    for (int bn = 0; bn < TBN; ++bn) {
      const int k = c0 + (wn * TBN + bn) * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + (wm * TBM + bm) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (n < a.N && k < kb) slab[(int64_t)n * kb + k] = outer[bm][bn][r] + acc[bm][bn][r];
      }
    }
  if (do_bias) {
#pragma unroll
    for (int bm = 0; bm < TBM; ++bm) {
      // lanes l and l + 32 hold the sums over the two halves of each stage
      const float v = bouter[bm] + bsum[bm];
      const float tot = v + __shfl_xor(v, 32, 64);
      const int n = n0 + (wm * TBM + bm) * 32 + li;
      if (lh == 0 && n < a.N) a.part[(int64_t)bz * a.part_stride + a.bias_off + n] = tot;
    }
  }
}

}  // namespace
