// Training-mode BatchNorm1d (+ optional fused ReLU) for the HL blocks.
//
// Every HL block is HodgeLaguerreConv -> gnn.BatchNorm -> ReLU -> Dropout
// (lib/Hodge_ST_Model.py:556-566) and every NodeEdgeInt value MLP is
// Linear -> BatchNorm1d -> ReLU twice (lib/Hodge_Cheb_Conv.py:276-289), so
// each conv output passes through a batch-statistics reduction over all
// simplices (40 per direction in the config-2 step).
//
// The rows are split into `parts` row partitions x `tiles` column tiles, one
// workgroup each; every workgroup writes fp64 column partials (forward: sum,
// sum of squares; backward: sum g, sum g (x - mean), g = dy masked by the ReLU).
//
// Forward in ONE launch (default, k_bn_fwd_grid) when the whole grid is
// provably co-resident: each workgroup keeps its rows in REGISTERS, writes its
// partials, meets the other partitions of its column tile at a bounded grid
// barrier, sums ALL partials itself in a fixed order (flat_reduce), and
// normalises from the registers -- no second read of x, no last-arriver tail,
// no flag hand-off.  Workgroup 0 of a tile writes the saved and running
// statistics.  (The same structure for the backward ran 12 % faster alone,
// 31.8 vs 35.5 us per fwd+bwd at the ZINC shape, but made the training step
// 1.2 % SLOWER in a same-box A/B -- its register-heavy workgroups wait at the
// barrier while the other stream's kernels need the CUs -- so it was removed.)
//
// Otherwise, and always for the backward: two launches, k_bn_stats /
// k_bn_bwd_reduce (the last workgroup to arrive sums the partials -- in the
// same flat order up to kFlatMax partitions, so both forward paths give
// bitwise the same results; a two-level last-arriver tree above) then
// k_bn_apply / k_bn_bwd_apply.
//
// Arithmetic (both paths): mean = S0/n, var = S1/n - mean^2 (fp64),
// invstd = 1/sqrt(var + eps); y = relu?((x - mean) * w invstd + b);
// dx = A g + (B (x - mean) + C) with A = w is, B = -w is^3 Sgx/n,
// C = -w is Sg/n -- the centred forms, as torch evaluates them.
//
// Inter-workgroup hand-off (MI355X_MICROARCH.md / cdna_hip_programming.md
// Guideline 16): partials are written through with agent-scope atomic stores
// drained by vmcnt(0) before a barrier; one lane takes a relaxed agent atomic
// ticket; readers use agent-scope atomic loads.
#include "gemm_core.h"

#include <cstdlib>

using namespace hlhgat;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxParts = 512;
constexpr int kFlatMax = 256;                     // flat reduction order up to this many parts
constexpr int kGroup = 16;                        // partitions per first-level tree group
constexpr int kMaxGroups = kMaxParts / kGroup;
constexpr int kMaxTiles = 1024;
constexpr int kGridBase = kMaxTiles * (1 + kMaxGroups);  // per tile: top + group counters
// + per tile: the one-launch kernels' barrier arrival and leave counters
constexpr int kCounters = kGridBase + 2 * kMaxTiles;
constexpr int APPLY_RPT = 2;  // rows per thread in the elementwise apply kernels
constexpr int kMaxRpt = 32;   // rows per thread the one-launch kernels hold in registers

struct BnLayout {
  int v;       // floats per thread (4 or 1)
  int tpr;     // threads per row within a column tile
  int rp;      // rows per pass (kThreads / tpr)
  int tile_c;  // columns per tile (tpr * v)
  int tiles;   // column tiles
  int parts;   // row partitions (grid.x)
  int64_t rows_per_part;
};

// hlhgat_set_bn_one_launch(0): two launches per direction even where one
// fits (tests; bitwise the same results).
bool& bn_one_launch_flag() {
  static bool v = true;
  return v;
}
bool bn_one_launch() { return bn_one_launch_flag(); }

// Row partitions: >= 128 (same-box A/B at the ZINC step, n ~ 25k: 64 ->
// 281.8k, 128 -> 287.2k, 256 -> 286.1k, 32 -> 265.8k graphs/s), one per 512
// rows above (config 3 / 5 heads, 1.4e5-2e5 rows: 64 workgroups left most of
// the 256 CUs idle).
int64_t bn_parts(int64_t n) {
  int64_t p = std::max<int64_t>(128, ceil_div(n, (int64_t)512));
  // small batches (the readout MLP: one row per graph): >= 64 rows per
  // partition, so the finaliser's partial loads stay one batch deep
  p = std::min<int64_t>(p, std::max<int64_t>(1, ceil_div(n, (int64_t)64)));
  return p < 1 ? 1 : (p > kMaxParts ? kMaxParts : p);
}

BnLayout bn_layout(int64_t n, int64_t C, bool vec) {
  BnLayout L;
  L.v = vec ? 4 : 1;
  int lanes = (int)ceil_div(C, L.v);
  L.tpr = next_pow2(lanes);
  if (L.tpr > kThreads / L.v) L.tpr = kThreads / L.v;  // tile_c <= kThreads
  L.rp = kThreads / L.tpr;
  L.tile_c = L.tpr * L.v;
  L.tiles = (int)ceil_div(C, L.tile_c);
  int64_t parts = bn_parts(n);
  int64_t max_parts = ceil_div(n, (int64_t)L.rp * 2);
  if (parts > max_parts) parts = max_parts;
  if (parts < 1) parts = 1;
  if (parts > kMaxParts) parts = kMaxParts;
  L.rows_per_part = ceil_div(n, parts);
  L.parts = (int)ceil_div(n > 0 ? n : 1, L.rows_per_part);
  return L;
}

struct BnWs {
  unsigned* count;   // [kCounters] at offset 0 (zero between launches)
  double* part;      // [parts][C][2]
  double* gpart;     // [groups][C][2]
  float* coef;       // [3][C] (bwd: a, b, c)
};

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

// Counters live at a FIXED offset so a launch with a different (n, C) never
// reads another launch's partials as a counter.
size_t bn_ws_bytes(int64_t n, int64_t C) {
  (void)n;
  return align_up(sizeof(unsigned) * kCounters) + align_up(sizeof(double) * 2 * kMaxParts * C) +
         align_up(sizeof(double) * 2 * kMaxGroups * C) + align_up(sizeof(float) * 3 * C);
}

BnWs carve(void* ws, int64_t n, int64_t C) {
  (void)n;
  char* p = (char*)ws;
  BnWs w;
  w.count = (unsigned*)p;
  p += align_up(sizeof(unsigned) * kCounters);
  w.part = (double*)p;
  p += align_up(sizeof(double) * 2 * kMaxParts * C);
  w.gpart = (double*)p;
  p += align_up(sizeof(double) * 2 * kMaxGroups * C);
  w.coef = (float*)p;
  return w;
}

// n_valid (optional, device int32): only rows [0, min(n, *n_valid)) are
// simplices of the batch; the rest are capacity padding (hlhgat.train static
// shapes).  Statistics use the valid rows only, outputs / gradients of padded
// rows are written as 0.
__device__ __forceinline__ int64_t eff_rows(int64_t n, const int32_t* nvalid) {
  if (!nvalid) return n;
  const int64_t v = (int64_t)*nvalid;
  return v < n ? (v < 0 ? 0 : v) : n;
}

struct StatsArgs {
  const int32_t* nvalid;
  const float* x;
  int64_t ldx;
  const float* y;   // bwd: forward output for the ReLU mask (or NULL)
  int64_t ldy;
  const float* dy;  // bwd only
  int64_t lddy;
  int64_t n;
  int C;
  int tpr, rp, tiles, parts;
  int64_t rows_per_part;
  double* part;
  double* gpart;
  unsigned* count;
  // forward finalisation
  const float* weight;
  const float* bias;
  float* running_mean;
  float* running_var;
  int64_t* nbt;
  float momentum, eps;
  float* save_mean;
  float* save_invstd;
  // backward finalisation
  float* coef;
  float* dweight;
  float* dbias;
  // one-launch kernels: output rows, poll limit of the barrier, error word
  float* out;
  int64_t ldo;
  int relu;
  unsigned poll_limit;
  unsigned* err;
  // SyncBatchNorm (hlhgat_bn_sums_*): the finaliser writes this rank's fp64
  // column sums [S0[C], S1[C], n_eff] here instead of finishing the statistics
  double* sums_out;
  // input rows produced in the launch (hlhgat_bn_fwd_produced), written to
  // xw (ldx) for the backward
  const int64_t* pei;  // edge rows: [2][n] endpoints
  const int32_t* prow;  // node rows: incidence CSR (node -> incident edge ids)
  const int32_t* peid;
  const float* prs;     // node rows: per-row scale
  const float* pp;      // gathered rows
  int64_t ldp;
  const float* pz;      // per-row addend
  int64_t ldz;
  float pca, pcb;
  float* xw;
};

// The NodeEdgeInt hidden layer's input rows, computed where the BatchNorm
// reads them (bitwise the producers' own arithmetic):
//   PROD 1 (edge rows, hlhgat_edge_gather2 with sa = sb = NULL):
//     x[e] = z[e] + (ca (1 p[i]) + cb (1 p[j]))
//   PROD 2 (node rows, hlhgat_poly_step over the binary incidence with
//     rs, alpha = gamma = 1): x[v] = 1 (rs[v] sum_{CSR order} p[eid]) + 1 z[v]
template <int PROD, int V>
__device__ __forceinline__ typename VecT<V>::type produce_row(const StatsArgs& a, int64_t r,
                                                              int c) {
  using vt = typename VecT<V>::type;
  vt o;
  if constexpr (PROD == 1) {
    const int64_t i = a.pei[r], j = a.pei[a.n + r];
    const float si = 1.f, sj = 1.f;
    vt xi = vload<V>(a.pp + i * a.ldp + c);
    vt xj = vload<V>(a.pp + j * a.ldp + c);
    vt zv = vload<V>(a.pz + r * a.ldz + c);
#pragma unroll
    for (int v = 0; v < V; ++v) vget(o, v) = a.pca * (si * vget(xi, v)) + a.pcb * (sj * vget(xj, v));
#pragma unroll
    for (int v = 0; v < V; ++v) vget(o, v) = vget(zv, v) + vget(o, v);
  } else {
    const int e0 = a.prow[r], e1 = a.prow[r + 1];
    vt acc;
#pragma unroll
    for (int v = 0; v < V; ++v) vget(acc, v) = 0.f;
    const float w = 1.f;
    int p = e0;
    for (; p + 1 < e1; p += 2) {  // two gathers in flight, adds in CSR order
      vt x0 = vload<V>(a.pp + (int64_t)a.peid[p] * a.ldp + c);
      vt x1 = vload<V>(a.pp + (int64_t)a.peid[p + 1] * a.ldp + c);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float s = vget(acc, v);
        s = s + w * vget(x0, v);
        s = s + w * vget(x1, v);
        vget(acc, v) = s;
      }
    }
    for (; p < e1; ++p) {
      vt x0 = vload<V>(a.pp + (int64_t)a.peid[p] * a.ldp + c);
#pragma unroll
      for (int v = 0; v < V; ++v) vget(acc, v) = vget(acc, v) + w * vget(x0, v);
    }
    const float rsv = a.prs[r];
    const float alpha = 1.f, gamma = 1.f;
    vt zv = vload<V>(a.pz + r * a.ldz + c);
#pragma unroll
    for (int v = 0; v < V; ++v) vget(o, v) = alpha * (rsv * vget(acc, v));
#pragma unroll
    for (int v = 0; v < V; ++v) vget(o, v) = vget(o, v) + gamma * vget(zv, v);
  }
  return o;
}

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// wait timeouts of the one-launch kernels (hlhgat_bn_wait_timeouts)
__device__ unsigned g_bn_wait_timeouts = 0;

// A workgroup that gives up at the barrier (poll limit reached) must not use
// partial statistics: it writes NaN into its rows, counts the timeout and
// raises HLHGAT_DEVERR_BN_WAIT in the host-visible error word
// (hlhgat_device_errors), which hlhgat.train.TrainStep, the bench and
// hlhgat.ops.check_device_errors turn into a Python exception.
__device__ __forceinline__ void report_wait_timeout(unsigned* err) {
  __hip_atomic_fetch_add(&g_bn_wait_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (err) __hip_atomic_store(err, (unsigned)HLHGAT_DEVERR_BN_WAIT, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_SYSTEM);
}

// Signal arrival; returns true in the last workgroup of `total`.  Every wave
// has drained its write-through partial stores (vmcnt(0)) before the barrier;
// ONE lane adds to the counter; the workgroup whose add returned total-1
// resets it and reads the partials after the second barrier.
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned total) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    s_last = (prev == total - 1) ? 1u : 0u;
    if (s_last) *counter = 0u;  // ready for the next launch (stream-ordered)
  }
  __syncthreads();
  return s_last != 0u;
}

// Grid barrier of the `total` workgroups of one column tile (all co-resident,
// see pick_grid) on ONE 64-bit word: count in the low half, generation in the
// high half.  Every workgroup adds 1; the one that completes the count turns
// it back to 0 and bumps the generation in the same word (a single atomic add
// of 2^32 - total), the others poll until the generation changes or the poll
// limit runs out (poll_limit == 0, a test hook: give up at once).  Nothing is
// left to reset afterwards, whatever `total` the next launch uses.  Returns
// false on timeout.
typedef __attribute__((address_space(1))) unsigned long long gu64c_t;
__device__ __forceinline__ bool bar_wait(unsigned long long* word, unsigned total,
                                         unsigned poll_limit, unsigned* err) {
  __shared__ unsigned s_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long old =
        __hip_atomic_fetch_add((gu64c_t*)word, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned ok = 0;
    if ((unsigned)(old & 0xffffffffull) == total - 1) {
      __hip_atomic_fetch_add((gu64c_t*)word, (1ull << 32) - (unsigned long long)total,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = 1;
    } else {
      const unsigned gen = (unsigned)(old >> 32);
      for (unsigned it = 0; it < poll_limit; ++it) {
        const unsigned long long w =
            __hip_atomic_load((gu64c_t*)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(w >> 32) != gen) {
          ok = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (!ok) report_wait_timeout(err);
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0u;
}

// the barrier word of this launch's column tile (8-byte aligned: kGridBase is even)
__device__ __forceinline__ unsigned long long* barrier_word(const StatsArgs& a, const Blk& blk) {
  return reinterpret_cast<unsigned long long*>(a.count + kGridBase) + blk.y;
}

// Block-level column partials: threads (row group rg, column lane cl) hold V
// columns each; reduce over the rp row groups through LDS in fixed order.
template <int V, int NT>
__device__ __forceinline__ void write_partials(double (&s0)[V], double (&s1)[V],
                                               const StatsArgs& a, int c0, const Blk& blk) {
  __shared__ double red[2][NT * 4];
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    red[0][rg * a.tpr * V + cl * V + v] = s0[v];
    red[1][rg * a.tpr * V + cl * V + v] = s1[v];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < a.tpr * V; t += NT) {
    double u0 = 0.0, u1 = 0.0;
    for (int g = 0; g < a.rp; ++g) {
      u0 += red[0][g * a.tpr * V + t];
      u1 += red[1][g * a.tpr * V + t];
    }
    const int c = c0 + t;
    if (c < a.C) {
      double* dst = a.part + ((int64_t)blk.x * a.C + c) * 2;
      st_wt(dst, u0);
      st_wt(dst + 1, u1);
    }
  }
}

// The flat order (both paths, parts <= kFlatMax): thread group j of G =
// NT / tile_c sums partials p = j, j + G, j + 2G, ... in ascending order
// (loads in batches of 32), then the groups are added in order 0..G-1.
// Result in out0 / out1[0 .. tile_c).
template <int NT>
__device__ __forceinline__ void flat_reduce(const double* src, int parts, const StatsArgs& a,
                                            int c0, int tile_c, double* out0, double* out1) {
  __shared__ double fin[2][NT];
  const int G = NT / tile_c > 0 ? NT / tile_c : 1;
  const int t = threadIdx.x % tile_c;
  const int j = threadIdx.x / tile_c;
  const int c = c0 + t;
  double u0 = 0.0, u1 = 0.0;
  if (j < G && c < a.C) {
    for (int p0 = j; p0 < parts; p0 += 32 * G) {  // 32 loads of each in flight
      double v0[32], v1[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        const int p = p0 + u * G;
        const bool ok = p < parts;
        const double* q = src + ((int64_t)(ok ? p : 0) * a.C + c) * 2;
        v0[u] = ok ? ld_wt(q) : 0.0;
        v1[u] = ok ? ld_wt(q + 1) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        u0 += v0[u];
        u1 += v1[u];
      }
    }
  }
  fin[0][threadIdx.x] = u0;
  fin[1][threadIdx.x] = u1;
  __syncthreads();
  if (threadIdx.x < tile_c) {
    double s0 = 0.0, s1 = 0.0;
    for (int g = 0; g < G; ++g) {
      s0 += fin[0][g * tile_c + threadIdx.x];
      s1 += fin[1][g * tile_c + threadIdx.x];
    }
    out0[threadIdx.x] = s0;
    out1[threadIdx.x] = s1;
  }
  __syncthreads();
}

// Sum of partials [first, first+count) of src ([*][C][2]) for the tile's
// columns (the tree levels, parts > kFlatMax): all threads take part (column
// t % tile_c, partial group t / tile_c, loads in batches of 16), groups
// combined in fixed order through LDS -> deterministic.
template <int NT>
__device__ __forceinline__ void reduce_range(const double* src, int first, int count,
                                             const StatsArgs& a, int c0, int tile_c,
                                             double* out0, double* out1) {
  __shared__ double fin[2][NT];
  const int groups = NT / tile_c > 0 ? NT / tile_c : 1;
  const int t = threadIdx.x % tile_c;
  const int grp = threadIdx.x / tile_c;
  const int c = c0 + t;
  const int per = (count + groups - 1) / groups;
  const int p0 = grp * per;
  double u0 = 0.0, u1 = 0.0;
  if (grp < groups && c < a.C) {
    for (int pb = 0; pb < per; pb += 16) {
      double v0[16], v1[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int p = p0 + pb + u;
        const bool ok = pb + u < per && p < count;
        const double* q = src + ((int64_t)(first + (ok ? p : 0)) * a.C + c) * 2;
        v0[u] = ok ? ld_wt(q) : 0.0;
        v1[u] = ok ? ld_wt(q + 1) : 0.0;
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        u0 += v0[u];
        u1 += v1[u];
      }
    }
  }
  fin[0][threadIdx.x] = u0;
  fin[1][threadIdx.x] = u1;
  __syncthreads();
  if (threadIdx.x < tile_c) {
    double s0 = 0.0, s1 = 0.0;
    for (int g = 0; g < groups; ++g) {
      s0 += fin[0][g * tile_c + threadIdx.x];
      s1 += fin[1][g * tile_c + threadIdx.x];
    }
    out0[threadIdx.x] = s0;
    out1[threadIdx.x] = s1;
  }
  __syncthreads();
}

// The two-launch reduction: true (sums in out0/out1) in the one workgroup of
// the column tile that finalises.  Flat order up to kFlatMax partitions
// (one arrival counter), else a two-level last-arriver tree.
template <int NT>
__device__ __forceinline__ bool last_reduce(const StatsArgs& a, int c0, int tile_c,
                                            double* out0, double* out1, const Blk& blk) {
  const int tile = blk.y;
  if (a.parts <= kFlatMax) {
    if (!arrive_last(a.count + tile, (unsigned)a.parts)) return false;
    flat_reduce<NT>(a.part, a.parts, a, c0, tile_c, out0, out1);
    return true;
  }
  const int g = blk.x / kGroup;
  const int ng = (a.parts + kGroup - 1) / kGroup;
  const int first = g * kGroup;
  const int cnt = a.parts - first < kGroup ? a.parts - first : kGroup;
  if (!arrive_last(a.count + kMaxTiles + tile * kMaxGroups + g, (unsigned)cnt)) return false;
  reduce_range<NT>(a.part, first, cnt, a, c0, tile_c, out0, out1);
  for (int t = threadIdx.x; t < tile_c; t += NT) {
    const int c = c0 + t;
    if (c < a.C) {
      double* dst = a.gpart + ((int64_t)g * a.C + c) * 2;
      st_wt(dst, out0[t]);
      st_wt(dst + 1, out1[t]);
    }
  }
  if (!arrive_last(a.count + tile, (unsigned)ng)) return false;
  reduce_range<NT>(a.gpart, 0, ng, a, c0, tile_c, out0, out1);
  return true;
}

// Forward finalisation of one column (all paths, SyncBatchNorm included:
// there n_eff and the sums are the totals over ranks): mean, invstd, and the
// running statistics when `update`.
__device__ __forceinline__ void finalize_col(double u0, double u1, double n_eff, float eps,
                                             float momentum, float* running_mean,
                                             float* running_var, int cc, float& mean_f,
                                             float& invstd_f, bool update) {
  const double nn = n_eff > 0.0 ? n_eff : 1.0;
  const double mean = u0 / nn;
  double var = u1 / nn - mean * mean;
  if (var < 0.0) var = 0.0;
  mean_f = (float)mean;
  invstd_f = (float)(1.0 / sqrt(var + (double)eps));
  if (update && running_mean) {
    const double unb = n_eff > 1.0 ? var * nn / (nn - 1.0) : var;
    running_mean[cc] = (1.f - momentum) * running_mean[cc] + momentum * (float)mean;
    running_var[cc] = (1.f - momentum) * running_var[cc] + momentum * (float)unb;
  }
}

__device__ __forceinline__ void fwd_finalize(const StatsArgs& a, int cc, double u0, double u1,
                                             int64_t n_eff, float& mean_f, float& invstd_f,
                                             bool update) {
  finalize_col(u0, u1, (double)n_eff, a.eps, a.momentum, a.running_mean, a.running_var, cc,
               mean_f, invstd_f, update);
}

// Backward coefficients of one column (all paths): dx = A g + (B (x - mean) + C).
__device__ __forceinline__ void bwd_coefs(float is_f, float w_f, double sg, double sgx,
                                          double n_eff, float& A, float& B, float& Cc) {
  const double is = (double)is_f;
  const double w = (double)w_f;
  const double nn = n_eff > 0.0 ? n_eff : 1.0;
  A = (float)(w * is);
  B = (float)(-w * is * is * is * sgx / nn);
  Cc = (float)(-w * is * sg / nn);
}

// SyncBatchNorm: the column tile's sums and the valid row count of this rank
// (layout [S0[C], S1[C], n_eff], fp64: hlhgat_bn_sums_fwd / _bwd).
__device__ __forceinline__ void write_sums(const StatsArgs& a, int c0, int tile_c,
                                           const double* sum0, const double* sum1,
                                           int64_t n_eff, const Blk& blk) {
  for (int t = threadIdx.x; t < tile_c; t += kThreads) {
    const int cc = c0 + t;
    if (cc >= a.C) continue;
    a.sums_out[cc] = sum0[t];
    a.sums_out[a.C + cc] = sum1[t];
  }
  if (blk.y == 0 && threadIdx.x == 0) a.sums_out[2 * a.C] = (double)n_eff;
}

// ---------------------------------------------------------------------------
// two-launch path
// ---------------------------------------------------------------------------
template <int V>
__device__ __forceinline__ void k_bn_stats_body(const StatsArgs& a, Blk blk) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c0 = blk.y * a.tpr * V;
  const int c = c0 + cl * V;
  const int64_t r_lo = (int64_t)blk.x * a.rows_per_part;
  int64_t r_hi = r_lo + a.rows_per_part;
  const int64_t n_eff = eff_rows(a.n, a.nvalid);
  if (r_hi > n_eff) r_hi = n_eff;
  double s0[V], s1[V];
#pragma unroll
  for (int v = 0; v < V; ++v) s0[v] = s1[v] = 0.0;
  if (c < a.C) {
    int64_t r = r_lo + rg;
    for (; r + 7 * a.rp < r_hi; r += 8 * a.rp) {  // 8 rows in flight
      vt x4[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x4[u] = vload<V>(a.x + (r + u * a.rp) * a.ldx + c);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const double xd = (double)vget(x4[u], v);
          s0[v] += xd;
          s1[v] += xd * xd;
        }
    }
    for (; r < r_hi; r += a.rp) {
      vt xv = vload<V>(a.x + r * a.ldx + c);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const double xd = (double)vget(xv, v);
        s0[v] += xd;
        s1[v] += xd * xd;
      }
    }
  }
  write_partials<V, kThreads>(s0, s1, a, c0, blk);
  __shared__ double sum0[kThreads], sum1[kThreads];
  const int tile_c = a.tpr * V;
  if (!last_reduce<kThreads>(a, c0, tile_c, sum0, sum1, blk)) return;
  if (a.sums_out) {  // SyncBatchNorm: this rank's sums, finalised after the all-gather
    write_sums(a, c0, tile_c, sum0, sum1, n_eff, blk);
    return;
  }
  for (int t = threadIdx.x; t < tile_c; t += kThreads) {
    const int cc = c0 + t;
    if (cc >= a.C) continue;
    float m, is;
    fwd_finalize(a, cc, sum0[t], sum1[t], n_eff, m, is, true);
    a.save_mean[cc] = m;
    a.save_invstd[cc] = is;
  }
  if (a.nbt && blk.y == 0 && threadIdx.x == 0) a.nbt[0] += 1;
}

template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_stats(StatsArgs a) {
  k_bn_stats_body<V>(a, blk_hw());
}

struct ApplyArgs {
  const int32_t* nvalid;
  const float* x;
  int64_t ldx;
  float* y;
  int64_t ldy;
  int64_t n;
  int C;
  const float* mean;
  const float* invstd;
  const float* weight;
  const float* bias;
  int relu;
  int tpr, rp;
};

template <int V>
__device__ __forceinline__ void k_bn_apply_body(const ApplyArgs& a, Blk blk) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c = blk.y * a.tpr * V + cl * V;
  if (c >= a.C) return;
  float s[V], m[V], t[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const float w = a.weight ? a.weight[c + v] : 1.f;
    s[v] = w * a.invstd[c + v];
    m[v] = a.mean[c + v];
    t[v] = a.bias ? a.bias[c + v] : 0.f;
  }
  // APPLY_RPT rows per thread, all loads issued before any store
  const int64_t n_eff = eff_rows(a.n, a.nvalid);
  const int64_t r0 = (int64_t)blk.x * a.rp * APPLY_RPT + rg;
  vt xv[APPLY_RPT];
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r < n_eff) xv[u] = vload<V>(a.x + r * a.ldx + c);
  }
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r >= a.n) break;
    vt o;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float z = (vget(xv[u], v) - m[v]) * s[v] + t[v];
      vget(o, v) = r >= n_eff ? 0.f : ((a.relu && z < 0.f) ? 0.f : z);
    }
    vstore<V>(a.y + r * a.ldy + c, o);
  }
}

template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_apply(ApplyArgs a) {
  k_bn_apply_body<V>(a, blk_hw());
}

struct BwdApplyArgs {
  const int32_t* nvalid;
  const float* x;
  int64_t ldx;
  const float* y;
  int64_t ldy;
  const float* dy;
  int64_t lddy;
  float* dx;
  int64_t lddx;
  int64_t n;
  int C;
  const float* coef;
  const float* mean;
  int tpr, rp;
};

// Backward statistics (two-launch path): partials of sum(g), sum(g (x - mean));
// the finalising workgroup of a column tile forms dweight, dbias and dx's
// coefficients.
template <int V>
__device__ __forceinline__ void k_bn_bwd_reduce_body(const StatsArgs& a, Blk blk) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c0 = blk.y * a.tpr * V;
  const int c = c0 + cl * V;
  const int64_t r_lo = (int64_t)blk.x * a.rows_per_part;
  int64_t r_hi = r_lo + a.rows_per_part;
  const int64_t n_eff = eff_rows(a.n, a.nvalid);
  if (r_hi > n_eff) r_hi = n_eff;
  double s0[V], s1[V];
  float mu[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    s0[v] = s1[v] = 0.0;
    mu[v] = (c + v < a.C) ? a.save_mean[c + v] : 0.f;
  }
  if (c < a.C) {
    auto acc = [&](vt xv, vt gv, vt yv) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float g = vget(gv, v);
        if (a.y && !(vget(yv, v) > 0.f)) g = 0.f;
        s0[v] += (double)g;
        s1[v] += (double)g * (double)(vget(xv, v) - mu[v]);
      }
    };
    int64_t r = r_lo + rg;
    for (; r + 3 * a.rp < r_hi; r += 4 * a.rp) {  // 4 rows (12 loads) in flight
      vt xv[4], gv[4], yv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t rr = r + u * a.rp;
        xv[u] = vload<V>(a.x + rr * a.ldx + c);
        gv[u] = vload<V>(a.dy + rr * a.lddy + c);
        if (a.y) yv[u] = vload<V>(a.y + rr * a.ldy + c);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc(xv[u], gv[u], yv[u]);
    }
    for (; r < r_hi; r += a.rp) {
      vt xv = vload<V>(a.x + r * a.ldx + c);
      vt gv = vload<V>(a.dy + r * a.lddy + c);
      vt yv = gv;
      if (a.y) yv = vload<V>(a.y + r * a.ldy + c);
      acc(xv, gv, yv);
    }
  }
  write_partials<V, kThreads>(s0, s1, a, c0, blk);
  __shared__ double sum0[kThreads], sum1[kThreads];
  const int tile_c = a.tpr * V;
  if (!last_reduce<kThreads>(a, c0, tile_c, sum0, sum1, blk)) return;
  if (a.sums_out) {  // SyncBatchNorm: local dweight / dbias, global coefficients later
    write_sums(a, c0, tile_c, sum0, sum1, n_eff, blk);
    for (int t = threadIdx.x; t < tile_c; t += kThreads) {
      const int cc = c0 + t;
      if (cc >= a.C) continue;
      if (a.dweight) a.dweight[cc] = (float)(sum1[t] * (double)a.save_invstd[cc]);
      if (a.dbias) a.dbias[cc] = (float)sum0[t];
    }
    return;
  }
  for (int t = threadIdx.x; t < tile_c; t += kThreads) {
    const int cc = c0 + t;
    if (cc >= a.C) continue;
    float A, B, Cc;
    bwd_coefs(a.save_invstd[cc], a.weight ? a.weight[cc] : 1.f, sum0[t], sum1[t], n_eff, A, B,
              Cc);
    if (a.dweight) a.dweight[cc] = (float)(sum1[t] * (double)a.save_invstd[cc]);
    if (a.dbias) a.dbias[cc] = (float)sum0[t];
    a.coef[cc] = A;
    a.coef[a.C + cc] = B;
    a.coef[2 * a.C + cc] = Cc;
  }
}

template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_bwd_reduce(StatsArgs a) {
  k_bn_bwd_reduce_body<V>(a, blk_hw());
}

template <int V>
__device__ __forceinline__ void k_bn_bwd_apply_body(const BwdApplyArgs& a, Blk blk) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c = blk.y * a.tpr * V + cl * V;
  if (c >= a.C) return;
  float A[V], B[V], Cc[V], mu[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    A[v] = a.coef[c + v];
    B[v] = a.coef[a.C + c + v];
    Cc[v] = a.coef[2 * a.C + c + v];
    mu[v] = a.mean[c + v];
  }
  const int64_t n_eff = eff_rows(a.n, a.nvalid);
  const int64_t r0 = (int64_t)blk.x * a.rp * APPLY_RPT + rg;
  vt xv[APPLY_RPT], gv[APPLY_RPT], yv[APPLY_RPT];
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r < n_eff) {
      xv[u] = vload<V>(a.x + r * a.ldx + c);
      gv[u] = vload<V>(a.dy + r * a.lddy + c);
      if (a.y) yv[u] = vload<V>(a.y + r * a.ldy + c);
    }
  }
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r >= a.n) break;
    vt o;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float g = vget(gv[u], v);
      if (a.y && !(vget(yv[u], v) > 0.f)) g = 0.f;
      vget(o, v) = r >= n_eff ? 0.f : A[v] * g + (B[v] * (vget(xv[u], v) - mu[v]) + Cc[v]);
    }
    vstore<V>(a.dx + r * a.lddx + c, o);
  }
}

template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_bwd_apply(BwdApplyArgs a) {
  k_bn_bwd_apply_body<V>(a, blk_hw());
}

// ---------------------------------------------------------------------------
// SyncBatchNorm apply kernels: every thread totals its columns' sums over the
// gathered ranks IN RANK ORDER (the same fp64 operations in every workgroup
// and on every rank, so all ranks hold the same statistics), then finishes
// exactly as the single-rank kernels do.  One rank: 0 + S = S, so the
// results are bitwise those of hlhgat_bn_fwd_train / hlhgat_bn_bwd_train on
// the same layout.
// ---------------------------------------------------------------------------
struct SyncArgs {
  const int32_t* nvalid;
  const float* x;
  int64_t ldx;
  const float* y;   // bwd: forward output (ReLU mask) or NULL
  int64_t ldy;
  const float* dy;  // bwd only
  int64_t lddy;
  float* out;       // fwd: y; bwd: dx
  int64_t ldo;
  int64_t n;
  int C;
  int tpr, rp;
  const double* gathered;  // [world][2C+1]
  int world;
  const float* weight;
  const float* bias;
  float* running_mean;
  float* running_var;
  int64_t* nbt;
  float momentum, eps;
  float* save_mean;    // fwd: written; bwd: read
  float* save_invstd;  // fwd: written; bwd: read
  int relu;
};

__device__ __forceinline__ void sync_totals(const SyncArgs& a, int cc, double& s0, double& s1,
                                            double& cnt) {
  s0 = s1 = cnt = 0.0;
  const int64_t stride = 2 * (int64_t)a.C + 1;
  for (int r = 0; r < a.world; ++r) {
    const double* g = a.gathered + r * stride;
    s0 += g[cc];
    s1 += g[a.C + cc];
    cnt += g[2 * a.C];
  }
}

template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_sync_apply(SyncArgs a) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c = blockIdx.y * a.tpr * V + cl * V;
  if (c >= a.C) return;
  float s[V], m[V], t[V];
  const bool writer = blockIdx.x == 0 && rg == 0;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    double s0, s1, cnt;
    sync_totals(a, c + v, s0, s1, cnt);
    float mean, is;
    finalize_col(s0, s1, cnt, a.eps, a.momentum, a.running_mean, a.running_var, c + v, mean, is,
                 writer);
    if (writer) {
      a.save_mean[c + v] = mean;
      a.save_invstd[c + v] = is;
    }
    const float w = a.weight ? a.weight[c + v] : 1.f;
    s[v] = w * is;
    m[v] = mean;
    t[v] = a.bias ? a.bias[c + v] : 0.f;
  }
  if (a.nbt && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) a.nbt[0] += 1;
  const int64_t n_eff = eff_rows(a.n, a.nvalid);
  const int64_t r0 = (int64_t)blockIdx.x * a.rp * APPLY_RPT + rg;
  vt xv[APPLY_RPT];
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r < n_eff) xv[u] = vload<V>(a.x + r * a.ldx + c);
  }
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r >= a.n) break;
    vt o;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float z = (vget(xv[u], v) - m[v]) * s[v] + t[v];
      vget(o, v) = r >= n_eff ? 0.f : ((a.relu && z < 0.f) ? 0.f : z);
    }
    vstore<V>(a.out + r * a.ldo + c, o);
  }
}

template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_sync_bwd_apply(SyncArgs a) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c = blockIdx.y * a.tpr * V + cl * V;
  if (c >= a.C) return;
  float A[V], B[V], Cc[V], mu[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    double sg, sgx, cnt;
    sync_totals(a, c + v, sg, sgx, cnt);
    bwd_coefs(a.save_invstd[c + v], a.weight ? a.weight[c + v] : 1.f, sg, sgx, cnt, A[v], B[v],
              Cc[v]);
    mu[v] = a.save_mean[c + v];
  }
  const int64_t n_eff = eff_rows(a.n, a.nvalid);
  const int64_t r0 = (int64_t)blockIdx.x * a.rp * APPLY_RPT + rg;
  vt xv[APPLY_RPT], gv[APPLY_RPT], yv[APPLY_RPT];
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r < n_eff) {
      xv[u] = vload<V>(a.x + r * a.ldx + c);
      gv[u] = vload<V>(a.dy + r * a.lddy + c);
      if (a.y) yv[u] = vload<V>(a.y + r * a.ldy + c);
    }
  }
#pragma unroll
  for (int u = 0; u < APPLY_RPT; ++u) {
    const int64_t r = r0 + u * a.rp;
    if (r >= a.n) break;
    vt o;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float g = vget(gv[u], v);
      if (a.y && !(vget(yv[u], v) > 0.f)) g = 0.f;
      vget(o, v) = r >= n_eff ? 0.f : A[v] * g + (B[v] * (vget(xv[u], v) - mu[v]) + Cc[v]);
    }
    vstore<V>(a.out + r * a.ldo + c, o);
  }
}

// ---------------------------------------------------------------------------
// one-launch path: rows held in registers across a grid barrier
// ---------------------------------------------------------------------------
// Forward: thread (rg, cl) owns rows r_lo + rg + j * rp (j < RPT) of its
// partition; statistics rows stop at n_eff, output rows at n.
template <int V, int RPT, int PROD = 0>
__device__ __forceinline__ void k_bn_fwd_grid_body(const StatsArgs& a, Blk blk) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c0 = blk.y * a.tpr * V;
  const int c = c0 + cl * V;
  const int64_t r_lo = (int64_t)blk.x * a.rows_per_part;
  const int64_t n_eff = eff_rows(a.n, a.nvalid);
  int64_t r_hi = r_lo + a.rows_per_part;
  if (r_hi > n_eff) r_hi = n_eff;
  vt xr[RPT];
  double s0[V], s1[V];
#pragma unroll
  for (int v = 0; v < V; ++v) s0[v] = s1[v] = 0.0;
  if (c < a.C) {
    if constexpr (PROD != 0) {
      // every row of the partition (padding rows too: the producer wrote them)
      int64_t r_end = r_lo + a.rows_per_part;
      if (r_end > a.n) r_end = a.n;
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int64_t r = r_lo + rg + (int64_t)j * a.rp;
        if (r < r_end) {
          xr[j] = produce_row<PROD, V>(a, r, c);
          vstore<V>(a.xw + r * a.ldx + c, xr[j]);
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int64_t r = r_lo + rg + (int64_t)j * a.rp;
        if (r < r_hi) xr[j] = vload<V>(a.x + r * a.ldx + c);
      }
    }
#pragma unroll
    for (int j = 0; j < RPT; ++j) {  // row order, as k_bn_stats
      const int64_t r = r_lo + rg + (int64_t)j * a.rp;
      if (r < r_hi) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const double xd = (double)vget(xr[j], v);
          s0[v] += xd;
          s1[v] += xd * xd;
        }
      }
    }
  }
  // per-column parameters fetched before the barrier (off the critical path)
  float wv[V], bv[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const bool in = c + v < a.C;
    wv[v] = (a.weight && in) ? a.weight[c + v] : 1.f;
    bv[v] = (a.bias && in) ? a.bias[c + v] : 0.f;
  }
  write_partials<V, kThreads>(s0, s1, a, c0, blk);
  const bool ok = bar_wait(barrier_word(a, blk), blk.gx, a.poll_limit, a.err);
  __shared__ double sum0[kThreads], sum1[kThreads];
  __shared__ float sm[kThreads], ss[kThreads];
  const int tile_c = a.tpr * V;
  if (ok) flat_reduce<kThreads>(a.part, blk.gx, a, c0, tile_c, sum0, sum1);
  for (int t = threadIdx.x; t < tile_c; t += kThreads) {
    const int cc = c0 + t;
    float m = __builtin_nanf(""), is = __builtin_nanf("");
    if (ok && cc < a.C) {
      fwd_finalize(a, cc, sum0[t], sum1[t], n_eff, m, is, blk.x == 0);
      if (blk.x == 0) {
        a.save_mean[cc] = m;
        a.save_invstd[cc] = is;
      }
    }
    sm[t] = m;
    ss[t] = is;
  }
  if (ok && a.nbt && blk.x == 0 && blk.y == 0 && threadIdx.x == 0) a.nbt[0] += 1;
  __syncthreads();
  if (c < a.C) {
    float sc[V], mu[V], sh[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      sc[v] = wv[v] * ss[cl * V + v];  // NaN after a barrier timeout
      mu[v] = sm[cl * V + v];
      sh[v] = bv[v];
    }
    int64_t r_end = r_lo + a.rows_per_part;
    if (r_end > a.n) r_end = a.n;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int64_t r = r_lo + rg + (int64_t)j * a.rp;
      if (r < r_end) {
        vt o;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float z = (vget(xr[j], v) - mu[v]) * sc[v] + sh[v];
          vget(o, v) = r >= n_eff ? 0.f : ((a.relu && z < 0.f) ? 0.f : z);  // NaN passes
        }
        vstore<V>(a.out + r * a.ldo + c, o);
      }
    }
  }
}

template <int V, int RPT>
__global__ __launch_bounds__(kThreads) void k_bn_fwd_grid(StatsArgs a) {
  k_bn_fwd_grid_body<V, RPT>(a, blk_hw());
}

template <int RPT, int PROD>
__global__ __launch_bounds__(kThreads) void k_bn_fwd_produced(StatsArgs a) {
  k_bn_fwd_grid_body<4, RPT, PROD>(a, blk_hw());
}

// ---------------------------------------------------------------------------
// Projection + BatchNorm (+ ReLU) forward in ONE launch (hlhgat_proj_bn_fwd)
//
// Every BatchNorm of the HL blocks and of the NodeEdgeInt MLPs reads the
// output of the Linear / conv projection just before it (lib/Hodge_ST_Model.py:
// 556-566, lib/Hodge_Cheb_Conv.py:276-289).  Here the projection's workgroups
// (64 rows x 64 columns each, proj_fwd_lds_mainloop) keep their output tile
// in registers and finish the BatchNorm themselves:
//   1. x = A W^T + bias is stored (the backward needs it) and the tile's fp64
//      column sums over its valid rows are formed in a fixed order (rows of a
//      lane, lanes q by xor 16 then 32, waves 0..3) and written through;
//   2. a two-level last-arriver tree per 64-column tile: the last workgroup of
//      each group of kGroup partials sums them (reduce_range, fixed order),
//      the last group sums the group partials, finalises mean / invstd and the
//      running statistics, and bumps the tile's generation word;
//   3. every other workgroup polls that word (bounded: a timeout writes NaN
//      rows and raises HLHGAT_DEVERR_BN_WAIT, as k_bn_fwd_grid), reads the
//      statistics and normalises its tile from the registers: y = relu?((x -
//      mean) * (w invstd) + b), rows >= n_valid written as 0.
// All workgroups must be co-resident (the host checks half of the chip's
// capacity, as for k_bn_fwd_grid).  Against projection -> k_bn_fwd_grid this
// saves the BatchNorm launch, its read of x and its own load latency.  The
// statistics are the same sums in a different fp64 order (not bitwise the
// two-kernel path; equal to 1e-6, tests/test_gpu_parity.py).
// ---------------------------------------------------------------------------
struct ProjBnArgs {
  FwdArgs g;    // the projection: g.C = x (pre-BatchNorm), g.ldc
  StatsArgs s;  // the BatchNorm: s.out = y, partials / counters / error word
};

constexpr int kPbTN = 4;  // 64 columns per workgroup: one BatchNorm column tile

__device__ __forceinline__ unsigned long long* gen_word(const StatsArgs& a, int tile) {
  return reinterpret_cast<unsigned long long*>(a.count + kGridBase) + tile;
}

__global__ __launch_bounds__(kThreads) void k_proj_bn_fwd(ProjBnArgs a) {
  __shared__ __attribute__((aligned(16))) float wl[2][kPbTN * 16][KCP];
  __shared__ unsigned s_gen0, s_ok;
  const FwdArgs& g = a.g;
  const StatsArgs& s = a.s;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = lane >> 4, i = lane & 15;
  const int bx = (int)blockIdx.x, by = (int)blockIdx.y;
  const int64_t m_base = ((int64_t)bx * 4 + wave) * 16;
  const int n_base = by * (kPbTN * 16);
  floatx4 acc[kPbTN];
  proj_fwd_lds_mainloop<kPbTN>(g, bx, by, wl, acc);
  // x = acc + bias, as store_tile_rows adds it
  if (g.bias) {
#pragma unroll
    for (int tn = 0; tn < kPbTN; ++tn) {
      const float bv = g.bias[n_base + tn * 16 + i];
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[tn][r] = acc[tn][r] + bv;
    }
  }
  // LDS after the main loop: per-wave row-store scratch in the first 17 KB,
  // the column sums behind it
  float* scratch = &wl[0][0][0] + wave * 16 * (kPbTN * 16 + 4);
  double* red = reinterpret_cast<double*>(&wl[0][0][0] + 4 * 16 * (kPbTN * 16 + 4));  // [2][4][64]
  double* sum0 = red + 2 * 4 * 64;  // [64]
  double* sum1 = sum0 + 64;         // [64]
  const bool vx = (g.ldc % 4) == 0 && (reinterpret_cast<uintptr_t>(g.C) & 15) == 0;
  store_tile_rows<kPbTN>(acc, scratch, m_base, g.M, g.C + n_base, g.ldc, kPbTN * 16, nullptr, 0,
                         vx);
  const int64_t n_eff = eff_rows(s.n, s.nvalid);
#pragma unroll
  for (int tn = 0; tn < kPbTN; ++tn) {
    double u0 = 0.0, u1 = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (m_base + 4 * q + r < n_eff) {
        const double xd = (double)acc[tn][r];
        u0 += xd;
        u1 += xd * xd;
      }
    }
    u0 += __shfl_xor(u0, 16, 64);
    u1 += __shfl_xor(u1, 16, 64);
    u0 += __shfl_xor(u0, 32, 64);
    u1 += __shfl_xor(u1, 32, 64);
    if (q == 0) {
      red[(0 * 4 + wave) * 64 + tn * 16 + i] = u0;
      red[(1 * 4 + wave) * 64 + tn * 16 + i] = u1;
    }
  }
  __syncthreads();
  unsigned long long* word = gen_word(s, by);
  if (threadIdx.x < 64) {
    const int t = threadIdx.x;
    const double v0 = ((red[0 * 256 + t] + red[0 * 256 + 64 + t]) + red[0 * 256 + 128 + t]) +
                      red[0 * 256 + 192 + t];
    const double v1 = ((red[1 * 256 + t] + red[1 * 256 + 64 + t]) + red[1 * 256 + 128 + t]) +
                      red[1 * 256 + 192 + t];
    double* dst = s.part + ((int64_t)bx * s.C + n_base + t) * 2;
    st_wt(dst, v0);
    st_wt(dst + 1, v1);
  }
  if (threadIdx.x == 0)  // the generation before this workgroup's arrival
    s_gen0 = (unsigned)(__hip_atomic_load((gu64c_t*)word, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) >> 32);
  const int parts = (int)gridDim.x;
  const int grp = bx / kGroup, ng = (parts + kGroup - 1) / kGroup;
  const int first = grp * kGroup;
  const int cnt = parts - first < kGroup ? parts - first : kGroup;
  bool top = false;
  if (arrive_last(s.count + kMaxTiles + by * kMaxGroups + grp, (unsigned)cnt)) {
    reduce_range<kThreads>(s.part, first, cnt, s, n_base, 64, sum0, sum1);
    if (threadIdx.x < 64) {
      double* dst = s.gpart + ((int64_t)grp * s.C + n_base + threadIdx.x) * 2;
      st_wt(dst, sum0[threadIdx.x]);
      st_wt(dst + 1, sum1[threadIdx.x]);
    }
    top = arrive_last(s.count + by, (unsigned)ng);
  }
  float* sm = reinterpret_cast<float*>(sum1 + 64);  // [64]
  float* ss = sm + 64;                              // [64]
  if (top) {
    reduce_range<kThreads>(s.gpart, 0, ng, s, n_base, 64, sum0, sum1);
    if (threadIdx.x < 64) {
      const int cc = n_base + threadIdx.x;
      float m, is;
      fwd_finalize(s, cc, sum0[threadIdx.x], sum1[threadIdx.x], n_eff, m, is, true);
      __hip_atomic_store(reinterpret_cast<unsigned*>(s.save_mean + cc), __float_as_uint(m),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(reinterpret_cast<unsigned*>(s.save_invstd + cc), __float_as_uint(is),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sm[threadIdx.x] = m;
      ss[threadIdx.x] = is;
    }
    if (s.nbt && by == 0 && threadIdx.x == 0) s.nbt[0] += 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add((gu64c_t*)word, 1ull << 32, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (threadIdx.x == 0) {
      unsigned ok = 0;
      for (unsigned it = 0; it < s.poll_limit; ++it) {
        const unsigned long long w =
            __hip_atomic_load((gu64c_t*)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(w >> 32) != s_gen0) {
          ok = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (!ok) report_wait_timeout(s.err);
      s_ok = ok;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int cc = n_base + threadIdx.x;
      float m = __builtin_nanf(""), is = __builtin_nanf("");
      if (s_ok) {
        m = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(s.save_mean + cc),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        is = __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(s.save_invstd + cc),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
      sm[threadIdx.x] = m;
      ss[threadIdx.x] = is;
    }
  }
  __syncthreads();
  // y from the registers (k_bn_fwd_grid's arithmetic)
#pragma unroll
  for (int tn = 0; tn < kPbTN; ++tn) {
    const int cl = tn * 16 + i, cc = n_base + cl;
    const float sc = (s.weight ? s.weight[cc] : 1.f) * ss[cl];  // NaN after a timeout
    const float mu = sm[cl];
    const float sh = s.bias ? s.bias[cc] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = (acc[tn][r] - mu) * sc + sh;
      acc[tn][r] = m_base + 4 * q + r >= n_eff ? 0.f : ((s.relu && z < 0.f) ? 0.f : z);
    }
  }
  const bool vy = (s.ldo % 4) == 0 && (reinterpret_cast<uintptr_t>(s.out) & 15) == 0;
  store_tile_rows<kPbTN>(acc, scratch, m_base, g.M, s.out + n_base, s.ldo, kPbTN * 16, nullptr,
                         0, vy);
}

bool& proj_bn_fused_flag() {
  static bool v = true;
  return v;
}

bool bn_vec_ok(int64_t C, std::initializer_list<int64_t> lds,
               std::initializer_list<const void*> ptrs) {
  if (C % 4) return false;
  for (int64_t ld : lds)
    if (ld % 4) return false;
  for (const void* p : ptrs)
    if (p && !aligned16(p)) return false;
  return true;
}

unsigned apply_grid_x(int64_t n, int rp) {
  int64_t g = ceil_div(n, (int64_t)rp * APPLY_RPT);  // every row owned by one thread
  if (g < 1) g = 1;
  return (unsigned)g;
}

StatsArgs stats_args(const BnLayout& L, const BnWs& w, const float* x, int64_t ldx, int64_t n,
                     const int32_t* n_valid, int64_t C) {
  StatsArgs s{};
  s.nvalid = n_valid;
  s.x = x;
  s.ldx = ldx;
  s.n = n;
  s.C = (int)C;
  s.tpr = L.tpr;
  s.rp = L.rp;
  s.tiles = L.tiles;
  s.parts = L.parts;
  s.rows_per_part = L.rows_per_part;
  s.part = w.part;
  s.gpart = w.gpart;
  s.count = w.count;
  return s;
}

// --- one-launch selection: co-residency and registers ------------------------
// The one-launch kernels' barrier needs every workgroup of a column tile
// resident at once.  They are used only when the whole grid fits in HALF of
// the chip's resident-workgroup capacity for that kernel
// (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs): the HL blocks' node
// and edge chains run on two streams (hlhgat.ops.fork) and each may be inside
// one such launch at the same time; every other kernel on the device
// completes without waiting, so it only delays residency.  Also: grid <= 256
// workgroups, the partials use the flat order, and a thread's rows fit the
// register budget (RPT <= kMaxRpt).  Anything that still stalls the barrier
// is caught by the bounded poll (NaN rows + HLHGAT_DEVERR_BN_WAIT, never
// numbers from partial statistics).
unsigned g_poll_limit = 1u << 22;

int64_t capacity_of(const void* kernel) {
  static auto* cache = new std::vector<std::pair<const void*, int64_t>>();
  for (const auto& kv : *cache)
    if (kv.first == kernel) return kv.second;
  int dev = 0, cus = 0, occ = 0;
  int64_t c = 0;
  // the share of the chip one barrier grid may take: 1 / HLHGAT_BN_COLOCATE
  // (default 2: two chains' barrier launches resident at once)
  static const int share = [] {
    const char* e = std::getenv("HLHGAT_BN_COLOCATE");
    const int v = e ? std::atoi(e) : 2;
    return v >= 1 && v <= 16 ? v : 2;
  }();
  if (hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, kThreads, 0) == hipSuccess)
    c = (int64_t)occ * cus / share;
  cache->push_back({kernel, c});
  return c;
}

int rpt_bucket(const BnLayout& L) {
  const int64_t need = ceil_div(L.rows_per_part, (int64_t)L.rp);
  if (need > kMaxRpt) return 0;
  for (int r : {2, 4, 8, 16, 32})
    if (need <= r) return r;
  return 0;
}


using GridFn = void (*)(StatsArgs);

GridFn fwd_grid_fn(bool vec, int rpt) {
  switch (rpt * 2 + (vec ? 1 : 0)) {
    case 4: return k_bn_fwd_grid<1, 2>;
    case 5: return k_bn_fwd_grid<4, 2>;
    case 8: return k_bn_fwd_grid<1, 4>;
    case 9: return k_bn_fwd_grid<4, 4>;
    case 16: return k_bn_fwd_grid<1, 8>;
    case 17: return k_bn_fwd_grid<4, 8>;
    case 32: return k_bn_fwd_grid<1, 16>;
    case 33: return k_bn_fwd_grid<4, 16>;
    case 64: return k_bn_fwd_grid<1, 32>;
    case 65: return k_bn_fwd_grid<4, 32>;
    default: return nullptr;
  }
}

// hlhgat_set_bn_produced(1): the rows produced inside the one-launch
// BatchNorm.  Off by default: same-box A/B of the replayed config-2 step
// (tools/ab_step.py, round 4) 2.80 ms with the producer's own launch vs 2.87
// ms produced in the grid-barrier launch -- the gathers lose the parallelism
// of their own wide launch inside the co-resident (<= 256 workgroup) grid.
// Bitwise the same results either way.
bool& bn_produced_flag() {
  static bool v = false;
  return v;
}

GridFn produced_fn(int prod, int rpt) {
  switch (rpt * 4 + prod) {
    case 9: return k_bn_fwd_produced<2, 1>;
    case 10: return k_bn_fwd_produced<2, 2>;
    case 17: return k_bn_fwd_produced<4, 1>;
    case 18: return k_bn_fwd_produced<4, 2>;
    case 33: return k_bn_fwd_produced<8, 1>;
    case 34: return k_bn_fwd_produced<8, 2>;
    case 65: return k_bn_fwd_produced<16, 1>;
    case 66: return k_bn_fwd_produced<16, 2>;
    case 129: return k_bn_fwd_produced<32, 1>;
    case 130: return k_bn_fwd_produced<32, 2>;
    default: return nullptr;
  }
}

// The one-launch kernel for this layout, or nullptr (two launches).
GridFn pick_grid(const BnLayout& L, bool vec) {
  if (!bn_one_launch() || L.parts > kFlatMax) return nullptr;
  const int64_t grid = (int64_t)L.parts * L.tiles;
  const int rpt = rpt_bucket(L);
  GridFn f = rpt ? fwd_grid_fn(vec, rpt) : nullptr;
  const int64_t cap = f ? capacity_of(reinterpret_cast<const void*>(f)) : 0;
  if (!f || grid > 256 || grid > cap) return nullptr;
  return f;
}


}  // namespace


extern "C" int hlhgat_bn_fwd_produced(int mode, const int64_t* edge_index,
                                      const int32_t* inc_rowptr, const int32_t* inc_eids,
                                      int64_t inc_nnz, const float* row_scale, const float* p,
                                      int64_t ldp, float ca, float cb, const float* z,
                                      int64_t ldz, float* x, int64_t ldx, int64_t n,
                                      const int32_t* n_valid, int64_t C, const float* weight,
                                      const float* bias, float* running_mean,
                                      float* running_var, int64_t* num_batches_tracked,
                                      float momentum, float eps, int relu, float* y, int64_t ldy,
                                      float* save_mean, float* save_invstd, void* workspace,
                                      int64_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(mode == HLHGAT_BN_PRODUCE_EDGE_GATHER || mode == HLHGAT_BN_PRODUCE_NODE_INCIDENCE,
                "bn_fwd_produced: bad mode %d", mode);
  HLH_CHECK_ARG(n >= 1 && C >= 1 && C < (1 << 20) && ldx >= C && ldy >= C && ldp >= C &&
                    ldz >= C,
                "bn_fwd_produced: bad sizes n=%lld C=%lld", (long long)n, (long long)C);
  HLH_CHECK_ARG(p && z && x && y && save_mean && save_invstd, "bn_fwd_produced: NULL pointer");
  const bool edge = mode == HLHGAT_BN_PRODUCE_EDGE_GATHER;
  HLH_CHECK_ARG(edge ? edge_index != nullptr
                     : (inc_rowptr && row_scale && (inc_nnz == 0 || inc_eids)),
                "bn_fwd_produced: missing producer arrays");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                "bn_fwd_produced: workspace too small");
  const bool vec = bn_vec_ok(C, {ldx, ldy, ldp, ldz}, {x, y, p, z});
  const BnLayout L = bn_layout(n, C, vec);
  GridFn f = nullptr;
  if (vec && bn_one_launch() && bn_produced_flag() && L.parts <= kFlatMax &&
      L.tiles <= kMaxTiles) {
    const int rpt = rpt_bucket(L);
    f = rpt ? produced_fn(edge ? 1 : 2, rpt) : nullptr;
    const int64_t cap = f ? capacity_of(reinterpret_cast<const void*>(f)) : 0;
    if ((int64_t)L.parts * L.tiles > 256 || (int64_t)L.parts * L.tiles > cap) f = nullptr;
  }
  if (!f) {  // the producer's own launch, then the BatchNorm
    int rc;
    if (edge)
      rc = hlhgat_edge_gather2(edge_index, n, p, ldp, (int)C, nullptr, nullptr, ca, cb, z, ldz, x,
                               ldx, 0, stream);
    else
      rc = hlhgat_poly_step(inc_rowptr, inc_nnz ? inc_eids : nullptr, nullptr, row_scale, n,
                            inc_nnz, nullptr, nullptr, p, ldp, (int)C, z, ldz, nullptr, 0, nullptr,
                            0, 1.f, 0.f, 1.f, 1.f, 0.f, 0.f, x, ldx, stream);
    if (rc != HLHGAT_OK) return rc;
    return hlhgat_bn_fwd_train(x, ldx, n, n_valid, C, weight, bias, running_mean, running_var,
                               num_batches_tracked, momentum, eps, relu, y, ldy, save_mean,
                               save_invstd, workspace, workspace_bytes, stream);
  }
  StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
  s.weight = weight;
  s.bias = bias;
  s.running_mean = running_mean;
  s.running_var = running_var;
  s.nbt = num_batches_tracked;
  s.momentum = momentum;
  s.eps = eps;
  s.save_mean = save_mean;
  s.save_invstd = save_invstd;
  s.out = y;
  s.ldo = ldy;
  s.relu = relu;
  s.poll_limit = g_poll_limit;
  s.err = hlhgat::device_error_word();
  HLH_CHECK_ARG(s.err, "bn_fwd_produced: no device error word (%s)", hlhgat_last_error());
  s.pei = edge_index;
  s.prow = inc_rowptr;
  s.peid = inc_eids;
  s.prs = row_scale;
  s.pp = p;
  s.ldp = ldp;
  s.pz = z;
  s.ldz = ldz;
  s.pca = ca;
  s.pcb = cb;
  s.xw = x;
  ProfScope prof(HLHGAT_PROF_BN_FWD, as_stream(stream), 8.0 * (double)n * C, 0.0);
  launch(f, dim3(L.parts, L.tiles), dim3(kThreads), 0, as_stream(stream), &prof, s);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int64_t hlhgat_bn_workspace_bytes(int64_t n, int64_t C) {
  if (n < 0 || C <= 0) return 0;
  return (int64_t)bn_ws_bytes(n, C);
}

extern "C" int hlhgat_bn_stats_train(const float* x, int64_t ldx, int64_t n,
                                     const int32_t* n_valid, int64_t C, float* running_mean,
                                     float* running_var, int64_t* num_batches_tracked,
                                     float momentum, float eps, float* save_mean,
                                     float* save_invstd, void* workspace,
                                     int64_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && C < (1 << 20) && ldx >= C,
                "bn_stats_train: bad sizes n=%lld C=%lld", (long long)n, (long long)C);
  HLH_CHECK_ARG(x && save_mean && save_invstd, "bn_stats_train: NULL pointer");
  HLH_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                "bn_stats_train: running_mean/var must both be given or both NULL");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                "bn_stats_train: workspace too small");
  const bool vec = bn_vec_ok(C, {ldx}, {x});
  BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_stats_train: C too large");
  StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
  s.running_mean = running_mean;
  s.running_var = running_var;
  s.nbt = num_batches_tracked;
  s.momentum = momentum;
  s.eps = eps;
  s.save_mean = save_mean;
  s.save_invstd = save_invstd;
  hipStream_t st = as_stream(stream);
  dim3 g1(L.parts, L.tiles);
  if (vec)
    launch(k_bn_stats<4>, dim3(g1), dim3(kThreads), 0, st, nullptr, s);
  else
    launch(k_bn_stats<1>, dim3(g1), dim3(kThreads), 0, st, nullptr, s);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_apply(const float* x, int64_t ldx, int64_t n, const int32_t* n_valid,
                               int64_t C, const float* weight, const float* bias,
                               const float* save_mean, const float* save_invstd, int relu,
                               float* y, int64_t ldy, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && C < (1 << 20) && ldx >= C && ldy >= C,
                "bn_apply: bad sizes n=%lld C=%lld", (long long)n, (long long)C);
  HLH_CHECK_ARG(x && y && save_mean && save_invstd, "bn_apply: NULL pointer");
  const bool vec = bn_vec_ok(C, {ldx, ldy}, {x, y});
  BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_apply: C too large");
  ApplyArgs p{n_valid, x, ldx, y, ldy, n, (int)C, save_mean, save_invstd, weight, bias, relu,
              L.tpr, L.rp};
  hipStream_t st = as_stream(stream);
  dim3 g2(apply_grid_x(n, L.rp), L.tiles);
  if (vec)
    launch(k_bn_apply<4>, dim3(g2), dim3(kThreads), 0, st, nullptr, p);
  else
    launch(k_bn_apply<1>, dim3(g2), dim3(kThreads), 0, st, nullptr, p);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_fwd_train(const float* x, int64_t ldx, int64_t n,
                                   const int32_t* n_valid, int64_t C,
                                   const float* weight, const float* bias,
                                   float* running_mean, float* running_var,
                                   int64_t* num_batches_tracked, float momentum,
                                   float eps, int relu, float* y, int64_t ldy,
                                   float* save_mean, float* save_invstd,
                                   void* workspace, int64_t workspace_bytes,
                                   void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && C < (1 << 20) && ldx >= C && ldy >= C,
                "bn_fwd_train: bad sizes n=%lld C=%lld", (long long)n, (long long)C);
  HLH_CHECK_ARG(x && y && save_mean && save_invstd, "bn_fwd_train: NULL pointer");
  HLH_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                "bn_fwd_train: running_mean/var must both be given or both NULL");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                "bn_fwd_train: workspace too small");
  const bool vec = bn_vec_ok(C, {ldx, ldy}, {x, y});
  const BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_fwd_train: C too large");
  // the two-launch path must see the same layout (vector width) to give the
  // same bits: both use bn_vec_ok over x AND y here
  if (GridFn f = pick_grid(L, vec)) {
    StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
    s.weight = weight;
    s.bias = bias;
    s.running_mean = running_mean;
    s.running_var = running_var;
    s.nbt = num_batches_tracked;
    s.momentum = momentum;
    s.eps = eps;
    s.save_mean = save_mean;
    s.save_invstd = save_invstd;
    s.out = y;
    s.ldo = ldy;
    s.relu = relu;
    s.poll_limit = g_poll_limit;
    s.err = hlhgat::device_error_word();
    HLH_CHECK_ARG(s.err, "bn_fwd_train: no device error word (%s)", hlhgat_last_error());
    // algorithmic bytes: x read once, y written once
    ProfScope prof(HLHGAT_PROF_BN_FWD, as_stream(stream), 8.0 * (double)n * C, 0.0);
    launch(f, dim3(L.parts, L.tiles), dim3(kThreads), 0, as_stream(stream), &prof, s);
    HLH_CHECK_LAUNCH();
    return HLHGAT_OK;
  }
  // two launches on the same layout
  StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
  s.running_mean = running_mean;
  s.running_var = running_var;
  s.nbt = num_batches_tracked;
  s.momentum = momentum;
  s.eps = eps;
  s.save_mean = save_mean;
  s.save_invstd = save_invstd;
  hipStream_t st = as_stream(stream);
  dim3 g1(L.parts, L.tiles);
  if (vec)
    launch(k_bn_stats<4>, dim3(g1), dim3(kThreads), 0, st, nullptr, s);
  else
    launch(k_bn_stats<1>, dim3(g1), dim3(kThreads), 0, st, nullptr, s);
  HLH_CHECK_LAUNCH();
  ApplyArgs p{n_valid, x, ldx, y, ldy, n, (int)C, save_mean, save_invstd, weight, bias, relu,
              L.tpr, L.rp};
  dim3 g2(apply_grid_x(n, L.rp), L.tiles);
  if (vec)
    launch(k_bn_apply<4>, dim3(g2), dim3(kThreads), 0, st, nullptr, p);
  else
    launch(k_bn_apply<1>, dim3(g2), dim3(kThreads), 0, st, nullptr, p);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// Projection + BatchNorm (+ ReLU) forward (see k_proj_bn_fwd): one launch where
// the projection's grid fits co-resident, else hlhgat_proj_fwd then
// hlhgat_bn_fwd_train on x.
extern "C" int hlhgat_proj_bn_fwd(int nblocks, const float* const* A, const int64_t* lda,
                                  const float* const* W, const int64_t* ldw, const int64_t* kb,
                                  int64_t M, int64_t N, const float* bias, float* x, int64_t ldx,
                                  const int32_t* n_valid, const float* bn_weight,
                                  const float* bn_bias, float* running_mean, float* running_var,
                                  int64_t* num_batches_tracked, float momentum, float eps,
                                  int relu, float* y, int64_t ldy, float* save_mean,
                                  float* save_invstd, void* workspace, int64_t workspace_bytes,
                                  void* stream) {
  HLH_CHECK_ARG(nblocks >= 1 && nblocks <= MAXB, "proj_bn_fwd: nblocks=%d", nblocks);
  HLH_CHECK_ARG(M >= 1 && N >= 1 && N < (1 << 20) && ldx >= N && ldy >= N,
                "proj_bn_fwd: bad sizes M=%lld N=%lld", (long long)M, (long long)N);
  HLH_CHECK_ARG(x && y && save_mean && save_invstd, "proj_bn_fwd: NULL pointer");
  HLH_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                "proj_bn_fwd: running_mean/var must both be given or both NULL");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(M, N),
                "proj_bn_fwd: workspace too small");
  bool vec = true;
  int64_t ktot = 0;
  for (int b = 0; b < nblocks; ++b) {
    HLH_CHECK_ARG(A[b] && W[b] && kb[b] > 0 && lda[b] >= kb[b] && ldw[b] >= kb[b],
                  "proj_bn_fwd: bad block %d", b);
    vec = vec && aligned16(A[b]) && aligned16(W[b]) && lda[b] % 4 == 0 && ldw[b] % 4 == 0 &&
          kb[b] % 4 == 0;
    ktot += kb[b];
  }
  const unsigned gx = (unsigned)ceil_div(M, (int64_t)64), gy = (unsigned)(N / 64);
  bool fused = proj_bn_fused_flag() && vec && N % 64 == 0 && gy <= (unsigned)kMaxTiles &&
               gx <= (unsigned)kMaxParts;
  if (fused) {
    const int64_t cap = capacity_of(reinterpret_cast<const void*>(k_proj_bn_fwd));
    fused = (int64_t)gx * gy <= cap;
  }
  if (!fused) {
    const int rc = hlhgat_proj_fwd(nblocks, A, lda, W, ldw, kb, M, N, bias, x, ldx, 0, stream);
    if (rc != HLHGAT_OK) return rc;
    return hlhgat_bn_fwd_train(x, ldx, M, n_valid, N, bn_weight, bn_bias, running_mean,
                               running_var, num_batches_tracked, momentum, eps, relu, y, ldy,
                               save_mean, save_invstd, workspace, workspace_bytes, stream);
  }
  ProjBnArgs a{};
  a.g.nb = nblocks;
  a.g.M = M;
  a.g.N = (int)N;
  a.g.bias = bias;
  a.g.C = x;
  a.g.ldc = ldx;
  for (int b = 0; b < nblocks; ++b) {
    a.g.A[b] = A[b];
    a.g.W[b] = W[b];
    a.g.lda[b] = lda[b];
    a.g.ldw[b] = ldw[b];
    a.g.kb[b] = (int)kb[b];
  }
  BnWs w = carve(workspace, M, N);
  StatsArgs& s = a.s;
  s.nvalid = n_valid;
  s.n = M;
  s.C = (int)N;
  s.part = w.part;
  s.gpart = w.gpart;
  s.count = w.count;
  s.weight = bn_weight;
  s.bias = bn_bias;
  s.running_mean = running_mean;
  s.running_var = running_var;
  s.nbt = num_batches_tracked;
  s.momentum = momentum;
  s.eps = eps;
  s.save_mean = save_mean;
  s.save_invstd = save_invstd;
  s.out = y;
  s.ldo = ldy;
  s.relu = relu;
  s.poll_limit = g_poll_limit;
  s.err = hlhgat::device_error_word();
  HLH_CHECK_ARG(s.err, "proj_bn_fwd: no device error word (%s)", hlhgat_last_error());
  // algorithmic: A read once, x and y written once; flops of the projection
  const double flops = 2.0 * (double)M * (double)N * (double)ktot;
  const double bytes = 4.0 * (double)M * ((double)ktot + 2.0 * (double)N);
  hipStream_t st = as_stream(stream);
  ProfScope prof(HLHGAT_PROF_PROJ_BN, st, bytes, flops);
  launch(k_proj_bn_fwd, dim3(gx, gy), dim3(kThreads), 0, st, &prof, a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_set_proj_bn_fused(int on) {
  proj_bn_fused_flag() = on != 0;
  return HLHGAT_OK;
}

extern "C" int hlhgat_proj_bn_fused_capacity(int64_t* out) {
  HLH_CHECK_ARG(out, "proj_bn_fused_capacity: NULL pointer");
  *out = capacity_of(reinterpret_cast<const void*>(k_proj_bn_fwd));
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_bwd_train(const float* x, int64_t ldx, const float* y,
                                   int64_t ldy, const float* dy, int64_t lddy,
                                   int64_t n, const int32_t* n_valid, int64_t C,
                                   const float* weight,
                                   const float* save_mean, const float* save_invstd,
                                   float* dx, int64_t lddx, float* dweight,
                                   float* dbias, void* workspace,
                                   int64_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && ldx >= C && lddy >= C && lddx >= C && (!y || ldy >= C),
                "bn_bwd_train: bad sizes");
  HLH_CHECK_ARG(x && dy && dx && save_mean && save_invstd, "bn_bwd_train: NULL pointer");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                "bn_bwd_train: workspace too small");
  const bool vec = bn_vec_ok(C, {ldx, lddy, lddx, y ? ldy : 4}, {x, y, dy, dx});
  BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_bwd_train: C too large");
  BnWs w = carve(workspace, n, C);
  StatsArgs s = stats_args(L, w, x, ldx, n, n_valid, C);
  s.y = y;
  s.ldy = ldy;
  s.dy = dy;
  s.lddy = lddy;
  s.weight = weight;
  s.save_mean = const_cast<float*>(save_mean);
  s.save_invstd = const_cast<float*>(save_invstd);
  s.coef = w.coef;
  s.dweight = dweight;
  s.dbias = dbias;
  hipStream_t st = as_stream(stream);
  dim3 g1(L.parts, L.tiles);
  {  // algorithmic bytes of the reduction: x, dy (and y for the ReLU mask) read once
    ProfScope prof(HLHGAT_PROF_BN_BWD, st, (y ? 12.0 : 8.0) * (double)n * C, 0.0);
    if (vec)
      launch(k_bn_bwd_reduce<4>, g1, dim3(kThreads), 0, st, &prof, s);
    else
      launch(k_bn_bwd_reduce<1>, g1, dim3(kThreads), 0, st, &prof, s);
  }
  HLH_CHECK_LAUNCH();
  BwdApplyArgs p{n_valid, x, ldx, y, ldy, dy, lddy, dx, lddx, n, (int)C, w.coef, save_mean,
                 L.tpr, L.rp};
  dim3 g2(apply_grid_x(n, L.rp), L.tiles);
  if (vec)
    launch(k_bn_bwd_apply<4>, dim3(g2), dim3(kThreads), 0, st, nullptr, p);
  else
    launch(k_bn_bwd_apply<1>, dim3(g2), dim3(kThreads), 0, st, nullptr, p);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_bwd_reduce(const float* x, int64_t ldx, const float* y, int64_t ldy,
                                    const float* dy, int64_t lddy, int64_t n,
                                    const int32_t* n_valid, int64_t C, const float* weight,
                                    const float* save_mean, const float* save_invstd,
                                    float* coef, float* dweight, float* dbias, void* workspace,
                                    int64_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && ldx >= C && lddy >= C && (!y || ldy >= C),
                "bn_bwd_reduce: bad sizes");
  HLH_CHECK_ARG(x && dy && coef && save_mean && save_invstd, "bn_bwd_reduce: NULL pointer");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                "bn_bwd_reduce: workspace too small");
  // the layout hlhgat_bn_bwd_train picks for an aligned dx: the same bits
  const bool vec = bn_vec_ok(C, {ldx, lddy, y ? ldy : 4}, {x, y, dy});
  BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_bwd_reduce: C too large");
  BnWs w = carve(workspace, n, C);
  StatsArgs s = stats_args(L, w, x, ldx, n, n_valid, C);
  s.y = y;
  s.ldy = ldy;
  s.dy = dy;
  s.lddy = lddy;
  s.weight = weight;
  s.save_mean = const_cast<float*>(save_mean);
  s.save_invstd = const_cast<float*>(save_invstd);
  s.coef = coef;
  s.dweight = dweight;
  s.dbias = dbias;
  hipStream_t st = as_stream(stream);
  ProfScope prof(HLHGAT_PROF_BN_BWD, st, (y ? 12.0 : 8.0) * (double)n * C, 0.0);
  if (vec)
    launch(k_bn_bwd_reduce<4>, dim3(L.parts, L.tiles), dim3(kThreads), 0, st, &prof, s);
  else
    launch(k_bn_bwd_reduce<1>, dim3(L.parts, L.tiles), dim3(kThreads), 0, st, &prof, s);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// ---------------------------------------------------------------------------
// SyncBatchNorm: sums -> (caller all-gathers [world][2C+1]) -> apply
// ---------------------------------------------------------------------------
extern "C" int64_t hlhgat_bn_sums_len(int64_t C) { return C > 0 ? 2 * C + 1 : 0; }

extern "C" int hlhgat_bn_sums_fwd(const float* x, int64_t ldx, const float* y, int64_t ldy,
                                  int64_t n, const int32_t* n_valid, int64_t C, double* sums,
                                  void* workspace, int64_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && C < (1 << 20) && ldx >= C && (!y || ldy >= C),
                "bn_sums_fwd: bad sizes n=%lld C=%lld", (long long)n, (long long)C);
  HLH_CHECK_ARG(x && sums, "bn_sums_fwd: NULL pointer");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                "bn_sums_fwd: workspace too small");
  // the layout (hence the partial order) of hlhgat_bn_fwd_train over (x, y)
  const bool vec = bn_vec_ok(C, {ldx, y ? ldy : 4}, {x, y});
  const BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_sums_fwd: C too large");
  StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
  s.sums_out = sums;
  dim3 g1(L.parts, L.tiles);
  if (vec)
    launch(k_bn_stats<4>, dim3(g1), dim3(kThreads), 0, as_stream(stream), nullptr, s);
  else
    launch(k_bn_stats<1>, dim3(g1), dim3(kThreads), 0, as_stream(stream), nullptr, s);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_sync_fwd_apply(const float* x, int64_t ldx, int64_t n,
                                        const int32_t* n_valid, int64_t C,
                                        const double* gathered, int world, const float* weight,
                                        const float* bias, float* running_mean,
                                        float* running_var, int64_t* num_batches_tracked,
                                        float momentum, float eps, int relu, float* y,
                                        int64_t ldy, float* save_mean, float* save_invstd,
                                        void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && C < (1 << 20) && ldx >= C && ldy >= C && world >= 1,
                "bn_sync_fwd_apply: bad sizes n=%lld C=%lld world=%d", (long long)n,
                (long long)C, world);
  HLH_CHECK_ARG(x && y && gathered && save_mean && save_invstd, "bn_sync_fwd_apply: NULL pointer");
  HLH_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                "bn_sync_fwd_apply: running_mean/var must both be given or both NULL");
  const bool vec = bn_vec_ok(C, {ldx, ldy}, {x, y});
  const BnLayout L = bn_layout(n, C, vec);
  SyncArgs a{};
  a.nvalid = n_valid;
  a.x = x;
  a.ldx = ldx;
  a.out = y;
  a.ldo = ldy;
  a.n = n;
  a.C = (int)C;
  a.tpr = L.tpr;
  a.rp = L.rp;
  a.gathered = gathered;
  a.world = world;
  a.weight = weight;
  a.bias = bias;
  a.running_mean = running_mean;
  a.running_var = running_var;
  a.nbt = num_batches_tracked;
  a.momentum = momentum;
  a.eps = eps;
  a.save_mean = save_mean;
  a.save_invstd = save_invstd;
  a.relu = relu;
  dim3 g2(apply_grid_x(n, L.rp), L.tiles);
  if (vec)
    launch(k_bn_sync_apply<4>, dim3(g2), dim3(kThreads), 0, as_stream(stream), nullptr, a);
  else
    launch(k_bn_sync_apply<1>, dim3(g2), dim3(kThreads), 0, as_stream(stream), nullptr, a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_sums_bwd(const float* x, int64_t ldx, const float* y, int64_t ldy,
                                  const float* dy, int64_t lddy, float* dx_layout,
                                  int64_t lddx, int64_t n, const int32_t* n_valid, int64_t C,
                                  const float* save_mean, const float* save_invstd,
                                  double* sums, float* dweight, float* dbias, void* workspace,
                                  int64_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && ldx >= C && lddy >= C && (!y || ldy >= C) &&
                    (!dx_layout || lddx >= C),
                "bn_sums_bwd: bad sizes");
  HLH_CHECK_ARG(x && dy && sums && save_mean && save_invstd, "bn_sums_bwd: NULL pointer");
  HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                "bn_sums_bwd: workspace too small");
  // the layout of hlhgat_bn_bwd_train over (x, y, dy, dx)
  const bool vec = bn_vec_ok(C, {ldx, lddy, dx_layout ? lddx : 4, y ? ldy : 4},
                             {x, y, dy, dx_layout});
  const BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_sums_bwd: C too large");
  StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
  s.y = y;
  s.ldy = ldy;
  s.dy = dy;
  s.lddy = lddy;
  s.save_mean = const_cast<float*>(save_mean);
  s.save_invstd = const_cast<float*>(save_invstd);
  s.dweight = dweight;
  s.dbias = dbias;
  s.sums_out = sums;
  dim3 g1(L.parts, L.tiles);
  if (vec)
    launch(k_bn_bwd_reduce<4>, dim3(g1), dim3(kThreads), 0, as_stream(stream), nullptr, s);
  else
    launch(k_bn_bwd_reduce<1>, dim3(g1), dim3(kThreads), 0, as_stream(stream), nullptr, s);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_sync_bwd_apply(const float* x, int64_t ldx, const float* y,
                                        int64_t ldy, const float* dy, int64_t lddy, int64_t n,
                                        const int32_t* n_valid, int64_t C, const float* weight,
                                        const float* save_mean, const float* save_invstd,
                                        const double* gathered, int world, float* dx,
                                        int64_t lddx, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && ldx >= C && lddy >= C && lddx >= C && (!y || ldy >= C) &&
                    world >= 1,
                "bn_sync_bwd_apply: bad sizes");
  HLH_CHECK_ARG(x && dy && dx && gathered && save_mean && save_invstd,
                "bn_sync_bwd_apply: NULL pointer");
  const bool vec = bn_vec_ok(C, {ldx, lddy, lddx, y ? ldy : 4}, {x, y, dy, dx});
  const BnLayout L = bn_layout(n, C, vec);
  SyncArgs a{};
  a.nvalid = n_valid;
  a.x = x;
  a.ldx = ldx;
  a.y = y;
  a.ldy = ldy;
  a.dy = dy;
  a.lddy = lddy;
  a.out = dx;
  a.ldo = lddx;
  a.n = n;
  a.C = (int)C;
  a.tpr = L.tpr;
  a.rp = L.rp;
  a.gathered = gathered;
  a.world = world;
  a.weight = weight;
  a.save_mean = const_cast<float*>(save_mean);
  a.save_invstd = const_cast<float*>(save_invstd);
  dim3 g2(apply_grid_x(n, L.rp), L.tiles);
  if (vec)
    launch(k_bn_sync_bwd_apply<4>, dim3(g2), dim3(kThreads), 0, as_stream(stream), nullptr, a);
  else
    launch(k_bn_sync_bwd_apply<1>, dim3(g2), dim3(kThreads), 0, as_stream(stream), nullptr, a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_set_bn_produced(int on) {
  bn_produced_flag() = on != 0;
  return HLHGAT_OK;
}

extern "C" int hlhgat_set_bn_one_launch(int on) {
  bn_one_launch_flag() = on != 0;
  return HLHGAT_OK;
}

extern "C" int hlhgat_get_bn_one_launch(void) { return bn_one_launch_flag() ? 1 : 0; }

extern "C" int hlhgat_set_bn_poll_limit(unsigned limit) {
  g_poll_limit = limit;
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_wait_timeouts(unsigned* out) {
  HLH_CHECK_ARG(out, "bn_wait_timeouts: NULL pointer");
  HLH_CHECK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bn_wait_timeouts), sizeof(unsigned)));
  return HLHGAT_OK;
}
