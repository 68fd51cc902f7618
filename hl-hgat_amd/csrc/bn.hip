// Training-mode BatchNorm1d (+ optional fused ReLU) for the HL blocks.
//
// Every HL block is HodgeLaguerreConv -> gnn.BatchNorm -> ReLU -> Dropout
// (lib/Hodge_ST_Model.py:556-566) and every NodeEdgeInt value MLP is
// Linear -> BatchNorm1d -> ReLU twice (lib/Hodge_Cheb_Conv.py:276-289), so
// each conv output passes through a batch-statistics reduction over all
// simplices.  Two launches per direction:
//   fwd: k_bn_stats  — per-workgroup column partials (fp64 sum, sum of squares)
//                      and, in the LAST workgroup to arrive, the final mean /
//                      invstd and the running-stat update (deterministic: the
//                      last arriver sums the partials in workgroup order);
//        k_bn_apply  — y = relu?((x - mean) * s + bias).
//        (default: k_bn_train_fused, both in ONE launch when the grid is
//        provably co-resident; see hlhgat_bn_fwd_train)
//   bwd: k_bn_bwd_reduce — partials of sum(g) and sum(g*(x-mean)), g = dy *
//                      [y > 0]; the last arriver forms dweight, dbias and the
//                      per-channel coefficients of dx;
//        k_bn_bwd_apply  — dx = a*g + b*(x - mean) + c (centred: no cancellation).
// Inter-workgroup hand-off follows MI355X_MICROARCH.md / cdna_hip_programming.md
// Guideline 16: plain stores, every wave's vmcnt(0), barrier, lane-0 agent
// release fence, relaxed agent atomic ticket; the last arriver issues an
// agent acquire fence before reading the partials.
#include "common.h"

#include <cstdlib>

using namespace hlhgat;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxParts = 512;
constexpr int kGroup = 16;                        // partitions per first-level group
constexpr int kMaxGroups = kMaxParts / kGroup;
constexpr int kMaxTiles = 1024;
constexpr int kFlagBase = kMaxTiles * (1 + kMaxGroups);  // per tile: top + group counters
// + per tile: the one-launch forward's "statistics ready" flag and leave counter
constexpr int kCounters = kFlagBase + 2 * kMaxTiles;
constexpr int APPLY_RPT = 2;  // rows per thread in the elementwise apply kernels

struct BnLayout {
  int v;       // floats per thread (4 or 1)
  int tpr;     // threads per row within a column tile
  int rp;      // rows per pass (kThreads / tpr)
  int tile_c;  // columns per tile (tpr * v)
  int tiles;   // column tiles
  int parts;   // row partitions (grid.x)
  int64_t rows_per_part;
};

// Row partitions of the statistics pass: each partition is one workgroup
// whose loads are all in flight within a couple of round trips.  The
// partials are combined by a two-level last-arriver tree (groups of kGroup
// partitions, then the groups), so many thin partitions cost two short tails
// instead of one long one.  In the ZINC step 64 partitions measured best
// (256: 264k -> 251k graphs/s; more workgroups crowd the concurrent chain).
// HLHGAT_BN_PARTS overrides (A/B measurements).
// Larger batches (config 3 / 5 heads: 1.4e5-2e5 rows) get one partition per
// 512 rows (up to kMaxParts): 64 workgroups leave most of the 256 CUs idle
// there (k_bn_bwd_reduce ran at ~1 TB/s, profiles/r01_h_*_head_kernel_stats.md).
// HLHGAT_BN_ONE_LAUNCH=0: BatchNorm forward statistics and apply as two
// launches instead of k_bn_train_fused (bitwise the same results).  Same-box
// A/B at the ZINC step with 128 partitions: 288.6k -> 291.1k graphs/s over
// five runs each (every one-launch run above every two-launch run; with 64
// partitions it was neutral).
bool& bn_one_launch_flag() {
  static bool v = [] {
    const char* e = getenv("HLHGAT_BN_ONE_LAUNCH");
    return !(e && e[0] == '0');
  }();
  return v;
}
bool bn_one_launch() { return bn_one_launch_flag(); }

int64_t bn_parts(int64_t n) {
  static int64_t fixed = [] {
    const char* e = getenv("HLHGAT_BN_PARTS");
    return e ? atoll(e) : (int64_t)0;
  }();
  // >= 128 partitions (same-box A/B at the ZINC step, n ~ 25k: 64 -> 281.8k,
  // 128 -> 287.2k, 256 -> 286.1k, 32 -> 265.8k graphs/s), ~512 rows each above
  int64_t p = fixed > 0 ? fixed : std::max<int64_t>(128, ceil_div(n, (int64_t)512));
  return p < 1 ? 1 : (p > kMaxParts ? kMaxParts : p);
}

BnLayout bn_layout(int64_t n, int64_t C, bool vec, int nt = kThreads) {
  BnLayout L;
  L.v = vec ? 4 : 1;
  int lanes = (int)ceil_div(C, L.v);
  L.tpr = next_pow2(lanes);
  if (L.tpr > kThreads / L.v) L.tpr = kThreads / L.v;  // tile_c <= kThreads
  L.rp = nt / L.tpr;
  L.tile_c = L.tpr * L.v;
  L.tiles = (int)ceil_div(C, L.tile_c);
  // <= kMaxParts row partitions per column tile (fat partitions keep the
  // last arriver's reduction to one batch of loads per thread)
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
  // one-launch forward: poll limit of the statistics wait, host-visible error word
  unsigned poll_limit;
  unsigned* err;
};

// Partials are handed to the last-arriving workgroup WRITE-THROUGH: 8-byte
// agent-scope atomic stores (global_store_dwordx2 sc1) drained by every
// storing wave, read back with sc1 loads -- no release fence (buffer_wbl2,
// which writes back the XCD L2's dirty lines: the freshly written BN input
// and everything else the concurrent stream left dirty, 1.7-6.5 us per
// workgroup) and no acquire fence (cdna_hip_programming.md Guideline 16 R1;
// MI355X_MICROARCH.md visibility table).
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// wait timeouts of the one-launch BatchNorm (hlhgat_bn_wait_timeouts)
__device__ unsigned g_bn_wait_timeouts = 0;

// A waiting workgroup that gives up (poll limit reached) must not normalise
// with stale statistics: it writes NaN into its rows, counts the timeout and
// raises HLHGAT_DEVERR_BN_WAIT in the host-visible error word
// (hlhgat_device_errors), which hlhgat.train.TrainStep, the bench and
// hlhgat.ops.check_device_errors turn into a Python exception.
__device__ __forceinline__ void report_wait_timeout(unsigned* err) {
  __hip_atomic_fetch_add(&g_bn_wait_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (err) __hip_atomic_store(err, (unsigned)HLHGAT_DEVERR_BN_WAIT, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_SYSTEM);
}

// Bounded wait of a non-finalising workgroup for its tile's statistics flag;
// poll_limit == 0 (test hook) gives up at once.  Returns false on timeout.
__device__ __forceinline__ bool wait_flag(unsigned* flag, unsigned poll_limit, unsigned* err) {
  __shared__ unsigned s_ok;
  if (threadIdx.x == 0) {
    unsigned ok = 0;
    if (poll_limit > 0) {
      for (unsigned it = 0; it < poll_limit; ++it) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
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

typedef __attribute__((address_space(1))) unsigned gu32_t;
__device__ __forceinline__ void st_wt32(float* p, float v) {
  __hip_atomic_store((gu32_t*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt32(const float* p) {
  return __uint_as_float(
      __hip_atomic_load((gu32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Signal arrival; returns true in the last workgroup of this column tile.
// Every wave has drained its write-through partial stores (vmcnt(0)) before
// the barrier; ONE lane adds to the counter; the workgroup whose add returned
// total-1 reads the partials (sc1 loads) after the second barrier.
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

// Block-level column partials: threads (row group rg, column lane cl) hold V
// columns each; reduce over the rp row groups through LDS in fixed order.
template <int V, int NT>
__device__ __forceinline__ void write_partials(double (&s0)[V], double (&s1)[V],
                                               const StatsArgs& a, int c0) {
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
      double* dst = a.part + ((int64_t)blockIdx.x * a.C + c) * 2;
      st_wt(dst, u0);
      st_wt(dst + 1, u1);
    }
  }
}

// Sum of partials [first, first+count) of src ([*][C][2]) for the tile's
// columns: all 256 threads take part (column t % tile_c, partial group
// t / tile_c, loads in batches of 16), groups combined in fixed order through
// LDS -> deterministic.  Result in out0/out1[0 .. tile_c).
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

// Two-level last-arriver tree over the `parts` partials of this column tile:
// the last workgroup of each group of kGroup partitions sums its group, the
// last group sums the group partials.  Returns true (sums in out0/out1) in
// the one workgroup that finalises; fixed summation order at both levels.
template <int NT>
__device__ __forceinline__ bool tree_reduce(const StatsArgs& a, int c0, int tile_c,
                                            double* out0, double* out1) {
  const int tile = blockIdx.y;
  const int g = blockIdx.x / kGroup;
  const int ng = (a.parts + kGroup - 1) / kGroup;
  const int first = g * kGroup;
  const int cnt = a.parts - first < kGroup ? a.parts - first : kGroup;
  if (!arrive_last(a.count + kMaxTiles + tile * kMaxGroups + g, (unsigned)cnt)) return false;
  reduce_range<NT>(a.part, first, cnt, a, c0, tile_c, out0, out1);
  if (ng == 1) return true;
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

// Statistics (and, APPLY, the normalisation in the same launch): with APPLY
// the finalising workgroup of a column tile publishes mean / invstd write-
// through and raises the tile's flag; the other workgroups of the tile (all
// co-resident: parts x tiles <= a few hundred workgroups of 256 threads) wait
// for it, normalise the rows they summed, and the last to leave resets the
// flag.  The wait is bounded so a stalled launch cannot hang the GPU.
template <int V, int NT, bool APPLY>
__device__ __forceinline__ void bn_stats_body(const StatsArgs& a, const ApplyArgs& p) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c0 = blockIdx.y * a.tpr * V;
  const int c = c0 + cl * V;
  const int64_t r_lo = (int64_t)blockIdx.x * a.rows_per_part;
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
  write_partials<V, NT>(s0, s1, a, c0);
  // the finalising workgroup of this column tile: finalise its columns
  __shared__ double sum0[kThreads], sum1[kThreads];
  const int tile_c = a.tpr * V;
  const bool fin = tree_reduce<NT>(a, c0, tile_c, sum0, sum1);
  if (!APPLY && !fin) return;
  if (fin) {
    for (int t = threadIdx.x; t < tile_c; t += NT) {
      const int cc = c0 + t;
      if (cc >= a.C) continue;
      const double u0 = sum0[t], u1 = sum1[t];
      const double nn = (double)(n_eff > 0 ? n_eff : 1);
      const double mean = u0 / nn;
      double var = u1 / nn - mean * mean;
      if (var < 0.0) var = 0.0;
      const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
      if (APPLY) {
        st_wt32(&a.save_mean[cc], (float)mean);
        st_wt32(&a.save_invstd[cc], invstd);
      } else {
        a.save_mean[cc] = (float)mean;
        a.save_invstd[cc] = invstd;
      }
      if (a.running_mean) {
        const double unb = n_eff > 1 ? var * nn / (nn - 1.0) : var;
        a.running_mean[cc] = (1.f - a.momentum) * a.running_mean[cc] + a.momentum * (float)mean;
        a.running_var[cc] = (1.f - a.momentum) * a.running_var[cc] + a.momentum * (float)unb;
      }
    }
    if (a.nbt && blockIdx.y == 0 && threadIdx.x == 0) a.nbt[0] += 1;
  }
  if (!APPLY) return;
  unsigned* flag = a.count + kFlagBase + blockIdx.y;
  unsigned* leave = flag + kMaxTiles;
  if (fin) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // a timed-out workgroup poisons its rows (NaN) instead of applying stale statistics
  const bool ok = fin || wait_flag(flag, a.poll_limit, a.err);
  if (c < a.C) {
    float sc[V], mu[V], sh[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const float w = p.weight ? p.weight[c + v] : 1.f;
      sc[v] = ok ? w * ld_wt32(&p.invstd[c + v]) : __builtin_nanf("");
      mu[v] = ok ? ld_wt32(&p.mean[c + v]) : __builtin_nanf("");
      sh[v] = p.bias ? p.bias[c + v] : 0.f;
    }
    int64_t r_end = r_lo + a.rows_per_part;
    if (r_end > a.n) r_end = a.n;
    auto out = [&](int64_t r, vt xv) {
      vt o;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float z = (vget(xv, v) - mu[v]) * sc[v] + sh[v];
        vget(o, v) = r >= n_eff ? 0.f : ((p.relu && z < 0.f) ? 0.f : z);  // NaN passes
      }
      vstore<V>(p.y + r * p.ldy + c, o);
    };
    int64_t r = r_lo + rg;
    for (; r + 7 * a.rp < r_end; r += 8 * a.rp) {  // 8 rows in flight
      vt x4[8] = {};
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t rr = r + u * a.rp;
        if (rr < n_eff) x4[u] = vload<V>(a.x + rr * a.ldx + c);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) out(r + u * a.rp, x4[u]);
    }
    for (; r < r_end; r += a.rp) {
      vt xv{};
      if (r < n_eff) xv = vload<V>(a.x + r * a.ldx + c);
      out(r, xv);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(leave, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {  // every workgroup of the tile has read the flag
      __hip_atomic_store(leave, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int V, int NT>
__global__ __launch_bounds__(NT) void k_bn_stats(StatsArgs a) {
  bn_stats_body<V, NT, false>(a, ApplyArgs{});
}

template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_train_fused(StatsArgs a, ApplyArgs p) {
  bn_stats_body<V, kThreads, true>(a, p);
}


template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_apply(ApplyArgs a) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c = blockIdx.y * a.tpr * V + cl * V;
  if (c >= a.C) return;
  float s[V], m[V], t[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const float w = a.weight ? a.weight[c + v] : 1.f;
    const float b = a.bias ? a.bias[c + v] : 0.f;
    s[v] = w * a.invstd[c + v];
    m[v] = a.mean[c + v];
    t[v] = b;
  }
  // APPLY_RPT rows per thread, all loads issued before any store
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
    vstore<V>(a.y + r * a.ldy + c, o);
  }
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

// Backward statistics: partials of sum(g), sum(g (x - mean)); the finalising
// workgroup of a column tile forms dweight, dbias and dx's coefficients.
template <int V, int NT>
__device__ __forceinline__ void bn_bwd_body(const StatsArgs& a) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c0 = blockIdx.y * a.tpr * V;
  const int c = c0 + cl * V;
  const int64_t r_lo = (int64_t)blockIdx.x * a.rows_per_part;
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
  write_partials<V, NT>(s0, s1, a, c0);
  __shared__ double sum0[kThreads], sum1[kThreads];
  const int tile_c = a.tpr * V;
  const bool fin = tree_reduce<NT>(a, c0, tile_c, sum0, sum1);
  if (!fin) return;
  for (int t = threadIdx.x; t < tile_c; t += NT) {
    const int cc = c0 + t;
    if (cc >= a.C) continue;
    const double sg = sum0[t], sgx = sum1[t];
    const double is = (double)a.save_invstd[cc];
    const double w = a.weight ? (double)a.weight[cc] : 1.0;
    const double nn = (double)(n_eff > 0 ? n_eff : 1);
    if (a.dweight) a.dweight[cc] = (float)(sgx * is);
    if (a.dbias) a.dbias[cc] = (float)sg;
    // dx = w*is*(g - sg/n - (x-mean)*is^2*sgx/n) = A*g + B*(x-mean) + Cc: the
    // centred form, as torch evaluates it -- B*x + (Cc - B*mean) cancels
    // catastrophically when a channel's variance is small against its mean
    const double A = w * is;
    const double B = -w * is * is * is * sgx / nn;
    const double Cc = -w * is * sg / nn;
    a.coef[cc] = (float)A;
    a.coef[a.C + cc] = (float)B;
    a.coef[2 * a.C + cc] = (float)Cc;
  }
}
template <int V, int NT>
__global__ __launch_bounds__(NT) void k_bn_bwd_reduce(StatsArgs a) {
  bn_bwd_body<V, NT>(a);
}


template <int V>
__global__ __launch_bounds__(kThreads) void k_bn_bwd_apply(BwdApplyArgs a) {
  using vt = typename VecT<V>::type;
  const int cl = threadIdx.x % a.tpr;
  const int rg = threadIdx.x / a.tpr;
  const int c = blockIdx.y * a.tpr * V + cl * V;
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
    vstore<V>(a.dx + r * a.lddx + c, o);
  }
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

// --- one-launch forward: co-residency and the poll limit -------------------
// k_bn_train_fused's waiting workgroups need their tile's finalising
// workgroup to be resident at the same time.  The launch is used only when
// the whole grid fits in a QUARTER of the chip's resident-workgroup capacity
// (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs), so the node / edge /
// interaction streams each running one such launch still leave room; and it
// is capped at 256 workgroups.  Anything that still stalls a wait is caught
// by the bounded poll (NaN rows + HLHGAT_DEVERR_BN_WAIT, never stale numbers).
unsigned g_poll_limit = 1u << 22;

int64_t fused_capacity(bool vec) {
  static int64_t cap[2] = {-1, -1};
  int64_t& c = cap[vec ? 1 : 0];
  if (c >= 0) return c;
  int dev = 0, cus = 0, occ = 0;
  c = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return c;
  hipError_t e = vec ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                           &occ, reinterpret_cast<const void*>(&k_bn_train_fused<4>), kThreads, 0)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                           &occ, reinterpret_cast<const void*>(&k_bn_train_fused<1>), kThreads, 0);
  if (e != hipSuccess) return c;
  c = (int64_t)occ * cus / 4;
  return c;
}

}  // namespace

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
    k_bn_stats<4, kThreads><<<g1, kThreads, 0, st>>>(s);
  else
    k_bn_stats<1, kThreads><<<g1, kThreads, 0, st>>>(s);
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
    k_bn_apply<4><<<g2, kThreads, 0, st>>>(p);
  else
    k_bn_apply<1><<<g2, kThreads, 0, st>>>(p);
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
  HLH_CHECK_ARG(y, "bn_fwd_train: NULL pointer");
  const bool vec = bn_vec_ok(C, {ldx}, {x});
  const BnLayout L = bn_layout(n, C, vec);
  const int64_t grid = (int64_t)L.parts * L.tiles;
  if (bn_one_launch() && grid <= 256 && grid <= fused_capacity(vec) &&
      vec == bn_vec_ok(C, {ldx, ldy}, {x, y})) {
    // statistics and normalisation in one launch (k_bn_train_fused)
    HLH_CHECK_ARG(x && save_mean && save_invstd, "bn_fwd_train: NULL pointer");
    HLH_CHECK_ARG((running_mean == nullptr) == (running_var == nullptr),
                  "bn_fwd_train: running_mean/var must both be given or both NULL");
    HLH_CHECK_ARG(workspace && workspace_bytes >= (int64_t)bn_ws_bytes(n, C),
                  "bn_fwd_train: workspace too small");
    HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_fwd_train: C too large");
    StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
    s.running_mean = running_mean;
    s.running_var = running_var;
    s.nbt = num_batches_tracked;
    s.momentum = momentum;
    s.eps = eps;
    s.save_mean = save_mean;
    s.save_invstd = save_invstd;
    s.poll_limit = g_poll_limit;
    s.err = hlhgat::device_error_word();
    HLH_CHECK_ARG(s.err, "bn_fwd_train: no device error word (%s)", hlhgat_last_error());
    ApplyArgs p{n_valid, x, ldx, y, ldy, n, (int)C, save_mean, save_invstd, weight, bias,
                relu, L.tpr, L.rp};
    hipStream_t st = as_stream(stream);
    dim3 g1(L.parts, L.tiles);
    if (vec)
      k_bn_train_fused<4><<<g1, kThreads, 0, st>>>(s, p);
    else
      k_bn_train_fused<1><<<g1, kThreads, 0, st>>>(s, p);
    HLH_CHECK_LAUNCH();
    return HLHGAT_OK;
  }
  int rc = hlhgat_bn_stats_train(x, ldx, n, n_valid, C, running_mean, running_var,
                                 num_batches_tracked, momentum, eps, save_mean, save_invstd,
                                 workspace, workspace_bytes, stream);
  if (rc) return rc;
  return hlhgat_bn_apply(x, ldx, n, n_valid, C, weight, bias, save_mean, save_invstd, relu, y,
                         ldy, stream);
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
  if (vec)
    k_bn_bwd_reduce<4, kThreads><<<g1, kThreads, 0, st>>>(s);
  else
    k_bn_bwd_reduce<1, kThreads><<<g1, kThreads, 0, st>>>(s);
  HLH_CHECK_LAUNCH();
  BwdApplyArgs p{n_valid, x, ldx, y, ldy, dy, lddy, dx, lddx, n, (int)C, w.coef, save_mean,
                 L.tpr, L.rp};
  dim3 g2(apply_grid_x(n, L.rp), L.tiles);
  if (vec)
    k_bn_bwd_apply<4><<<g2, kThreads, 0, st>>>(p);
  else
    k_bn_bwd_apply<1><<<g2, kThreads, 0, st>>>(p);
  HLH_CHECK_LAUNCH();
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
