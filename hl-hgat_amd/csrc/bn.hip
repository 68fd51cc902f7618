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

#include <atomic>
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
// + per tile: the one-launch kernels' barrier / generation word (64-bit)
constexpr int kCounters = kGridBase + 2 * kMaxTiles;
// give-up slots of the one-launch kernels, one 64-bit word per workgroup
constexpr int kMaxSlots = 4096;
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
int64_t bn_parts(int64_t n, int64_t min_parts = 128) {
  int64_t p = std::max<int64_t>(min_parts, ceil_div(n, (int64_t)512));
  // small batches (the readout MLP: one row per graph): >= 64 rows per
  // partition, so the finaliser's partial loads stay one batch deep
  p = std::min<int64_t>(p, std::max<int64_t>(1, ceil_div(n, (int64_t)64)));
  return p < 1 ? 1 : (p > kMaxParts ? kMaxParts : p);
}

// HLHGAT_BN_BWD_PARTS: minimum row partitions of the backward reduction
// (default 128, the forward's; A/B)
int64_t bn_bwd_min_parts() {
  static const int64_t v = [] {
    const char* e = std::getenv("HLHGAT_BN_BWD_PARTS");
    const int64_t p = e ? (int64_t)std::atoll(e) : 128;
    return p < 1 ? (int64_t)1 : (p > kMaxParts ? (int64_t)kMaxParts : p);
  }();
  return v;
}

// The backward reduction's partials go through the two-level tree (groups of
// kGroup) from 16 partitions up: same-box A/B at config 2 (128 partitions,
// profiles/r05/ab_cfg2_bn_bwd_tree.txt) 2.695 vs 2.710-2.718 ms with the flat
// pass.  (The backward has one path, so no other launch's summation order has
// to match it; the forward keeps the flat order its one- and two-launch paths
// share.)  HLHGAT_BN_BWD_FLAT_MAX overrides (A/B).
int bn_bwd_flat_max() {
  static const int v = [] {
    const char* e = std::getenv("HLHGAT_BN_BWD_FLAT_MAX");
    const int f = e ? std::atoi(e) : kGroup;
    return f < 1 ? 1 : (f > kFlatMax ? kFlatMax : f);
  }();
  return v;
}

BnLayout bn_layout(int64_t n, int64_t C, bool vec, int64_t min_parts = 128) {
  BnLayout L;
  L.v = vec ? 4 : 1;
  int lanes = (int)ceil_div(C, L.v);
  L.tpr = next_pow2(lanes);
  if (L.tpr > kThreads / L.v) L.tpr = kThreads / L.v;  // tile_c <= kThreads
  L.rp = kThreads / L.tpr;
  L.tile_c = L.tpr * L.v;
  L.tiles = (int)ceil_div(C, L.tile_c);
  int64_t parts = bn_parts(n, min_parts);
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
  unsigned long long* slots;  // [kMaxSlots] (tagged by generation, never reset)
  double* part;      // [parts][C][2]
  double* gpart;     // [groups][C][2]
  float* coef;       // [3][C] (bwd: a, b, c)
};

size_t align_up(size_t v) { return (v + 255) & ~size_t(255); }

// Counters live at a FIXED offset so a launch with a different (n, C) never
// reads another launch's partials as a counter.
size_t bn_ws_bytes(int64_t n, int64_t C) {
  (void)n;
  return align_up(sizeof(unsigned) * kCounters) + align_up(sizeof(unsigned long long) * kMaxSlots) +
         align_up(sizeof(double) * 2 * kMaxParts * C) +
         align_up(sizeof(double) * 2 * kMaxGroups * C) + align_up(sizeof(float) * 3 * C);
}

BnWs carve(void* ws, int64_t n, int64_t C) {
  (void)n;
  char* p = (char*)ws;
  BnWs w;
  w.count = (unsigned*)p;
  p += align_up(sizeof(unsigned) * kCounters);
  w.slots = (unsigned long long*)p;
  p += align_up(sizeof(unsigned long long) * kMaxSlots);
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
  // one-launch kernels: output rows, the wait bound of the barrier
  // (microseconds), the error word, the tile's give-up slots
  float* out;
  int64_t ldo;
  int relu;
  unsigned wait_us;
  unsigned* err;
  unsigned long long* slots;
  // SyncBatchNorm (hlhgat_bn_sums_*): the finaliser writes this rank's fp64
  // column sums [S0[C], S1[C], n_eff] here instead of finishing the statistics
  double* sums_out;
  // last_reduce: one flat pass over the partials up to this many, else the
  // two-level tree (groups of kGroup); kFlatMax except in the backward
  int flat_max;
};

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// --- the one-launch kernels' barrier --------------------------------------
// A workgroup of a one-launch kernel (k_bn_fwd_grid, k_proj_bn_fwd) arrives
// (its partials written through), then waits for the workgroup that arrives
// LAST -- the finaliser -- to publish the tile's statistics by bumping the
// tile's generation word.  Nothing in the design may depend on every
// workgroup being resident at once: the hardware places the workgroups of
// concurrent kernels (the other chain's, RCCL's, a user's) as it likes, and
// two barrier grids of different resource shapes on two queues can each hold
// CUs the other one's unplaced workgroups need.  So the wait is bounded in
// TIME (wait_us of the 100 MHz constant clock), and a workgroup whose wait
// runs out does not fail: it leaves its rows to the finaliser and exits,
// freeing its CU for the workgroups still unplaced:
//   waiter  : slot[blk] = (gen0 << 2) | 1 ("left")  --  seq_cst, agent scope
//             then reads the generation again; if it has moved, it races the
//             finaliser for the slot (CAS left -> taken) and normalises its
//             own rows from its registers when it wins;
//   finaliser: after bumping the generation, reads every slot of its tile and
//             takes (CAS left -> taken) each one marked "left" in THIS
//             generation, then normalises those rows from x in memory with
//             the same fp32 operations.
// Of the waiter's (slot store, generation load) and the finaliser's
// (generation bump, slot load) at least one side sees the other's write, so
// every row is normalised exactly once, by its owner or by the finaliser,
// with bitwise the same result; the slots are tagged with the generation,
// so a slot left in an earlier launch never matches.  No workgroup waits for
// anything without a time bound, so the kernel cannot deadlock whatever the
// residency.  A give-up is counted (hlhgat_bn_wait_timeouts) and logged
// (hlhgat_bn_giveup_log: tile, arrivals, total, generations) -- it costs
// time, never correctness.
//
// The counters reset themselves (an arrival word returns to 0, the
// generation only grows); a counter found beyond its total (state written by
// something else) raises HLHGAT_DEVERR_BN_STATE in the host-visible error
// word: the statistics of that launch are not trusted.
__device__ unsigned g_bn_wait_timeouts = 0;
__device__ unsigned g_bn_log_n = 0;
__device__ hlhgat_bn_giveup_t g_bn_log[HLHGAT_BN_LOG_MAX];

constexpr uint64_t kTicksPerUs = 100;  // s_memrealtime runs at 100 MHz
enum : unsigned { kKidBnGrid = 1, kKidProjBn = 2 };

__device__ __forceinline__ void report_state_error(unsigned* err) {
  if (err) __hip_atomic_store(err, (unsigned)HLHGAT_DEVERR_BN_STATE, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_SYSTEM);
}

// Signal arrival; returns true in the last workgroup of `total`.  Every wave
// has drained its write-through partial stores (vmcnt(0)) before the barrier;
// ONE lane adds to the counter; the workgroup whose add returned total-1
// resets it (an atomic store: the word is only ever touched by atomics) and
// reads the partials after the second barrier.
__device__ __forceinline__ bool arrive_last(unsigned* counter, unsigned total, unsigned* err) {
  __shared__ unsigned s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    s_last = (prev == total - 1) ? 1u : 0u;
    if (prev >= total) report_state_error(err);
    if (s_last)  // ready for the next launch (stream-ordered)
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return s_last != 0u;
}

typedef __attribute__((address_space(1))) unsigned long long gu64c_t;

__device__ __forceinline__ unsigned long long slot_mark(unsigned gen0) {
  return ((unsigned long long)gen0 << 2) | 1ull;  // "left"; | 2 = "taken"
}

// Thread 0 of a waiting workgroup: poll the tile's generation word for at most
// wait_us; true when it moved (the statistics are final).  wait_us == 0 looks
// once (a test hook that forces the give-up path).
__device__ __forceinline__ bool poll_gen(unsigned long long* word, unsigned gen0,
                                         unsigned wait_us) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t lim = (uint64_t)wait_us * kTicksPerUs;
  for (;;) {
    const unsigned long long w =
        __hip_atomic_load((gu64c_t*)word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(w >> 32) != gen0) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 >= lim) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

// Thread 0 of a workgroup whose wait ran out (see above).  Returns true when
// the workgroup reclaimed its rows (the statistics are final by then).
// `arr` / `total`: the arrival counter and the count it waits for (log only).
__device__ __forceinline__ bool give_up(unsigned long long* word, unsigned long long* slot,
                                        unsigned gen0, unsigned kid, const unsigned* arr,
                                        bool arr_low64, unsigned total, unsigned wait_us) {
  const unsigned long long mark = slot_mark(gen0);
  __hip_atomic_store((gu64c_t*)slot, mark, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long w =
      __hip_atomic_load((gu64c_t*)word, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
  bool mine = false;
  if ((unsigned)(w >> 32) != gen0) {
    unsigned long long exp = mark;
    mine = __hip_atomic_compare_exchange_strong((gu64c_t*)slot, &exp, mark + 1ull,
                                                __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST,
                                                __HIP_MEMORY_SCOPE_AGENT);
  }
  __hip_atomic_fetch_add(&g_bn_wait_timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned k =
      __hip_atomic_fetch_add(&g_bn_log_n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (k < HLHGAT_BN_LOG_MAX) {
    hlhgat_bn_giveup_t r;
    r.kernel = kid;
    r.tile = blockIdx.y;
    r.block = blockIdx.x;
    r.total = total;
    r.arrivals = arr_low64
                     ? (unsigned)(__hip_atomic_load((gu64c_t*)arr, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) & 0xffffffffull)
                     : __hip_atomic_load(arr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    r.gen0 = gen0;
    r.gen_seen = (unsigned)(w >> 32);
    r.wait_us = wait_us;
    r.outcome = mine ? 1u : 2u;
    g_bn_log[k] = r;
  }
  return mine;
}

// The finaliser's generation bump (thread 0): a RETURNING agent-scope RMW,
// performed at the coherence point, that thread 0 waits for (vmcnt(0))
// before the workgroup barrier preceding take_left's slot loads -- so every
// slot load is issued after the bump is visible to every workgroup.  With the
// waiter's seq_cst slot store then generation load (give_up), one of the two
// sides sees the other's write.  No agent-scope fence: what the
// waiting workgroups read after the bump (partials, mean / invstd) was
// written through with atomic stores and drained before it, and the fence's
// L2 write-back cost ~2 us on every launch's critical path (round 6: the
// config-2 step 2.73 vs 2.64 ms with it, profiles/r06/ab_bn_bump.txt).
__device__ __forceinline__ void publish_gen(unsigned long long* word, unsigned long long inc) {
  const unsigned long long old =
      __hip_atomic_fetch_add((gu64c_t*)word, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("" ::"v"(old));  // the returning form: its completion is what vmcnt waits for
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The finaliser, after publish_gen: take every slot of [slots, slots + n)
// left in this generation; taken[j] (LDS) = 1 for those (agent-scope atomic
// loads, issued after the bump completed; a match is taken with a seq_cst
// CAS).  Returns (in every thread) whether any was taken.
template <int NT>
__device__ __forceinline__ bool take_left(unsigned long long* slots, int n, unsigned gen0,
                                          unsigned char* taken) {
  __shared__ unsigned s_any;
  if (threadIdx.x == 0) s_any = 0u;
  __syncthreads();
  const unsigned long long mark = slot_mark(gen0);
  for (int j = threadIdx.x; j < n; j += NT) {
    unsigned char t = 0;
    const unsigned long long v =
        __hip_atomic_load((gu64c_t*)(slots + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == mark) {
      unsigned long long exp = mark;
      if (__hip_atomic_compare_exchange_strong((gu64c_t*)(slots + j), &exp, mark + 1ull,
                                               __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        t = 1;
        s_any = 1u;
      }
    }
    taken[j] = t;
  }
  __syncthreads();
  return s_any != 0u;
}

// Grid barrier of the `total` workgroups of one column tile on ONE 64-bit
// word: arrival count in the low half, generation in the high half.  Every
// workgroup adds 1; the one that completes the count turns it back to 0 and
// bumps the generation in the same word (one atomic add of 2^32 - total): it
// is the finaliser (kFinal) and returns at once.  The others wait (above):
// kOwn = normalise your own rows, kLeft = the finaliser does.  *gen0 = the
// generation of this launch.  Nothing is left to reset afterwards, whatever
// `total` the next launch uses.
enum : unsigned { kOwn = 0, kFinal = 1, kLeft = 2 };
__device__ __forceinline__ unsigned bar_wait(unsigned long long* word, unsigned long long* slot,
                                             unsigned total, unsigned wait_us, unsigned* err,
                                             unsigned* gen0_out) {
  __shared__ unsigned s_role, s_gen0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long old =
        __hip_atomic_fetch_add((gu64c_t*)word, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned gen0 = (unsigned)(old >> 32);
    const unsigned arrived = (unsigned)(old & 0xffffffffull);
    unsigned role;
    if (arrived >= total) report_state_error(err);
    if (arrived == total - 1) {
      // the bump, completed before the workgroup barrier that precedes
      // take_left's slot loads (publish_gen: the finaliser's half of the
      // store-load handshake with give_up)
      publish_gen(word, (1ull << 32) - (unsigned long long)total);
      role = kFinal;
    } else if (poll_gen(word, gen0, wait_us)) {
      role = kOwn;
    } else {
      role = give_up(word, slot, gen0, kKidBnGrid, reinterpret_cast<const unsigned*>(word), true,
                     total, wait_us)
                 ? kOwn
                 : kLeft;
    }
    s_role = role;
    s_gen0 = gen0;
  }
  __syncthreads();
  *gen0_out = s_gen0;
  return s_role;
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
  if (a.parts <= a.flat_max) {
    if (!arrive_last(a.count + tile, (unsigned)a.parts, a.err)) return false;
    flat_reduce<NT>(a.part, a.parts, a, c0, tile_c, out0, out1);
    return true;
  }
  const int g = blk.x / kGroup;
  const int ng = (a.parts + kGroup - 1) / kGroup;
  const int first = g * kGroup;
  const int cnt = a.parts - first < kGroup ? a.parts - first : kGroup;
  if (!arrive_last(a.count + kMaxTiles + tile * kMaxGroups + g, (unsigned)cnt, a.err))
    return false;
  reduce_range<NT>(a.part, first, cnt, a, c0, tile_c, out0, out1);
  for (int t = threadIdx.x; t < tile_c; t += NT) {
    const int c = c0 + t;
    if (c < a.C) {
      double* dst = a.gpart + ((int64_t)g * a.C + c) * 2;
      st_wt(dst, out0[t]);
      st_wt(dst + 1, out1[t]);
    }
  }
  if (!arrive_last(a.count + tile, (unsigned)ng, a.err)) return false;
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
  // eval mode (hlhgat_bn_apply_running): invstd = 1 / sqrt(var + eps) per
  // column from the running variance instead of `invstd`
  const float* var;
  float eps;
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
    const float is = a.var ? 1.f / sqrtf(a.var[c + v] + a.eps) : a.invstd[c + v];
    s[v] = w * is;
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

void launch_bwd_reduce(bool vec, dim3 grid, hipStream_t st, ProfScope* prof, const StatsArgs& s) {
  if (vec)
    launch(k_bn_bwd_reduce<4>, grid, dim3(kThreads), 0, st, prof, s);
  else
    launch(k_bn_bwd_reduce<1>, grid, dim3(kThreads), 0, st, prof, s);
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
template <int V>
__device__ __forceinline__ typename VecT<V>::type bn_row_out(typename VecT<V>::type x,
                                                             const float (&mu)[V],
                                                             const float (&sc)[V],
                                                             const float (&sh)[V], bool pad,
                                                             int relu) {
  typename VecT<V>::type o;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    const float z = (vget(x, v) - mu[v]) * sc[v] + sh[v];
    vget(o, v) = pad ? 0.f : ((relu && z < 0.f) ? 0.f : z);
  }
  return o;
}

template <int V, int RPT>
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
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int64_t r = r_lo + rg + (int64_t)j * a.rp;
      if (r < r_hi) xr[j] = vload<V>(a.x + r * a.ldx + c);
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
  unsigned long long* tile_slots = a.slots + (int64_t)blk.y * blk.gx;
  unsigned gen0 = 0;
  const unsigned role =
      bar_wait(barrier_word(a, blk), tile_slots + blk.x, blk.gx, a.wait_us, a.err, &gen0);
  if (role == kLeft) return;  // the finaliser normalises these rows
  __shared__ double sum0[kThreads], sum1[kThreads];
  __shared__ float sm[kThreads], ss[kThreads];
  const int tile_c = a.tpr * V;
  flat_reduce<kThreads>(a.part, blk.gx, a, c0, tile_c, sum0, sum1);
  // the finaliser writes the saved and running statistics (exactly once)
  const bool fin = role == kFinal;
  for (int t = threadIdx.x; t < tile_c; t += kThreads) {
    const int cc = c0 + t;
    float m = 0.f, is = 0.f;
    if (cc < a.C) {
      fwd_finalize(a, cc, sum0[t], sum1[t], n_eff, m, is, fin);
      if (fin) {
        a.save_mean[cc] = m;
        a.save_invstd[cc] = is;
      }
    }
    sm[t] = m;
    ss[t] = is;
  }
  if (fin && a.nbt && blk.y == 0 && threadIdx.x == 0) a.nbt[0] += 1;
  __syncthreads();
  float sc[V], mu[V], sh[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    sc[v] = wv[v] * ss[cl * V + v];
    mu[v] = sm[cl * V + v];
    sh[v] = bv[v];
  }
  if (c < a.C) {
    int64_t r_end = r_lo + a.rows_per_part;
    if (r_end > a.n) r_end = a.n;
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int64_t r = r_lo + rg + (int64_t)j * a.rp;
      if (r < r_end) vstore<V>(a.out + r * a.ldo + c, bn_row_out<V>(xr[j], mu, sc, sh, r >= n_eff, a.relu));
    }
  }
  if (!fin) return;
  // rows of partitions whose owners gave up: from x in memory, same operations
  __shared__ unsigned char taken[kMaxParts];
  if (!take_left<kThreads>(tile_slots, (int)blk.gx, gen0, taken)) return;
  if (c >= a.C) return;
  for (unsigned p = 0; p < blk.gx; ++p) {
    if (!taken[p]) continue;
    const int64_t p_lo = (int64_t)p * a.rows_per_part;
    int64_t p_end = p_lo + a.rows_per_part;
    if (p_end > a.n) p_end = a.n;
    for (int64_t r = p_lo + rg; r < p_end; r += a.rp) {
      vt xv = vload<V>(a.x + (r < n_eff ? r : 0) * a.ldx + c);
      vstore<V>(a.out + r * a.ldo + c, bn_row_out<V>(xv, mu, sc, sh, r >= n_eff, a.relu));
    }
  }
}

template <int V, int RPT>
__global__ __launch_bounds__(kThreads) void k_bn_fwd_grid(StatsArgs a) {
  k_bn_fwd_grid_body<V, RPT>(a, blk_hw());
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
//   3. every other workgroup polls that word, reads the statistics and
//      normalises its tile from the registers: y = relu?((x - mean) *
//      (w invstd) + b), rows >= n_valid written as 0.  The wait is bounded
//      in time; a workgroup whose wait runs out leaves its tile to the
//      finaliser, which normalises it from the stored x (the barrier protocol
//      above: no residency assumption, bitwise the same y).
// Against projection -> k_bn_fwd_grid this
// saves the BatchNorm launch, its read of x and its own load latency.  The
// statistics are the same sums in a different fp64 order (not bitwise the
// two-kernel path; equal to 1e-6, tests/test_gpu_parity.py).
// ---------------------------------------------------------------------------
struct ProjBnArgs {
  FwdArgs g;    // the projection: g.C = x (pre-BatchNorm), g.ldc
  StatsArgs s;  // the BatchNorm: s.out = y, partials / counters / error word
  int stats_only;  // 1: no wait -- the finaliser writes the statistics, k_bn_apply follows
  // diagnostics (hlhgat_set_proj_bn_stamps): 8 words per workgroup, thread 0
  // stamps s_memrealtime (100 MHz) at each phase boundary; NULL = off
  unsigned long long* stamps;
};

// one phase stamp of k_proj_bn_fwd (a plain vector store from one lane); a
// separate instantiation (STAMPS), so the product kernel keeps its registers
// (the stamps cost the 4th resident workgroup per CU)
template <bool STAMPS>
__device__ __forceinline__ void pb_stamp(const ProjBnArgs& a, int k, unsigned long long v) {
  if (STAMPS && a.stamps && threadIdx.x == 0)
    a.stamps[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + k] = v;
}
__device__ __forceinline__ unsigned long long pb_now() { return __builtin_amdgcn_s_memrealtime(); }

constexpr int kPbTN = 4;  // 64 columns per workgroup: one BatchNorm column tile

__device__ __forceinline__ unsigned long long* gen_word(const StatsArgs& a, int tile) {
  return reinterpret_cast<unsigned long long*>(a.count + kGridBase) + tile;
}

template <bool STAMPS>
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
  pb_stamp<STAMPS>(a, 0, pb_now());
  proj_fwd_lds_mainloop<kPbTN>(g, bx, by, wl, acc);
  pb_stamp<STAMPS>(a, 1, pb_now());
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
  // (Round 6: storing x after the partials and the running statistics after
  // the bump was bitwise and ~1 us shorter alone, but not faster in the
  // config-2 step -- profiles/r06/ab_proj_bn_order.txt; not kept.)
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
  pb_stamp<STAMPS>(a, 2, pb_now());
  const bool grp_last = arrive_last(s.count + kMaxTiles + by * kMaxGroups + grp, (unsigned)cnt,
                                    s.err);
  if (grp_last) {
    reduce_range<kThreads>(s.part, first, cnt, s, n_base, 64, sum0, sum1);
    if (threadIdx.x < 64) {
      double* dst = s.gpart + ((int64_t)grp * s.C + n_base + threadIdx.x) * 2;
      st_wt(dst, sum0[threadIdx.x]);
      st_wt(dst + 1, sum1[threadIdx.x]);
    }
    top = arrive_last(s.count + by, (unsigned)ng, s.err);
  }
  pb_stamp<STAMPS>(a, 3, pb_now());
  pb_stamp<STAMPS>(a, 6, (grp_last ? 1ull : 0ull) | (top ? 2ull : 0ull));
  float* sm = reinterpret_cast<float*>(sum1 + 64);  // [64]
  float* ss = sm + 64;                              // [64]
  unsigned long long* tile_slots = s.slots + (int64_t)by * gridDim.x;
  if (a.stats_only) {  // x and the statistics only: nobody waits (k_bn_apply normalises)
    if (!top) return;
    reduce_range<kThreads>(s.gpart, 0, ng, s, n_base, 64, sum0, sum1);
    if (threadIdx.x < 64) {
      const int cc = n_base + threadIdx.x;
      float m, is;
      fwd_finalize(s, cc, sum0[threadIdx.x], sum1[threadIdx.x], n_eff, m, is, true);
      s.save_mean[cc] = m;
      s.save_invstd[cc] = is;
    }
    if (s.nbt && by == 0 && threadIdx.x == 0) s.nbt[0] += 1;
    return;
  }
  // (Round 6: releasing the waiting workgroups as soon as the group partials
  // were complete, each summing them itself, moved the bump 1.6 us earlier
  // but their own sum cost the same: end of launch unchanged, step neutral --
  // profiles/r06/proj_bn_phases_early.log, ab_proj_bn_early.txt.)
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
    if (threadIdx.x == 0) publish_gen(word, 1ull << 32);  // completed (see take_left)
    pb_stamp<STAMPS>(a, 4, pb_now());
  } else {
    if (threadIdx.x == 0) {
      unsigned ok = poll_gen(word, s_gen0, s.wait_us) ? 1u : 0u;
      pb_stamp<STAMPS>(a, 4, pb_now());
      if (!ok)
        ok = give_up(word, tile_slots + bx, s_gen0, kKidProjBn, s.count + by, false,
                     (unsigned)ng, s.wait_us)
                 ? 1u
                 : 0u;
      s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) return;  // the finaliser normalises this tile from the stored x
    if (threadIdx.x < 64) {
      const int cc = n_base + threadIdx.x;
      sm[threadIdx.x] = __uint_as_float(__hip_atomic_load(
          reinterpret_cast<unsigned*>(s.save_mean + cc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      ss[threadIdx.x] = __uint_as_float(__hip_atomic_load(
          reinterpret_cast<unsigned*>(s.save_invstd + cc), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT));
    }
  }
  __syncthreads();
  // y from the registers (k_bn_fwd_grid's arithmetic)
#pragma unroll
  for (int tn = 0; tn < kPbTN; ++tn) {
    const int cl = tn * 16 + i, cc = n_base + cl;
    const float sc = (s.weight ? s.weight[cc] : 1.f) * ss[cl];
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
  pb_stamp<STAMPS>(a, 5, pb_now());
  if (!top) return;
  // row blocks whose owners gave up: y from the x they stored, same operations
  __shared__ unsigned char taken[kMaxParts];
  if (!take_left<kThreads>(tile_slots, parts, s_gen0, taken)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // their x stores (released at give-up)
  const int c4 = threadIdx.x & 15, rr = threadIdx.x >> 4;
  float sc[4], mu[4], sh[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int cl = 4 * c4 + v, cc = n_base + cl;
    sc[v] = (s.weight ? s.weight[cc] : 1.f) * ss[cl];
    mu[v] = sm[cl];
    sh[v] = s.bias ? s.bias[cc] : 0.f;
  }
  for (int p = 0; p < parts; ++p) {
    if (!taken[p]) continue;
    for (int64_t r = (int64_t)p * 64 + rr; r < (int64_t)p * 64 + 64 && r < g.M; r += 16) {
      float4 xv;
      const float* xp = g.C + r * g.ldc + n_base + 4 * c4;
      if (vx) xv = *reinterpret_cast<const float4*>(xp);
      else xv = make_float4(xp[0], xp[1], xp[2], xp[3]);
      const float4 o = bn_row_out<4>(xv, mu, sc, sh, r >= n_eff, s.relu);
      float* yp = s.out + r * s.ldo + n_base + 4 * c4;
      if (vy) {
        *reinterpret_cast<float4*>(yp) = o;
      } else {
        yp[0] = o.x;
        yp[1] = o.y;
        yp[2] = o.z;
        yp[3] = o.w;
      }
    }
  }
}

bool& proj_bn_fused_flag() {
  static bool v = true;
  return v;
}

// hlhgat_set_proj_bn_split(1): the projection + statistics launch (no wait;
// its last workgroup finalises) followed by k_bn_apply, instead of the one
// launch whose workgroups wait for the statistics; bitwise the same y.
bool& proj_bn_split_flag() {
  static bool v = false;
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
  s.slots = w.slots;
  s.err = hlhgat::device_error_word();
  s.flat_max = kFlatMax;
  return s;
}

// --- one-launch selection: grid size and registers -------------------------
// The one-launch kernels are taken when the grid is at most half of the
// chip's resident-workgroup capacity for that kernel
// (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs / 2), at most 256
// workgroups (the partials use the flat order) and a thread's rows fit the
// register budget (RPT <= kMaxRpt).  That sizing is for speed only: the
// barrier itself assumes nothing about residency (the bounded wait and the
// finaliser's hand-over above), so a launch beside any other kernels -- the
// other chain's barrier grid, RCCL, a whole-CU kernel -- completes with the
// same bits, at worst one wait bound later.
unsigned g_wait_us = 1000;

int64_t capacity_of(const void* kernel) {
  static auto* cache = new std::vector<std::pair<const void*, int64_t>>();
  for (const auto& kv : *cache)
    if (kv.first == kernel) return kv.second;
  int dev = 0, cus = 0, occ = 0;
  int64_t c = 0;
  // the share of the chip one barrier grid may take: 1 / HLHGAT_BN_COLOCATE
  // (default 2: the two chains' barrier launches usually overlap)
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

extern "C" int hlhgat_bn_apply_running(const float* x, int64_t ldx, int64_t n, int64_t C,
                                       const float* weight, const float* bias,
                                       const float* running_mean, const float* running_var,
                                       float eps, int relu, float* y, int64_t ldy, void* stream) {
  HLH_CHECK_ARG(n >= 1 && C >= 1 && C < (1 << 20) && ldx >= C && ldy >= C,
                "bn_apply_running: bad sizes n=%lld C=%lld", (long long)n, (long long)C);
  HLH_CHECK_ARG(x && y && running_mean && running_var, "bn_apply_running: NULL pointer");
  const bool vec = bn_vec_ok(C, {ldx, ldy}, {x, y});
  BnLayout L = bn_layout(n, C, vec);
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_apply_running: C too large");
  ApplyArgs p{nullptr, x, ldx, y, ldy, n, (int)C, running_mean, nullptr, weight, bias, relu,
              L.tpr, L.rp, running_var, eps};
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
    s.wait_us = g_wait_us;
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
unsigned long long* g_pb_stamps = nullptr;
int64_t g_pb_stamps_words = 0;

extern "C" int hlhgat_set_proj_bn_stamps(void* buf, int64_t words) {
  HLH_CHECK_ARG(words >= 0 && (buf != nullptr || words == 0), "set_proj_bn_stamps: bad buffer");
  g_pb_stamps = reinterpret_cast<unsigned long long*>(buf);
  g_pb_stamps_words = words;
  return HLHGAT_OK;
}

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
               gx <= (unsigned)kMaxParts && (int64_t)gx * gy <= kMaxSlots;
  if (fused) {
    const int64_t cap = capacity_of(reinterpret_cast<const void*>(k_proj_bn_fwd<false>));
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
  s.slots = w.slots;
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
  s.wait_us = g_wait_us;
  s.err = hlhgat::device_error_word();
  HLH_CHECK_ARG(s.err, "proj_bn_fwd: no device error word (%s)", hlhgat_last_error());
  // algorithmic: A read once, x and y written once; flops of the projection
  const double flops = 2.0 * (double)M * (double)N * (double)ktot;
  const double bytes = 4.0 * (double)M * ((double)ktot + 2.0 * (double)N);
  hipStream_t st = as_stream(stream);
  const bool split = proj_bn_split_flag();
  a.stats_only = split ? 1 : 0;
  if (g_pb_stamps && g_pb_stamps_words >= (int64_t)gx * gy * 8) a.stamps = g_pb_stamps;
  {
    ProfScope prof(HLHGAT_PROF_PROJ_BN, st, bytes, flops);
    if (a.stamps)
      launch(k_proj_bn_fwd<true>, dim3(gx, gy), dim3(kThreads), 0, st, &prof, a);
    else
      launch(k_proj_bn_fwd<false>, dim3(gx, gy), dim3(kThreads), 0, st, &prof, a);
  }
  HLH_CHECK_LAUNCH();
  if (split) {
    const bool vec2 = bn_vec_ok(N, {ldx, ldy}, {x, y});
    const BnLayout L = bn_layout(M, N, vec2);
    ApplyArgs p{n_valid, x, ldx, y, ldy, M, (int)N, save_mean, save_invstd, bn_weight, bn_bias,
                relu, L.tpr, L.rp};
    dim3 g2(apply_grid_x(M, L.rp), L.tiles);
    if (vec2)
      launch(k_bn_apply<4>, g2, dim3(kThreads), 0, st, nullptr, p);
    else
      launch(k_bn_apply<1>, g2, dim3(kThreads), 0, st, nullptr, p);
    HLH_CHECK_LAUNCH();
  }
  return HLHGAT_OK;
}

extern "C" int hlhgat_set_proj_bn_split(int on) {
  proj_bn_split_flag() = on != 0;
  return HLHGAT_OK;
}

extern "C" int hlhgat_set_proj_bn_fused(int on) {
  proj_bn_fused_flag() = on != 0;
  return HLHGAT_OK;
}

extern "C" int hlhgat_proj_bn_fused_capacity(int64_t* out) {
  HLH_CHECK_ARG(out, "proj_bn_fused_capacity: NULL pointer");
  *out = capacity_of(reinterpret_cast<const void*>(k_proj_bn_fwd<false>));
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
  BnLayout L = bn_layout(n, C, vec, bn_bwd_min_parts());
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_bwd_train: C too large");
  BnWs w = carve(workspace, n, C);
  StatsArgs s = stats_args(L, w, x, ldx, n, n_valid, C);
  s.flat_max = bn_bwd_flat_max();
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
      launch_bwd_reduce(true, g1, st, &prof, s);
    else
      launch_bwd_reduce(false, g1, st, &prof, s);
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
  BnLayout L = bn_layout(n, C, vec, bn_bwd_min_parts());
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_bwd_reduce: C too large");
  BnWs w = carve(workspace, n, C);
  StatsArgs s = stats_args(L, w, x, ldx, n, n_valid, C);
  s.flat_max = bn_bwd_flat_max();
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
    launch_bwd_reduce(true, dim3(L.parts, L.tiles), st, &prof, s);
  else
    launch_bwd_reduce(false, dim3(L.parts, L.tiles), st, &prof, s);
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
  const BnLayout L = bn_layout(n, C, vec, bn_bwd_min_parts());
  HLH_CHECK_ARG(L.tiles <= kMaxTiles, "bn_sums_bwd: C too large");
  StatsArgs s = stats_args(L, carve(workspace, n, C), x, ldx, n, n_valid, C);
  s.flat_max = bn_bwd_flat_max();  // the plain backward's partitions and order
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
    launch_bwd_reduce(true, dim3(g1), as_stream(stream), nullptr, s);
  else
    launch_bwd_reduce(false, dim3(g1), as_stream(stream), nullptr, s);
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

extern "C" int hlhgat_set_bn_one_launch(int on) {
  bn_one_launch_flag() = on != 0;
  return HLHGAT_OK;
}

extern "C" int hlhgat_get_bn_one_launch(void) { return bn_one_launch_flag() ? 1 : 0; }

extern "C" int hlhgat_set_bn_wait_us(unsigned wait_us) {
  g_wait_us = wait_us;
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_wait_timeouts(unsigned* out) {
  HLH_CHECK_ARG(out, "bn_wait_timeouts: NULL pointer");
  HLH_CHECK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bn_wait_timeouts), sizeof(unsigned)));
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_giveup_log(hlhgat_bn_giveup_t* out, int max, int* logged) {
  HLH_CHECK_ARG(logged && (max <= 0 || out), "bn_giveup_log: NULL pointer");
  unsigned n = 0;
  HLH_CHECK_HIP(hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_bn_log_n), sizeof(unsigned)));
  *logged = (int)n;
  int k = (int)n < HLHGAT_BN_LOG_MAX ? (int)n : HLHGAT_BN_LOG_MAX;
  if (k > max) k = max;
  if (k > 0)
    HLH_CHECK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bn_log), sizeof(hlhgat_bn_giveup_t) * k));
  return HLHGAT_OK;
}

extern "C" int hlhgat_bn_giveup_reset(void) {
  const unsigned z = 0;
  HLH_CHECK_HIP(hipDeviceSynchronize());
  HLH_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_bn_log_n), &z, sizeof(unsigned)));
  HLH_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_bn_wait_timeouts), &z, sizeof(unsigned)));
  return HLHGAT_OK;
}
