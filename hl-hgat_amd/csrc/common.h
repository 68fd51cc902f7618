// Shared helpers for the hlhgat HIP library (gfx950 / CDNA4 only).
//
// Every exported entry point (include/hlhgat.h) validates its arguments on the
// host, launches on the caller's stream and returns 0 on success or a nonzero
// code with a thread-local message readable through hlhgat_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <cstdio>
#include <cstdarg>
#include <functional>
#include <memory>
#include <string>
#include <tuple>

#include "../../include/hlhgat.h"

namespace hlhgat {

void set_error(const char* fmt, ...);

// The host-visible device error word (hlhgat_device_errors), allocated on
// first use; NULL (with the error set) if the pinned allocation fails.
unsigned* device_error_word();

#define HLH_CHECK_ARG(cond, ...)                     \
  do {                                               \
    if (!(cond)) {                                   \
      ::hlhgat::set_error(__VA_ARGS__);              \
      return HLHGAT_EINVAL;                          \
    }                                                \
  } while (0)

#define HLH_CHECK_HIP(expr)                                              \
  do {                                                                   \
    hipError_t _e = (expr);                                              \
    if (_e != hipSuccess) {                                              \
      ::hlhgat::set_error("%s failed: %s (%s:%d)", #expr,                \
                          hipGetErrorString(_e), __FILE__, __LINE__);    \
      return HLHGAT_EHIP;                                                \
    }                                                                    \
  } while (0)

#define HLH_CHECK_LAUNCH() HLH_CHECK_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}
inline bool aligned8(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 7u) == 0;
}

inline int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------------------
// Live kernel timing (hlhgat_prof_*): when enabled, launches of the kernel
// class being profiled are bracketed by hipEvents recorded on the SAME stream
// the kernel runs on, and the algorithmic bytes of each launch are recorded.
// ---------------------------------------------------------------------------
// The events are handed to hipExtLaunchKernel, which stamps them at the
// kernel's own start and end (the dispatch packet's timestamps, as rocprofv3
// reads them): no extra stream packets, so the timed launch is not slowed and
// the measured duration agrees with the rocprofv3 kernel trace.
struct ProfScope {
  int slot = -1;
  hipEvent_t start_ev = nullptr, stop_ev = nullptr;
  // what the scope measures, kept for launches deferred by a launch group
  // (the slot is then taken when the launch is finally issued)
  int cls = -1;
  double bytes = 0.0, flops = 0.0;
  ProfScope(int kernel_class, hipStream_t s, double bytes, double flops);
};

// ---------------------------------------------------------------------------
// Launch groups (hlhgat_group_begin / _next / _end, include/hlhgat.h): the
// node-side and edge-side launch sequences of an HL block are recorded as the
// two MEMBERS of a group instead of being issued; at the end the i-th launch
// of member 0 and the i-th of member 1 become ONE launch of the kernel's pair
// variant (both argument sets behind one grid: workgroups [0, start1) run
// member 0's grid, the rest member 1's) whenever both are the same kernel and
// a pair variant is registered, otherwise they are issued one after the
// other.  Each member's launches stay in their recorded order.
// ---------------------------------------------------------------------------
struct Blk {  // a workgroup's coordinates in its member's (x, y) grid
  unsigned x, y, gx, gy;
};
__device__ __forceinline__ Blk blk_hw() { return Blk{blockIdx.x, blockIdx.y, gridDim.x, gridDim.y}; }

template <class A>
struct Pair {
  A a[2];
  unsigned gx[2], gy[2];
  unsigned start1;  // first workgroup of member 1 (a multiple of 8: it starts on XCD 0)
};

// Member s and the workgroup's coordinates in its grid; false for the
// alignment padding between the two grids.
template <class A>
__device__ __forceinline__ bool pair_blk(const Pair<A>& p, int& s, Blk& b) {
  unsigned L = blockIdx.x;
  s = L >= p.start1 ? 1 : 0;
  if (s) L -= p.start1;
  b.gx = p.gx[s];
  b.gy = p.gy[s];
  b.x = L % b.gx;
  b.y = L / b.gx;
  return b.y < b.gy;
}

// Pair variant of a kernel whose body is BODY(const A&, Blk); each member's
// branch reads its own argument block at a static offset.
#define HLH_PAIR_KERNEL(NAME, A, BODY)                                          \
  __global__ __launch_bounds__(256) void NAME(::hlhgat::Pair<A> p) {          \
    int s;                                                                     \
    ::hlhgat::Blk b;                                                           \
    if (!::hlhgat::pair_blk(p, s, b)) return;                                  \
    if (s == 0)                                                                \
      BODY(p.a[0], b);                                                         \
    else                                                                       \
      BODY(p.a[1], b);                                                         \
  }

struct Recorded;
using PairLauncher = void (*)(const Recorded&, const Recorded&, hipStream_t, const ProfScope*);
struct Recorded {
  const void* kernel = nullptr;
  dim3 grid, block;
  uint32_t shmem = 0;
  int cls = -1;
  double bytes = 0.0, flops = 0.0;
  std::shared_ptr<void> args;                               // typed copy of the argument block
  std::function<void(hipStream_t, const ProfScope*)> solo;  // issue alone
  PairLauncher pair = nullptr;                              // issue with a partner (same kernel)
};

bool group_recording();         // this thread is recording a launch group
void group_record(Recorded&& r);  // append to the current member

// Registered pair variants: solo kernel -> (pair kernel, co-residency bound)
struct PairEntry {
  const void* pair_kernel;
  bool needs_coresidency;  // grid-barrier kernels: the pair grid must fit (see bn.hip)
};
void register_pair(const void* solo, const void* pair, bool needs_coresidency);
const PairEntry* find_pair(const void* solo);
// bn.hip: may this many workgroups of `pair_kernel` wait at a grid barrier?
bool pair_coresident(const void* pair_kernel, int64_t blocks);

template <class A>
void pair_launch_typed(const Recorded& r0, const Recorded& r1, hipStream_t s,
                       const ProfScope* p) {
  Pair<A> P;
  P.a[0] = *static_cast<const A*>(r0.args.get());
  P.a[1] = *static_cast<const A*>(r1.args.get());
  P.gx[0] = r0.grid.x;
  P.gy[0] = r0.grid.y;
  P.gx[1] = r1.grid.x;
  P.gy[1] = r1.grid.y;
  const unsigned n0 = r0.grid.x * r0.grid.y;
  P.start1 = (n0 + 7u) & ~7u;
  const unsigned total = P.start1 + r1.grid.x * r1.grid.y;
  auto* k = reinterpret_cast<void (*)(Pair<A>)>(const_cast<void*>(find_pair(r0.kernel)->pair_kernel));
  const uint32_t shmem = r0.shmem > r1.shmem ? r0.shmem : r1.shmem;
  if (p && p->start_ev)
    hipExtLaunchKernelGGL(k, dim3(total), r0.block, shmem, s, p->start_ev, p->stop_ev, 0, P);
  else
    hipLaunchKernelGGL(k, dim3(total), r0.block, shmem, s, P);
}

// Launch `k` on `s`; when `p` holds a live ProfScope the launch goes through
// hipExtLaunchKernelGGL with its start/stop events.  Inside a launch group
// the launch is recorded instead (single-argument kernels keep a typed copy
// so that a partner can be paired with it).
template <typename... KArgs, typename... Args>
inline void launch(void (*k)(KArgs...), dim3 grid, dim3 block, uint32_t shmem, hipStream_t s,
                   const ProfScope* p, Args... args) {
  if (group_recording()) {
    Recorded r;
    r.kernel = reinterpret_cast<const void*>(k);
    r.grid = grid;
    r.block = block;
    r.shmem = shmem;
    if (p) {
      r.cls = p->cls;
      r.bytes = p->bytes;
      r.flops = p->flops;
    }
    r.solo = [=](hipStream_t st, const ProfScope* q) {
      if (q && q->start_ev)
        hipExtLaunchKernelGGL(k, grid, block, shmem, st, q->start_ev, q->stop_ev, 0, args...);
      else
        hipLaunchKernelGGL(k, grid, block, shmem, st, args...);
    };
    if constexpr (sizeof...(Args) == 1) {
      using A = std::tuple_element_t<0, std::tuple<Args...>>;
      r.args = std::make_shared<A>(args...);
      r.pair = &pair_launch_typed<A>;
    }
    group_record(std::move(r));
    return;
  }
  if (p && p->start_ev)
    hipExtLaunchKernelGGL(k, grid, block, shmem, s, p->start_ev, p->stop_ev, 0, args...);
  else
    hipLaunchKernelGGL(k, grid, block, shmem, s, args...);
}

}  // namespace hlhgat

// Vector helpers ------------------------------------------------------------
template <int V> struct VecT;
template <> struct VecT<1> { using type = float; };
template <> struct VecT<2> { using type = float2; };
template <> struct VecT<4> { using type = float4; };

__device__ __forceinline__ float vzero1() { return 0.f; }

template <int V>
__device__ __forceinline__ typename VecT<V>::type vload(const float* p) {
  return *reinterpret_cast<const typename VecT<V>::type*>(p);
}
template <int V>
__device__ __forceinline__ void vstore(float* p, typename VecT<V>::type v) {
  *reinterpret_cast<typename VecT<V>::type*>(p) = v;
}

// Streaming (non-temporal) store of a whole vector as ONE dwordx2/x4 store.
// __builtin_nontemporal_store on the float4 components one by one issues V
// strided dword stores, each a partial cache line that the streaming path
// writes out on its own (the 1.3x write amplification of the factored edge
// step, profiles/r01_h_cfg5_pmc.txt); the clang vector type keeps it whole.
template <int V>
__device__ __forceinline__ void vstore_nt(float* p, typename VecT<V>::type v) {
  if constexpr (V == 1) {
    __builtin_nontemporal_store(v, p);
  } else {
    typedef float nv_t __attribute__((ext_vector_type(V)));
    nv_t n;
#pragma unroll
    for (int i = 0; i < V; ++i) n[i] = (&v.x)[i];
    __builtin_nontemporal_store(n, reinterpret_cast<nv_t*>(p));
  }
}

// Element access on the vector types so kernels can loop over components.
__device__ __forceinline__ float& vget(float& v, int) { return v; }
__device__ __forceinline__ float& vget(float2& v, int i) { return (&v.x)[i]; }
__device__ __forceinline__ float& vget(float4& v, int i) { return (&v.x)[i]; }
