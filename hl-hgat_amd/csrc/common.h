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
#include <string>

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
  int cls = -1;
  double bytes = 0.0, flops = 0.0;
  ProfScope(int kernel_class, hipStream_t s, double bytes, double flops);
};

struct Blk {  // a workgroup's coordinates in its (x, y) grid
  unsigned x, y, gx, gy;
};
__device__ __forceinline__ Blk blk_hw() { return Blk{blockIdx.x, blockIdx.y, gridDim.x, gridDim.y}; }

// Launch `k` on `s`; when `p` holds a live ProfScope the launch goes through
// hipExtLaunchKernelGGL with its start/stop events.
template <typename... KArgs, typename... Args>
inline void launch(void (*k)(KArgs...), dim3 grid, dim3 block, uint32_t shmem, hipStream_t s,
                   const ProfScope* p, Args... args) {
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
