// Cost of a grid barrier among N co-resident workgroups on MI355X (gfx950):
//   A: one agent-scope atomic counter (fetch_add, then poll)
//   B: per-workgroup flags (store own flag, poll all N flags)
//   0: no barrier (launch floor)
// Each variant runs `reps` launches back to back, timed with hipEvents.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_none(unsigned* c, unsigned n, unsigned epoch) {}

__global__ void k_counter(unsigned* c, unsigned n, unsigned epoch) {
  __shared__ unsigned ok;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = n * epoch;
    for (unsigned it = 0; it < (1u << 22); ++it) {
      if (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      __builtin_amdgcn_s_sleep(1);
    }
    ok = 1;
  }
  __syncthreads();
}

__global__ void k_flags(unsigned* f, unsigned n, unsigned epoch) {
  __shared__ unsigned done;
  if (threadIdx.x == 0) {
    __hip_atomic_store(f + blockIdx.x * 16, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    done = 0;
  }
  __syncthreads();
  for (unsigned it = 0; it < (1u << 22); ++it) {
    unsigned mine = 1;
    for (unsigned p = threadIdx.x; p < n; p += blockDim.x)
      if (__hip_atomic_load(f + p * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch) mine = 0;
    if (__syncthreads_and(mine)) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

int main() {
  unsigned* buf;
  hipMalloc(&buf, 1 << 20);
  hipMemset(buf, 0, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int reps = 200;
  for (unsigned n : {32u, 64u, 128u, 256u}) {
    for (int v = 0; v < 3; ++v) {
      hipMemset(buf, 0, 1 << 20);
      unsigned epoch = 0;
      auto run = [&](int r) {
        for (int i = 0; i < r; ++i) {
          ++epoch;
          if (v == 0) k_none<<<n, 256>>>(buf, n, epoch);
          if (v == 1) k_counter<<<n, 256>>>(buf, n, epoch);
          if (v == 2) k_flags<<<n, 256>>>(buf, n, epoch);
        }
      };
      run(10);
      hipDeviceSynchronize();
      hipEventRecord(a);
      run(reps);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      printf("n=%3u %-8s %.2f us/launch\n", n, v == 0 ? "none" : v == 1 ? "counter" : "flags",
             ms * 1e3 / reps);
    }
  }
  return 0;
}
