// Phase timing of the one-launch BatchNorm forward structure at the config-2
// shape (n = 25600 rows, C = 64, 128 row partitions x 200 rows, 256 threads):
// load rows -> LDS partials -> write-through fp64 partials -> grid barrier ->
// flat reduce of all partials -> normalise + store.  Thread 0 of every
// workgroup stamps s_memrealtime (100 MHz) at each phase boundary.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int NT = 256, C = 64, TPR = 16, RP = NT / TPR, RPT = 13;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

template <int MODE>  // MODE bit0: write-through partial stores; bit1: atomic partial loads
__global__ __launch_bounds__(NT) void k_probe(const float* x, float* y, double* part, unsigned* cnt,
                                              unsigned long long* ts, int parts, int rpp,
                                              unsigned epoch) {
  unsigned long long t[8];
  t[0] = now();
  const int cl = threadIdx.x % TPR, rg = threadIdx.x / TPR, c = cl * 4;
  const long r_lo = (long)blockIdx.x * rpp;
  float4 xr[RPT];
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const long r = r_lo + rg + j * RP;
    if (r < r_lo + rpp) xr[j] = *reinterpret_cast<const float4*>(x + r * C + c);
  }
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const long r = r_lo + rg + j * RP;
    if (r < r_lo + rpp) {
      const float v[4] = {xr[j].x, xr[j].y, xr[j].z, xr[j].w};
      for (int u = 0; u < 4; ++u) { s0[u] += v[u]; s1[u] += (double)v[u] * v[u]; }
    }
  }
  __syncthreads();
  t[1] = now();
  __shared__ double red[2][NT * 4];
  for (int u = 0; u < 4; ++u) { red[0][rg * C + c + u] = s0[u]; red[1][rg * C + c + u] = s1[u]; }
  __syncthreads();
  if (threadIdx.x < C) {
    double u0 = 0, u1 = 0;
    for (int g = 0; g < RP; ++g) { u0 += red[0][g * C + threadIdx.x]; u1 += red[1][g * C + threadIdx.x]; }
    double* d = part + ((long)blockIdx.x * C + threadIdx.x) * 2;
    if (MODE & 1) { st_wt(d, u0); st_wt(d + 1, u1); } else { d[0] = u0; d[1] = u1; }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  t[2] = now();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (unsigned it = 0; it < (1u << 22); ++it) {
      if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= parts * epoch) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  t[3] = now();
  __shared__ double fin[2][NT];
  const int G = NT / C, tt = threadIdx.x % C, jj = threadIdx.x / C;
  double u0 = 0, u1 = 0;
  for (int p0 = jj; p0 < parts; p0 += 16 * G) {
    double v0[16], v1[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int p = p0 + u * G;
      const double* q = part + ((long)(p < parts ? p : 0) * C + tt) * 2;
      if (MODE & 2) { v0[u] = p < parts ? ld_wt(q) : 0; v1[u] = p < parts ? ld_wt(q + 1) : 0; }
      else { v0[u] = p < parts ? q[0] : 0; v1[u] = p < parts ? q[1] : 0; }
    }
    for (int u = 0; u < 16; ++u) { u0 += v0[u]; u1 += v1[u]; }
  }
  fin[0][threadIdx.x] = u0; fin[1][threadIdx.x] = u1;
  __syncthreads();
  __shared__ float sm[C], ss[C];
  if (threadIdx.x < C) {
    double a = 0, b = 0;
    for (int g = 0; g < G; ++g) { a += fin[0][g * C + threadIdx.x]; b += fin[1][g * C + threadIdx.x]; }
    const double n = (double)parts * rpp, mean = a / n;
    sm[threadIdx.x] = (float)mean;
    ss[threadIdx.x] = (float)(1.0 / sqrt(b / n - mean * mean + 1e-5));
  }
  __syncthreads();
  t[4] = now();
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const long r = r_lo + rg + j * RP;
    if (r < r_lo + rpp) {
      float4 o;
      o.x = fmaxf((xr[j].x - sm[c]) * ss[c], 0.f);
      o.y = fmaxf((xr[j].y - sm[c + 1]) * ss[c + 1], 0.f);
      o.z = fmaxf((xr[j].z - sm[c + 2]) * ss[c + 2], 0.f);
      o.w = fmaxf((xr[j].w - sm[c + 3]) * ss[c + 3], 0.f);
      *reinterpret_cast<float4*>(y + r * C + c) = o;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  t[5] = now();
  if (threadIdx.x == 0)
    for (int i = 0; i < 6; ++i) ts[blockIdx.x * 8 + i] = t[i];
}

int main() {
  const int parts = 128, rpp = 200, n = parts * rpp;
  float *x, *y;
  double* part;
  unsigned* cnt;
  unsigned long long* ts;
  hipMalloc(&x, n * C * 4);
  hipMalloc(&y, n * C * 4);
  hipMalloc(&part, parts * C * 16);
  hipMalloc(&cnt, 64);
  hipMalloc(&ts, parts * 64);
  hipMemset(x, 0, n * C * 4);
  hipMemset(cnt, 0, 64);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  unsigned epoch = 0;
  for (int mode = 0; mode < 4; ++mode) {
    auto launch = [&]() {
      ++epoch;
      if (mode == 0) k_probe<0><<<parts, NT>>>(x, y, part, cnt, ts, parts, rpp, epoch);
      if (mode == 1) k_probe<1><<<parts, NT>>>(x, y, part, cnt, ts, parts, rpp, epoch);
      if (mode == 2) k_probe<2><<<parts, NT>>>(x, y, part, cnt, ts, parts, rpp, epoch);
      if (mode == 3) k_probe<3><<<parts, NT>>>(x, y, part, cnt, ts, parts, rpp, epoch);
    };
    for (int i = 0; i < 20; ++i) launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < 200; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    std::vector<unsigned long long> h(parts * 8);
    hipMemcpy(h.data(), ts, parts * 64, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull, tend = 0;
    double ph[5] = {0, 0, 0, 0, 0};
    for (int p = 0; p < parts; ++p) {
      t0 = std::min(t0, h[p * 8]);
      tend = std::max(tend, h[p * 8 + 5]);
      for (int i = 0; i < 5; ++i) ph[i] += (double)(h[p * 8 + i + 1] - h[p * 8 + i]) / parts;
    }
    printf("mode %d (wt-store %d, atomic-load %d): %.2f us/launch; span %.2f us; phases (us, avg over WGs): "
           "load %.2f, partials %.2f, barrier %.2f, reduce %.2f, apply %.2f\n",
           mode, mode & 1, (mode >> 1) & 1, ms * 1e3 / 200, (tend - t0) / 100.0, ph[0] / 100,
           ph[1] / 100, ph[2] / 100, ph[3] / 100, ph[4] / 100);
  }
  return 0;
}
