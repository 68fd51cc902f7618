// Probe: the fused Laguerre step over a ZINC-scale L0 with the row's entries
// found through rowptr (CSR: rowptr -> col/val -> gathers, three dependent
// round trips) against a row-padded entry table (ELL, 16 (col, value) pairs
// per row: the entries and the row length load together).  Same per-row
// arithmetic; prints us per launch (chain of launches between two events).
//   hipcc -O3 --offload-arch=gfx950 tools/probes/ell_probe.hip -o /tmp/ell_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x) do { hipError_t rc_ = (x); if (rc_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(rc_), __LINE__); exit(1);} } while (0)

constexpr int LPR = 16;
struct Args {
  const int* rowptr; const int* col; const float* val; const int2* ell;
  const float* X; const float* Z; float* Y; int n; int d;
};

template <bool ELL>
__global__ __launch_bounds__(256) void k_step(Args a) {
  const int slot = (blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  const bool live = slot < a.n;
  const int row = live ? slot : 0;
  int e0 = 0, e1 = 0, cm = 0;
  float wm = 0.f;
  if (ELL) {
    e0 = a.rowptr[row];
    e1 = a.rowptr[row + 1];
    const int2 cw = a.ell[(size_t)row * 16 + sub];
    cm = cw.x;
    wm = __int_as_float(cw.y);
  } else {
    e0 = live ? a.rowptr[row] : 0;
    e1 = live ? a.rowptr[row + 1] : 0;
    const int me = e0 + sub;
    cm = me < e1 ? a.col[me] : 0;
    wm = me < e1 ? a.val[me] : 0.f;
  }
  const int f = sub * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int cnt = live ? (e1 - e0 < LPR ? e1 - e0 : LPR) : 0;
  int j = 0;
  for (; j + 3 < cnt; j += 4) {
    const int c0 = __shfl(cm, j, LPR), c1 = __shfl(cm, j + 1, LPR), c2 = __shfl(cm, j + 2, LPR),
              c3 = __shfl(cm, j + 3, LPR);
    const float w0 = __shfl(wm, j, LPR), w1 = __shfl(wm, j + 1, LPR), w2 = __shfl(wm, j + 2, LPR),
                w3 = __shfl(wm, j + 3, LPR);
    const float4 x0 = *(const float4*)(a.X + (size_t)c0 * a.d + f);
    const float4 x1 = *(const float4*)(a.X + (size_t)c1 * a.d + f);
    const float4 x2 = *(const float4*)(a.X + (size_t)c2 * a.d + f);
    const float4 x3 = *(const float4*)(a.X + (size_t)c3 * a.d + f);
    acc.x += w0 * x0.x + w1 * x1.x + w2 * x2.x + w3 * x3.x;
    acc.y += w0 * x0.y + w1 * x1.y + w2 * x2.y + w3 * x3.y;
    acc.z += w0 * x0.z + w1 * x1.z + w2 * x2.z + w3 * x3.z;
    acc.w += w0 * x0.w + w1 * x1.w + w2 * x2.w + w3 * x3.w;
  }
  for (; j < cnt; ++j) {
    const int c = __shfl(cm, j, LPR);
    const float w = __shfl(wm, j, LPR);
    const float4 x = *(const float4*)(a.X + (size_t)c * a.d + f);
    acc.x += w * x.x; acc.y += w * x.y; acc.z += w * x.z; acc.w += w * x.w;
  }
  if (!live) return;
  const float4 xb = *(const float4*)(a.X + (size_t)row * a.d + f);
  const float4 z = *(const float4*)(a.Z + (size_t)row * a.d + f);
  float4 o;
  o.x = (-acc.x + 3.f * xb.x - z.x) / 2.f;
  o.y = (-acc.y + 3.f * xb.y - z.y) / 2.f;
  o.z = (-acc.z + 3.f * xb.z - z.z) / 2.f;
  o.w = (-acc.w + 3.f * xb.w - z.w) / 2.f;
  *(float4*)(a.Y + (size_t)row * a.d + f) = o;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 23552, d = 64;
  const int maxdeg = argc > 2 ? atoi(argv[2]) : 5;
  std::mt19937 rng(1);
  std::vector<int> rp(n + 1, 0), col;
  std::vector<float> val;
  for (int r = 0; r < n; ++r) {
    const int len = 2 + (int)(rng() % (maxdeg - 1));
    for (int k = 0; k < len; ++k) {
      int c = k == 0 ? r : (int)((r + (int)(rng() % 41) - 20 + n) % n);  // local neighbours
      col.push_back(c);
      val.push_back(0.1f * (float)(rng() % 17));
    }
    rp[r + 1] = (int)col.size();
  }
  std::vector<int2> ell((size_t)n * 16, make_int2(0, 0));
  for (int r = 0; r < n; ++r)
    for (int e = rp[r]; e < rp[r + 1]; ++e) {
      int2 v; v.x = col[e]; float f = val[e]; v.y = *(int*)&f;
      ell[(size_t)r * 16 + (e - rp[r])] = v;
    }
  std::vector<float> X((size_t)n * d);
  for (auto& x : X) x = (float)(rng() % 1000) / 1000.f;
  int *drp, *dcol; float *dval, *dX, *dZ, *dY; int2* dell;
  CK(hipMalloc(&drp, sizeof(int) * (n + 1))); CK(hipMalloc(&dcol, sizeof(int) * col.size()));
  CK(hipMalloc(&dval, sizeof(float) * val.size())); CK(hipMalloc(&dell, sizeof(int2) * ell.size()));
  CK(hipMalloc(&dX, sizeof(float) * X.size())); CK(hipMalloc(&dZ, sizeof(float) * X.size()));
  CK(hipMalloc(&dY, sizeof(float) * X.size()));
  CK(hipMemcpy(drp, rp.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice));
  CK(hipMemcpy(dcol, col.data(), sizeof(int) * col.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dval, val.data(), sizeof(float) * val.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dell, ell.data(), sizeof(int2) * ell.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dX, X.data(), sizeof(float) * X.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dZ, X.data(), sizeof(float) * X.size(), hipMemcpyHostToDevice));
  Args a{drp, dcol, dval, dell, dX, dZ, dY, n, d};
  const int grid = (n * LPR + 255) / 256;
  hipEvent_t s, e;
  CK(hipEventCreate(&s)); CK(hipEventCreate(&e));
  std::vector<float> y0(X.size()), y1(X.size());
  for (int rep = 0; rep < 4; ++rep) {
    for (int ellm = 0; ellm < 2; ++ellm) {
      for (int w = 0; w < 5; ++w) {
        if (ellm) hipLaunchKernelGGL(k_step<true>, dim3(grid), dim3(256), 0, 0, a);
        else hipLaunchKernelGGL(k_step<false>, dim3(grid), dim3(256), 0, 0, a);
      }
      CK(hipEventRecord(s));
      for (int it = 0; it < 50; ++it) {
        if (ellm) hipLaunchKernelGGL(k_step<true>, dim3(grid), dim3(256), 0, 0, a);
        else hipLaunchKernelGGL(k_step<false>, dim3(grid), dim3(256), 0, 0, a);
      }
      CK(hipEventRecord(e));
      CK(hipEventSynchronize(e));
      float ms; CK(hipEventElapsedTime(&ms, s, e));
      CK(hipMemcpy(ellm ? y1.data() : y0.data(), dY, sizeof(float) * X.size(), hipMemcpyDeviceToHost));
      printf("%s n=%d maxdeg=%d: %.2f us/launch\n", ellm ? "ELL" : "CSR", n, maxdeg, ms * 1e3f / 50);
    }
  }
  size_t diff = 0;
  for (size_t i = 0; i < y0.size(); ++i) diff += y0[i] != y1[i];
  printf("outputs differing: %zu\n", diff);
  return 0;
}
