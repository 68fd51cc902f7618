// Symmetric tridiagonal helpers shared by the Lanczos kernels (hodge.hip,
// eigpe.hip): T = tridiag(be[1..k-1], al[0..k-1], be[1..k-1]), fp64.
#pragma once

#include <hip/hip_runtime.h>

namespace hlhgat {

// number of eigenvalues of T below x (Sturm sequence of the LDL^T pivots; a
// zero off-diagonal splits T into independent blocks, as it should)
__device__ __forceinline__ int sturm_count(const double* al, const double* be, int k, double x) {
  int c = 0;
  double d = 1.0;
  for (int i = 0; i < k; ++i) {
    const double b2 = i ? be[i] * be[i] : 0.0;
    d = (al[i] - x) - (i ? b2 / d : 0.0);
    if (d == 0.0) d = -1e-300;
    if (d < 0.0) ++c;
  }
  return c;
}

// Gershgorin interval of T
__device__ __forceinline__ void gershgorin(const double* al, const double* be, int k, double& lo,
                                           double& hi) {
  lo = 0.0;
  hi = 0.0;
  for (int i = 0; i < k; ++i) {
    const double r = (i ? fabs(be[i]) : 0.0) + (i + 1 < k ? fabs(be[i + 1]) : 0.0);
    lo = fmin(lo, al[i] - r);
    hi = fmax(hi, al[i] + r);
  }
}

// The m-th smallest eigenvalue of T (0-based) by one wave: the 64 lanes
// count the Sturm sequence at 64 interior points of [lo, hi] at once, so the
// interval shrinks 65-fold per pass; stops at `tol` absolute width.  Every
// lane returns the same value.  Must be called by all 64 lanes of the wave.
__device__ __forceinline__ double wave_eigenvalue(const double* al, const double* be, int k,
                                                  int m, double lo, double hi, double tol) {
  const int lane = threadIdx.x & 63;
  for (int it = 0; it < 40 && hi - lo > tol; ++it) {
    const double h = (hi - lo) / 65.0;
    // lanes 0 .. t: fewer than m + 1 eigenvalues below the point, so lambda_m >= it
    const bool below = sturm_count(al, be, k, lo + h * (double)(lane + 1)) <= m;
    const unsigned long long mask = __ballot(below);
    const int t = mask ? 63 - __clzll(mask) : -1;
    const double nlo = t >= 0 ? lo + h * (double)(t + 1) : lo;
    const double nhi = t < 63 ? lo + h * (double)(t + 2) : hi;
    lo = nlo;
    hi = nhi;
  }
  return 0.5 * (lo + hi);
}

}  // namespace hlhgat
