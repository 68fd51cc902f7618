// Eigenvector positional encodings of a batch of graphs, and lambda_max, in
// ONE launch (the config-3 per-sample path).
//
// The reference's CIFAR10SP get() (main_cifar10SP_HL_HGCNN_dense_int3_attpool
// .py:67-125) takes, per sample, eig_pe(L0) = eigenvectors 1 .. k-1 of a dense
// float32 eigh of L0 (lib/Hodge_Dataset.py:97-112) and lambda_max of another
// (lib/Hodge_Dataset.py:282, :782): two O(n^3) LAPACK calls per sample per
// epoch.  A batched rocSOLVER eigh of the block-padded stack took ~3.9 ms per
// 256-graph batch (tridiagonalisation + divide and conquer, 100+ launches,
// and a host sync on its info word; profiles/r04_pipeline/).
//
// Here one workgroup per graph (the grid capped at half the CUs, each
// workgroup taking graphs in turn), everything in fp64:
//   1. Lanczos on L0 = deg .* x - A x with FULL re-orthogonalisation (two
//      classical Gram-Schmidt passes against every previous vector) for n
//      steps, restarting with a fresh vector orthogonal to the basis when an
//      invariant subspace closes (disconnected graphs, isolated nodes: the
//      repeated eigenvalues need one restart per extra copy), so Q is a full
//      orthonormal basis and T = Q^T L0 Q is tridiagonal with L0's spectrum;
//   2. the eigenvalues 0 .. k-1 and n-1 of T by wave multisection (Sturm
//      counts at 64 points per pass, tridiag.h);
//   3. T's eigenvectors 1 .. k-1 by inverse iteration (tridiagonal LU with
//      partial pivoting, as LAPACK dstein; eigenvalues closer than 1e-3 ||T||
//      form a cluster whose vectors are orthogonalised in order);
//   4. pe = Q y, written as float32 [n_nodes, ldpe] at the graph's node rows
//      (columns >= n - 1 of a graph with n < k nodes are zero, as the
//      block-padded eigh gives them); lambda_max = the largest eigenvalue.
// A graph whose basis, adjacency and work arrays fit the workgroup's LDS
// (n <~ 120 at CIFAR degrees) runs from the LDS; a larger one keeps them in
// its slice of the workspace (L2-resident) and reads the incidence CSR.
//
// Eigenvectors are defined up to sign (and, inside a cluster of equal
// eigenvalues, up to rotation); the reference flips PE signs at random anyway.
#include "common.h"
#include "tridiag.h"

#include <algorithm>

using namespace hlhgat;

namespace {

constexpr int kEpThreads = 1024;  // 16 waves: the CU's only workgroup (LDS-bound)
constexpr int kEpSplit = 8;       // max lanes per Gram-Schmidt dot product / update sum
constexpr int kEpLdsBytes = 158 * 1024;  // dynamic LDS of a workgroup (+ ~1 KB static: 160 KB)
constexpr int kEpSolvers = 3;            // eigenvectors of T solved at once (LU scratch each)
constexpr int kEpMaxK = 64;

struct EigArgs {
  const int32_t* inc_rowptr;
  const int32_t* inc_edge;
  const int64_t* ei;  // [2][n_edges]
  int64_t n_edges;
  const int64_t* node_ptr;
  int k;
  float* pe;
  int64_t ldpe;
  double* lmax;
  double* ws;  // [n_graphs][ws_per_graph] for graphs that miss the LDS
  int64_t ws_per_graph;
  int64_t n_graphs;
};

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wsum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kEpThreads / 64; ++w) s += red[w];
  return s;
}

// deterministic pseudo-random value in [-1, 1)
__device__ __forceinline__ double hash_unit(uint64_t a, uint64_t b) {
  uint64_t z = a * 0x9E3779B97F4A7C15ull + b * 0xBF58476D1CE4E5B9ull + 0x94D049BB133111EBull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

// per-graph arrays (LDS or workspace)
struct Work {
  double* Q;    // [n][ldq] Lanczos basis, row j = q_j
  double* w;    // [n]
  double* h;    // [n] Gram-Schmidt coefficients
  double* u;    // [kEpSplit][n] partial sums of the split update
  double* al;   // [n]
  double* be;   // [n + 1]
  double* vec;  // [k - 1][n] eigenvectors of T
  double* lu;   // [kEpSolvers][5][n] LU factors + pivots of T - lambda I
  int* rp;      // [n + 1] local adjacency (LDS layout only)
  int* nb;      // [2 E]
  int ldq;
};

__device__ __forceinline__ int64_t small_bytes(int n, int nnz, int k) {
  const int64_t ldq = n + 1;
  return 8 * ((int64_t)n * ldq + (3ll + kEpSplit) * n + (n + 1) + (int64_t)(k - 1) * n +
              (int64_t)kEpSolvers * 5 * n) +
         4 * ((int64_t)n + 1 + nnz);
}

__device__ __forceinline__ Work carve(char* p, int n, int k, bool adjacency) {
  Work W;
  W.ldq = n + 1;
  double* d = reinterpret_cast<double*>(p);
  W.Q = d;
  d += (int64_t)n * W.ldq;
  W.w = d;
  d += n;
  W.h = d;
  d += n;
  W.u = d;
  d += (int64_t)kEpSplit * n;
  W.al = d;
  d += n;
  W.be = d;
  d += n + 1;
  W.vec = d;
  d += (int64_t)(k - 1) * n;
  W.lu = d;
  d += (int64_t)kEpSolvers * 5 * n;
  W.rp = adjacency ? reinterpret_cast<int*>(d) : nullptr;
  W.nb = adjacency ? W.rp + n + 1 : nullptr;
  return W;
}

// w -= sum_{i < cnt} (q_i . w) q_i, twice; returns the coefficient of q_{cnt-1}
// summed over both passes (alpha_j in the Lanczos step).  Both products are
// spread over the whole workgroup: each coefficient by `parts` lanes
// (shuffle-combined), each node's update by `split` slices of the basis
// (partials through u, summed in slice order); 4 independent accumulators
// keep 4 LDS reads in flight per lane.
__device__ __forceinline__ double orthogonalise(const Work& W, int n, int cnt, double* red,
                                                double* nrm2) {
  const int tid = threadIdx.x;
  int parts = 1;
  while (parts < kEpSplit && parts * 2 * cnt <= kEpThreads) parts *= 2;
  int split = 1;
  while (split < kEpSplit && split * 2 * n <= kEpThreads && split * 2 <= cnt) split *= 2;
  const int slice = (cnt + split - 1) / split;
  double last = 0.0;
  for (int pass = 0; pass < 2; ++pass) {
    double ss = 0.0;
    for (int r0 = 0; r0 < cnt * parts; r0 += kEpThreads) {
      const int t = r0 + tid;
      const int i = t / parts, p = t % parts;
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      if (i < cnt) {
        const double* q = W.Q + (int64_t)i * W.ldq;
        int v = p;
        for (; v + 3 * parts < n; v += 4 * parts) {
          s0 += q[v] * W.w[v];
          s1 += q[v + parts] * W.w[v + parts];
          s2 += q[v + 2 * parts] * W.w[v + 2 * parts];
          s3 += q[v + 3 * parts] * W.w[v + 3 * parts];
        }
        for (; v < n; v += parts) s0 += q[v] * W.w[v];
      }
      double s = (s0 + s1) + (s2 + s3);
      for (int o = 1; o < parts; o <<= 1) s += __shfl_xor(s, o, 64);
      if (i < cnt && p == 0) W.h[i] = s;
    }
    __syncthreads();
    last += W.h[cnt - 1];  // h is stable until the next pass's coefficients
    for (int t = tid; t < n * split; t += kEpThreads) {
      const int v = t % n, sl = t / n;
      const int i0 = sl * slice;
      const int i1 = i0 + slice < cnt ? i0 + slice : cnt;
      double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
      int i = i0;
      for (; i + 3 < i1; i += 4) {
        s0 += W.h[i] * W.Q[(int64_t)i * W.ldq + v];
        s1 += W.h[i + 1] * W.Q[(int64_t)(i + 1) * W.ldq + v];
        s2 += W.h[i + 2] * W.Q[(int64_t)(i + 2) * W.ldq + v];
        s3 += W.h[i + 3] * W.Q[(int64_t)(i + 3) * W.ldq + v];
      }
      for (; i < i1; ++i) s0 += W.h[i] * W.Q[(int64_t)i * W.ldq + v];
      const double sum = (s0 + s1) + (s2 + s3);
      if (split == 1) {
        const double nw = W.w[v] - sum;
        W.w[v] = nw;
        ss += nw * nw;
      } else {
        W.u[(int64_t)sl * n + v] = sum;
      }
    }
    if (split > 1) {
      __syncthreads();
      for (int v = tid; v < n; v += kEpThreads) {
        double sum = 0.0;
        for (int sl = 0; sl < split; ++sl) sum += W.u[(int64_t)sl * n + v];
        const double nw = W.w[v] - sum;
        W.w[v] = nw;
        ss += nw * nw;
      }
    }
    if (pass == 1) {
      // |w|^2 of the result in the pass's closing barrier (no block_sum after)
      ss = wsum(ss);
      if ((tid & 63) == 0) red[tid >> 6] = ss;
    }
    __syncthreads();
  }
  double tot = 0.0;
#pragma unroll
  for (int wv = 0; wv < kEpThreads / 64; ++wv) tot += red[wv];
  *nrm2 = tot;
  return last;
}

// Inverse iteration for one eigenvector of T (one thread): LU of T - lam I
// with partial pivoting (dgttrf), three solves (dgtts2) from a pseudo-random
// start, each followed by a normalisation.
__device__ __forceinline__ void inverse_iteration(const double* al, const double* be, int n, double lam,
                                  double tiny, double* lu, double* x, uint64_t seed) {
  double* dl = lu;
  double* d = lu + n;
  double* du = lu + 2 * n;
  double* du2 = lu + 3 * n;
  double* piv = lu + 4 * n;
  for (int i = 0; i < n; ++i) {
    d[i] = al[i] - lam;
    du[i] = i + 1 < n ? be[i + 1] : 0.0;
    dl[i] = du[i];
    du2[i] = 0.0;
    piv[i] = 0.0;
  }
  for (int i = 0; i + 1 < n; ++i) {
    if (fabs(d[i]) >= fabs(dl[i])) {  // no interchange
      const double f = d[i] != 0.0 ? dl[i] / d[i] : 0.0;
      dl[i] = f;
      d[i + 1] -= f * du[i];
    } else {  // interchange rows i and i + 1
      const double f = d[i] / dl[i];
      d[i] = dl[i];
      dl[i] = f;
      const double t = du[i];
      du[i] = d[i + 1];
      d[i + 1] = t - f * d[i + 1];
      if (i + 2 < n) {
        du2[i] = du[i + 1];
        du[i + 1] = -f * du[i + 1];
      }
      piv[i] = 1.0;
    }
  }
  for (int i = 0; i < n; ++i)
    if (fabs(d[i]) < tiny) d[i] = d[i] < 0.0 ? -tiny : tiny;
  for (int i = 0; i < n; ++i) x[i] = hash_unit(seed, (uint64_t)i);
  for (int it = 0; it < 3; ++it) {
    for (int i = 0; i + 1 < n; ++i) {  // L
      if (piv[i] == 0.0) {
        x[i + 1] -= dl[i] * x[i];
      } else {
        const double t = x[i];
        x[i] = x[i + 1];
        x[i + 1] = t - dl[i] * x[i + 1];
      }
    }
    x[n - 1] /= d[n - 1];  // U
    if (n > 1) x[n - 2] = (x[n - 2] - du[n - 2] * x[n - 1]) / d[n - 2];
    for (int i = n - 3; i >= 0; --i) x[i] = (x[i] - du[i] * x[i + 1] - du2[i] * x[i + 2]) / d[i];
    double mx = 0.0;
    for (int i = 0; i < n; ++i) mx = fmax(mx, fabs(x[i]));
    const double sc = mx > 0.0 ? 1.0 / mx : 1.0;
    double s = 0.0;
    for (int i = 0; i < n; ++i) {
      x[i] *= sc;
      s += x[i] * x[i];
    }
    const double r = s > 0.0 ? 1.0 / sqrt(s) : 0.0;
    for (int i = 0; i < n; ++i) x[i] *= r;
  }
}

template <bool SMALL>
__device__ __forceinline__ void eig_pe_graph(const EigArgs& a, int g, int64_t n0, int n, char* base, double* red,
                             double* lam, int* clus) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int k = a.k;
  const int ebase = a.inc_rowptr[n0];
  const int nnz = a.inc_rowptr[n0 + n] - ebase;
  Work W = carve(base, n, k, SMALL);
  if (SMALL) {
    for (int v = tid; v <= n; v += kEpThreads) W.rp[v] = a.inc_rowptr[n0 + v] - ebase;
    for (int v = tid; v < n; v += kEpThreads) {
      const int e0 = a.inc_rowptr[n0 + v], e1 = a.inc_rowptr[n0 + v + 1];
      for (int p = e0; p < e1; ++p) {
        const int64_t e = a.inc_edge[p];
        const int64_t i = a.ei[e], j = a.ei[a.n_edges + e];
        W.nb[p - ebase] = (int)((i == n0 + v ? j : i) - n0);
      }
    }
  }
  (void)nnz;
  auto apply = [&](const double* x, double* y) {  // y = L0 x
    for (int v = tid; v < n; v += kEpThreads) {
      double s;
      if (SMALL) {
        const int p0 = W.rp[v], p1 = W.rp[v + 1];
        s = (double)(p1 - p0) * x[v];
        for (int p = p0; p < p1; ++p) s -= x[W.nb[p]];
      } else {
        const int e0 = a.inc_rowptr[n0 + v], e1 = a.inc_rowptr[n0 + v + 1];
        s = (double)(e1 - e0) * x[v];
        for (int p = e0; p < e1; ++p) {
          const int64_t e = a.inc_edge[p];
          const int64_t i = a.ei[e], j = a.ei[a.n_edges + e];
          s -= x[(i == n0 + v ? j : i) - n0];
        }
      }
      y[v] = s;
    }
  };
  // ---- 1. Lanczos, full re-orthogonalisation, restarts -------------------------
  double nrm = 0.0;
  for (int v = tid; v < n; v += kEpThreads) {
    const double x = 1.0 + (double)(((uint64_t)v * 2654435761ull) % 1000ull) * 1e-3;
    W.Q[v] = x;
    nrm += x * x;
  }
  nrm = sqrt(block_sum(nrm, red));
  for (int v = tid; v < n; v += kEpThreads) W.Q[v] /= nrm;
  if (tid == 0) W.be[0] = 0.0;
  __syncthreads();
  double scale = 1.0;
  for (int j = 0; j < n; ++j) {
    apply(W.Q + (int64_t)j * W.ldq, W.w);
    __syncthreads();
    double ww;
    const double alpha = orthogonalise(W, n, j + 1, red, &ww);
    if (tid == 0) W.al[j] = alpha;
    scale = fmax(scale, fabs(alpha));
    if (j + 1 == n) break;
    double b = sqrt(ww);
    scale = fmax(scale, b);
    double* qn = W.Q + (int64_t)(j + 1) * W.ldq;
    if (b > 1e-10 * scale) {
      if (tid == 0) W.be[j + 1] = b;
      for (int v = tid; v < n; v += kEpThreads) qn[v] = W.w[v] / b;
    } else {
      // invariant subspace closed: continue from a pseudo-random vector
      // orthogonal to the basis (T splits here: be = 0)
      if (tid == 0) W.be[j + 1] = 0.0;
      for (int attempt = 0;; ++attempt) {
        for (int v = tid; v < n; v += kEpThreads)
          W.w[v] = hash_unit(((uint64_t)g << 20) + (uint64_t)j, (uint64_t)v + 7919ull * attempt);
        __syncthreads();
        orthogonalise(W, n, j + 1, red, &ww);
        b = sqrt(ww);
        if (b > 1e-3 || attempt >= 8) break;  // |r| ~ sqrt(n / 3) before the projection
      }
      for (int v = tid; v < n; v += kEpThreads) qn[v] = b > 0.0 ? W.w[v] / b : 0.0;
    }
    __syncthreads();
  }
  __syncthreads();
  // ---- 2. eigenvalues 0 .. m-1 and n-1 of T -----------------------------------
  const int m = k < n ? k : n;  // eigenpairs 0 .. m-1 (0 is not output)
  double glo, ghi;
  gershgorin(W.al, W.be, n, glo, ghi);
  const double tnorm = fmax(fabs(glo), fabs(ghi));
  const double tol = 4e-16 * fmax(tnorm, 1e-300);
  for (int t = wave; t <= m; t += kEpThreads / 64) {
    const int idx = t < m ? t : n - 1;
    const double ev = wave_eigenvalue(W.al, W.be, n, idx, glo, ghi, tol);
    if (lane == 0) lam[t] = ev;  // lam[m] = lambda_max
  }
  __syncthreads();
  if (tid == 0) {
    a.lmax[g] = lam[m];
    // clusters (dstein: ORTOL = 1e-3 ||T||) and the perturbation that keeps
    // equal eigenvalues' factorisations distinct
    const double eps = 2.220446049250313e-16;
    for (int i = 1; i < m; ++i) {
      clus[i] = (i > 1 && lam[i] - lam[i - 1] < 1e-3 * tnorm) ? clus[i - 1] : i;
      if (i > 1 && lam[i] - lam[i - 1] < 10.0 * eps * fmax(tnorm, 1.0))
        lam[i] = lam[i - 1] + 10.0 * eps * fmax(tnorm, 1.0);
    }
  }
  __syncthreads();
  // ---- 3. eigenvectors 1 .. m-1 of T --------------------------------------------
  const double tiny = 2.220446049250313e-16 * fmax(tnorm, 1e-300);
  for (int s0 = 1; s0 < m; s0 += kEpSolvers) {
    const int i = s0 + tid;
    if (tid < kEpSolvers && i < m)
      inverse_iteration(W.al, W.be, n, lam[i], tiny, W.lu + (int64_t)tid * 5 * n,
                        W.vec + (int64_t)(i - 1) * n, ((uint64_t)g << 8) + (uint64_t)i);
  }
  __syncthreads();
  // members of a cluster: orthogonalised against the earlier members, in order
  for (int i = 2; i < m; ++i) {
    if (clus[i] == i) continue;
    double* x = W.vec + (int64_t)(i - 1) * n;
    for (int pass = 0; pass < 2; ++pass) {
      for (int j = clus[i]; j < i; ++j) {
        const double* y = W.vec + (int64_t)(j - 1) * n;
        double d = 0.0;
        for (int v = tid; v < n; v += kEpThreads) d += x[v] * y[v];
        d = block_sum(d, red);
        for (int v = tid; v < n; v += kEpThreads) x[v] -= d * y[v];
        __syncthreads();
      }
      double ss = 0.0;
      for (int v = tid; v < n; v += kEpThreads) ss += x[v] * x[v];
      const double r = sqrt(block_sum(ss, red));
      for (int v = tid; v < n; v += kEpThreads) x[v] = r > 0.0 ? x[v] / r : 0.0;
      __syncthreads();
    }
  }
  // ---- 4. pe = Q y ----------------------------------------------------------------
  for (int v = tid; v < n; v += kEpThreads) {
    float* out = a.pe + (n0 + v) * a.ldpe;
    for (int i = 1; i < k; ++i) {
      double s = 0.0;
      if (i < m) {
        const double* y = W.vec + (int64_t)(i - 1) * n;
        for (int j = 0; j < n; ++j) s += W.Q[(int64_t)j * W.ldq + v] * y[j];
      }
      out[i - 1] = (float)s;
    }
  }
}

__global__ __launch_bounds__(kEpThreads) void k_eig_pe(EigArgs a) {
  extern __shared__ __align__(16) char ep_lds[];
  __shared__ double red[kEpThreads / 64];
  __shared__ double lam[kEpMaxK + 1];
  __shared__ int clus[kEpMaxK + 1];
  for (int64_t g = blockIdx.x; g < a.n_graphs; g += gridDim.x) {
    const int64_t n0 = a.node_ptr[g];
    const int n = (int)(a.node_ptr[g + 1] - n0);
    if (n <= 0) {
      if (threadIdx.x == 0) a.lmax[g] = 0.0;
      continue;
    }
    const int nnz = a.inc_rowptr[n0 + n] - a.inc_rowptr[n0];
    if (small_bytes(n, nnz, a.k) <= kEpLdsBytes)
      eig_pe_graph<true>(a, (int)g, n0, n, ep_lds, red, lam, clus);
    else
      eig_pe_graph<false>(a, (int)g, n0, n,
                          reinterpret_cast<char*>(a.ws + (int64_t)blockIdx.x * a.ws_per_graph),
                          red, lam, clus);
    __syncthreads();  // the next graph reuses the LDS
  }
}

int64_t per_graph_doubles(int64_t max_nodes, int k) {
  const int64_t n = max_nodes;
  return n * (n + 1) + (3 + kEpSplit) * n + (n + 1) + (int64_t)(k - 1) * n +
         (int64_t)kEpSolvers * 5 * n + 8;
}

// One workgroup per CU (a workgroup holds a whole CU's LDS); graphs beyond
// the grid are taken in turn by the same workgroups, so the workspace (for
// graphs too large for the LDS) is one slice per WORKGROUP.  The full chip:
// the training step's one-launch BatchNorms beside it no longer need their
// grids resident (bn.hip: a workgroup whose wait runs out hands its rows to
// the finaliser), so nothing has to be throttled for them.
int64_t eig_pe_grid(int64_t n_graphs) {
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return std::max<int64_t>(1, std::min<int64_t>(n_graphs, cus));
}

}  // namespace

extern "C" int64_t hlhgat_eig_pe_workspace_bytes(int64_t n_graphs, int64_t max_nodes, int k) {
  if (n_graphs < 0 || max_nodes < 0 || k < 2 || k > kEpMaxK) return 0;
  return (int64_t)sizeof(double) * eig_pe_grid(n_graphs) * per_graph_doubles(max_nodes, k);
}

extern "C" int hlhgat_eig_pe(const int32_t* inc_rowptr, const int32_t* inc_edge,
                             const int64_t* edge_index, int64_t n_edges, int64_t n_nodes,
                             const int64_t* node_ptr, int64_t n_graphs, int64_t max_nodes, int k,
                             float* pe, int64_t ldpe, double* lmax, void* workspace,
                             int64_t workspace_bytes, void* stream) {
  HLH_CHECK_ARG(k >= 2 && k <= kEpMaxK, "eig_pe: k must be 2..%d", kEpMaxK);
  HLH_CHECK_ARG(n_graphs >= 0 && n_nodes >= 0 && n_edges >= 0 && max_nodes >= 0,
                "eig_pe: bad sizes");
  HLH_CHECK_ARG(ldpe >= k - 1, "eig_pe: ldpe < k - 1");
  if (n_graphs == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(inc_rowptr && node_ptr && lmax && pe && workspace &&
                    (n_edges == 0 || (inc_edge && edge_index)),
                "eig_pe: NULL pointer");
  HLH_CHECK_ARG(workspace_bytes >= hlhgat_eig_pe_workspace_bytes(n_graphs, max_nodes, k),
                "eig_pe: workspace too small");
  static bool attr = false;
  if (!attr) {
    HLH_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_eig_pe),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kEpLdsBytes));
    attr = true;
  }
  EigArgs a{};
  a.inc_rowptr = inc_rowptr;
  a.inc_edge = inc_edge;
  a.ei = edge_index;
  a.n_edges = n_edges;
  a.node_ptr = node_ptr;
  a.k = k;
  a.pe = pe;
  a.ldpe = ldpe;
  a.lmax = lmax;
  a.ws = reinterpret_cast<double*>(workspace);
  a.ws_per_graph = per_graph_doubles(max_nodes, k);
  a.n_graphs = n_graphs;
  const int64_t grid = eig_pe_grid(n_graphs);
  hipLaunchKernelGGL(k_eig_pe, dim3((unsigned)grid), dim3(kEpThreads), kEpLdsBytes,
                     as_stream(stream), a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}
