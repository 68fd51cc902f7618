// On-device Hodge Laplacian builder for block-diagonal batches of simplex
// graphs.
//
// The reference builds, per graph, the dense boundary B1 [N, E], the dense
// L0 = B1 B1^T, its largest eigenvalue with torch.linalg.eigh, and then the
// dense L0 = 2 B1 B1^T / lmax and L1 = 2 B1^T B1 / lmax, keeping nonzeros with
// dense_to_sparse (lib/Hodge_Dataset.py:451-468, :780-799): O(N^3) for lmax
// and an E x E dense L1 (10 GB at BASELINE config 5).  Here, from the edge
// list and the incidence CSR alone:
//   * k_lanczos_lmax: lmax of every graph's L0 in ONE launch, one
//     wave per graph: Lanczos on L0 x = deg .* x - A x (fp64, three-term
//     recurrence with local re-orthogonalisation, <= 64 steps), then the
//     largest eigenvalue of the tridiagonal matrix by Sturm-sequence bisection;
//   * k_hodge_l0_rows / k_hodge_l1_rows: the sparse L0 / L1 rows in CSR
//     (columns ascending, as dense_to_sparse orders them) with the
//     reference's float32 entries fl(fl(2 v) / lmax): L0 row v = {v: deg(v),
//     u in N(v): -1}; L1 row e = (i, j) = the merge of the incidence lists of
//     i and j: {e: 2, f sharing its tail or head with e's tail or head: +1,
//     tail-to-head: -1}.
// Row sizes (prefix sums) come from the incidence CSR; no sort, no atomics.
#include "common.h"
#include "tridiag.h"

using namespace hlhgat;

namespace {

constexpr int kLzThreads = 64;          // one wave per graph
constexpr int kLzMaxSteps = 64;
constexpr int kLzLdsBytes = 48 * 1024;  // a graph's vectors + local adjacency, when they fit

struct LanczosArgs {
  const int32_t* inc_rowptr;  // incidence CSR (node -> incident edge ids, ascending)
  const int32_t* inc_edge;
  const int64_t* ei;          // [2][n_edges]
  int64_t n_edges;
  const int64_t* node_ptr;    // [n_graphs + 1]
  int steps;
  double* Q;                  // [3][n_nodes] q_{j-1}, q_j, w for graphs that miss the LDS
  int64_t n_nodes;
  double* lmax;               // [n_graphs]
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Lanczos on one graph's L0 (n nodes, local ids; apply(x, y): y = L0 x) by
// the three-term recurrence with a local re-orthogonalisation against q_j
// (one extra dot product per step) and no global one: loss of orthogonality
// only adds ghost copies of converged Ritz values, it does not move the
// largest one past lambda_max (Paige), so lambda_max converges as with full
// re-orthogonalisation at 3 wave reductions per step instead of 2 (j + 1)
// block reductions (full Gram-Schmidt made this kernel ~3 ms for 256 CIFAR
// graphs, profiles/r04_pipeline/).  Lane l owns the nodes l, l + 64, ... in
// every loop, so q_{j-1}, q_j and w are lane-private except for the
// neighbour reads of apply.  Returns the size k of the tridiagonal (al, be).
template <typename Apply>
__device__ int lanczos(Apply apply, int n, int m, double* qp, double* q, double* w, double* al,
                       double* be) {
  const int lane = threadIdx.x;
  // deterministic start vector with a component along every eigenvector
  double nrm = 0.0;
  for (int v = lane; v < n; v += kLzThreads) {
    const double x = 1.0 + (double)(((uint64_t)v * 2654435761ull) % 1000ull) * 1e-3;
    q[v] = x;
    qp[v] = 0.0;
    nrm += x * x;
  }
  nrm = sqrt(wave_sum(nrm));
  for (int v = lane; v < n; v += kLzThreads) q[v] /= nrm;
  __syncthreads();
  int k = m;
  double beta = 0.0;
  for (int j = 0; j < m; ++j) {
    apply(q, w);
    double d = 0.0;
    for (int v = lane; v < n; v += kLzThreads) {
      const double t = w[v] - beta * qp[v];
      w[v] = t;
      d += t * q[v];
    }
    double alpha = wave_sum(d);
    d = 0.0;
    for (int v = lane; v < n; v += kLzThreads) {
      const double t = w[v] - alpha * q[v];
      w[v] = t;
      d += t * q[v];
    }
    const double c = wave_sum(d);  // local re-orthogonalisation
    alpha += c;
    d = 0.0;
    for (int v = lane; v < n; v += kLzThreads) {
      const double t = w[v] - c * q[v];
      w[v] = t;
      d += t * t;
    }
    const double b = sqrt(wave_sum(d));
    if (lane == 0) al[j] = alpha;
    if (j + 1 >= m) break;
    const double scale = fabs(alpha) > 1.0 ? fabs(alpha) : 1.0;
    if (b <= 1e-12 * scale) {  // invariant subspace found: T is complete
      k = j + 1;
      break;
    }
    if (lane == 0) be[j + 1] = b;
    for (int v = lane; v < n; v += kLzThreads) {
      qp[v] = q[v];
      q[v] = w[v] / b;
    }
    beta = b;
    __syncthreads();  // apply reads the neighbours' q
  }
  __syncthreads();
  return k;
}

// lambda_max of every graph's L0 = deg .* x - A x, one wave per graph.  A
// graph whose vectors and local adjacency (node -> neighbour ids) fit in
// kLzLdsBytes runs from the LDS (the CIFAR / ZINC / peptide graphs: ~8 KB);
// a larger one (brain skeleton, TSP) walks the incidence CSR in global
// memory with its vectors in the workspace.
__global__ __launch_bounds__(kLzThreads) void k_lanczos_lmax(LanczosArgs a) {
  extern __shared__ __align__(16) unsigned char lz_lds[];
  __shared__ double al[kLzMaxSteps + 1], be[kLzMaxSteps + 2];
  const int g = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t n0 = a.node_ptr[g], n1 = a.node_ptr[g + 1];
  const int n = (int)(n1 - n0);
  const int m = n < a.steps ? n : a.steps;
  int k = 0;
  if (n > 0) {
    const int base = a.inc_rowptr[n0];
    const int nnz = a.inc_rowptr[n1] - base;  // 2 E of this graph
    const int64_t need = 24ll * n + 4ll * (n + 1) + 4ll * nnz;
    if (need <= kLzLdsBytes) {
      double* qp = reinterpret_cast<double*>(lz_lds);
      double* q = qp + n;
      double* w = q + n;
      int* rp = reinterpret_cast<int*>(w + n);
      int* nb = rp + n + 1;
      for (int v = lane; v <= n; v += kLzThreads) rp[v] = a.inc_rowptr[n0 + v] - base;
      for (int v = lane; v < n; v += kLzThreads) {
        const int e0 = a.inc_rowptr[n0 + v], e1 = a.inc_rowptr[n0 + v + 1];
        for (int p = e0; p < e1; ++p) {
          const int64_t e = a.inc_edge[p];
          const int64_t i = a.ei[e], j = a.ei[a.n_edges + e];
          nb[p - base] = (int)((i == n0 + v ? j : i) - n0);
        }
      }
      __syncthreads();
      auto apply = [&](const double* x, double* y) {
        for (int v = lane; v < n; v += kLzThreads) {
          const int p0 = rp[v], p1 = rp[v + 1];
          double s = (double)(p1 - p0) * x[v];
          for (int p = p0; p < p1; ++p) s -= x[nb[p]];
          y[v] = s;
        }
      };
      k = lanczos(apply, n, m, qp, q, w, al, be);
    } else {
      double* qp = a.Q + n0;
      double* q = a.Q + a.n_nodes + n0;
      double* w = a.Q + 2 * a.n_nodes + n0;
      auto apply = [&](const double* x, double* y) {
        for (int v = lane; v < n; v += kLzThreads) {
          const int e0 = a.inc_rowptr[n0 + v], e1 = a.inc_rowptr[n0 + v + 1];
          double s = (double)(e1 - e0) * x[v];
          for (int p = e0; p < e1; ++p) {
            const int64_t e = a.inc_edge[p];
            const int64_t i = a.ei[e], j = a.ei[a.n_edges + e];
            s -= x[(i == n0 + v ? j : i) - n0];
          }
          y[v] = s;
        }
      };
      k = lanczos(apply, n, m, qp, q, w, al, be);
    }
  }
  // Gershgorin bounds, then multisection for the largest eigenvalue: the 64
  // lanes count the Sturm sequence at 64 interior points of [lo, hi] at once
  // (bisection by one lane cost ~0.4 ms of serial fp64 divides per launch)
  double lo, hi;
  gershgorin(al, be, k, lo, hi);
  if (k > 0) hi = wave_eigenvalue(al, be, k, k - 1, lo, hi, 1e-15 * fmax(1.0, fabs(hi)));
  if (lane == 0) a.lmax[g] = n > 0 ? hi : 0.0;
}

struct BuildArgs {
  const int32_t* inc_rowptr;
  const int32_t* inc_edge;
  const int64_t* ei;
  int64_t n_edges, n_nodes;
  const float* lam_node;   // [n_nodes] lmax (float32) of each node's graph
  const int32_t* rp;       // output row pointer of this operator
  int32_t* col;
  float* val;
  int64_t cap;             // entries col / val hold
  unsigned* err;           // device error word (HLHGAT_DEVERR_HODGE_SIZE)
};

// A row whose end lies past the buffers (row sizes the caller supplied that
// do not match the graph: duplicate edges, self-loops) writes nothing and
// raises HLHGAT_DEVERR_HODGE_SIZE; rp is a prefix sum of non-negative sizes,
// so rp[row + 1] <= cap puts the whole row in range.  The thread of the last
// row also checks rp[n_rows] == cap: sizes whose total exceeds the device's
// would otherwise leave the tail of col / val unwritten.
__device__ __forceinline__ void hodge_size_error(const BuildArgs& a) {
  if (a.err) __hip_atomic_store(a.err, (unsigned)HLHGAT_DEVERR_HODGE_SIZE, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool row_fits(const BuildArgs& a, int64_t row, int64_t n_rows) {
  if (row == n_rows - 1 && (int64_t)a.rp[n_rows] != a.cap) hodge_size_error(a);
  if ((int64_t)a.rp[row + 1] <= a.cap && a.rp[row] <= a.rp[row + 1]) return true;
  hodge_size_error(a);
  return false;
}

__device__ __forceinline__ float hodge_w(int v, float lam) {
  return (2.0f * (float)v) / lam;  // fl(fl(2 v) / lmax), the reference's float32 entry
}

// L0 row v: its neighbours and itself, columns ascending (selection by
// repeated minimum: rows are short, deg <= a few hundred)
__global__ __launch_bounds__(256) void k_hodge_l0_rows(BuildArgs a) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (v >= a.n_nodes) return;
  const int e0 = a.inc_rowptr[v], e1 = a.inc_rowptr[v + 1];
  const int deg = e1 - e0;
  if (deg == 0) return;  // isolated node: all-zero row, dropped as dense_to_sparse drops zeros
  if (!row_fits(a, v, a.n_nodes)) return;
  const float lam = a.lam_node[v];
  int out = a.rp[v];
  int64_t last = -1;
  for (int k = 0; k <= deg; ++k) {  // deg neighbours + the diagonal
    int64_t best = INT64_MAX;
    if (v > last) best = v;
    for (int p = e0; p < e1; ++p) {
      const int64_t e = a.inc_edge[p];
      const int64_t i = a.ei[e], j = a.ei[a.n_edges + e];
      const int64_t u = (i == v) ? j : i;
      if (u > last && u < best) best = u;
    }
    a.col[out] = (int32_t)best;
    a.val[out] = hodge_w(best == v ? deg : -1, lam);
    ++out;
    last = best;
  }
}

// L1 row e = (i, j): merge of the ascending incidence lists of i and j
__global__ __launch_bounds__(256) void k_hodge_l1_rows(BuildArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= a.n_edges) return;
  if (!row_fits(a, e, a.n_edges)) return;
  const int64_t i = a.ei[e], j = a.ei[a.n_edges + e];
  const float lam = a.lam_node[i];
  int p = a.inc_rowptr[i], pe = a.inc_rowptr[i + 1];
  int q = a.inc_rowptr[j], qe = a.inc_rowptr[j + 1];
  int out = a.rp[e];
  while (p < pe || q < qe) {
    const int32_t fp = p < pe ? a.inc_edge[p] : INT32_MAX;
    const int32_t fq = q < qe ? a.inc_edge[q] : INT32_MAX;
    const int32_t f = fp < fq ? fp : fq;
    int v;
    if (f == (int32_t)e) {
      v = 2;
      ++p;
      ++q;  // e is in both lists
    } else {
      const int64_t fi = a.ei[f], fj = a.ei[a.n_edges + f];
      // shared node s: +1 when s is the tail of both or the head of both
      if (fp == f) {  // shares node i (e's tail)
        v = (fi == i) ? 1 : -1;
        ++p;
      } else {        // shares node j (e's head)
        v = (fj == j) ? 1 : -1;
        ++q;
      }
    }
    a.col[out] = f;
    a.val[out] = hodge_w(v, lam);
    ++out;
  }
}

// row sizes: L0 deg(v) + [deg > 0]; L1 deg(i) + deg(j) - 1
__global__ __launch_bounds__(256) void k_hodge_row_sizes(const int32_t* inc_rowptr,
                                                         const int64_t* ei, int64_t n_edges,
                                                         int64_t n_nodes, int32_t* sz0,
                                                         int32_t* sz1) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < n_nodes) {
    const int d = inc_rowptr[t + 1] - inc_rowptr[t];
    sz0[t] = d > 0 ? d + 1 : 0;
  }
  if (t < n_edges) {
    const int64_t i = ei[t], j = ei[n_edges + t];
    sz1[t] = (inc_rowptr[i + 1] - inc_rowptr[i]) + (inc_rowptr[j + 1] - inc_rowptr[j]) - 1;
  }
}

}  // namespace

extern "C" int64_t hlhgat_hodge_lmax_workspace_bytes(int64_t n_nodes, int steps) {
  if (n_nodes < 0 || steps < 1 || steps > kLzMaxSteps) return 0;
  return (int64_t)sizeof(double) * n_nodes * 3;
}

extern "C" int hlhgat_hodge_lmax(const int32_t* inc_rowptr, const int32_t* inc_edge,
                                 const int64_t* edge_index, int64_t n_edges, int64_t n_nodes,
                                 const int64_t* node_ptr, int64_t n_graphs, int steps,
                                 double* lmax, void* workspace, int64_t workspace_bytes,
                                 void* stream) {
  HLH_CHECK_ARG(steps >= 1 && steps <= kLzMaxSteps, "hodge_lmax: steps must be 1..%d",
                kLzMaxSteps);
  HLH_CHECK_ARG(n_graphs >= 0 && n_nodes >= 0 && n_edges >= 0, "hodge_lmax: bad sizes");
  if (n_graphs == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(inc_rowptr && node_ptr && lmax && workspace && (n_edges == 0 || (inc_edge && edge_index)),
                "hodge_lmax: NULL pointer");
  HLH_CHECK_ARG(workspace_bytes >= hlhgat_hodge_lmax_workspace_bytes(n_nodes, steps),
                "hodge_lmax: workspace too small");
  LanczosArgs a{};
  a.inc_rowptr = inc_rowptr;
  a.inc_edge = inc_edge;
  a.ei = edge_index;
  a.n_edges = n_edges;
  a.node_ptr = node_ptr;
  a.steps = steps;
  a.Q = reinterpret_cast<double*>(workspace);
  a.n_nodes = n_nodes;
  a.lmax = lmax;
  hipLaunchKernelGGL(k_lanczos_lmax, dim3((unsigned)n_graphs), dim3(kLzThreads), kLzLdsBytes,
                     as_stream(stream), a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_hodge_row_sizes(const int32_t* inc_rowptr, const int64_t* edge_index,
                                      int64_t n_edges, int64_t n_nodes, int32_t* sizes_l0,
                                      int32_t* sizes_l1, void* stream) {
  HLH_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && inc_rowptr && sizes_l0 && sizes_l1 &&
                    (n_edges == 0 || edge_index),
                "hodge_row_sizes: bad arguments");
  const int64_t n = n_nodes > n_edges ? n_nodes : n_edges;
  if (n == 0) return HLHGAT_OK;
  hipLaunchKernelGGL(k_hodge_row_sizes, dim3((unsigned)ceil_div(n, (int64_t)256)), dim3(256), 0,
                     as_stream(stream), inc_rowptr, edge_index, n_edges, n_nodes, sizes_l0,
                     sizes_l1);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_hodge_build(const int32_t* inc_rowptr, const int32_t* inc_edge,
                                  const int64_t* edge_index, int64_t n_edges, int64_t n_nodes,
                                  const float* lam_node, const int32_t* rowptr_l0,
                                  int32_t* col_l0, float* val_l0, int64_t cap_l0,
                                  const int32_t* rowptr_l1, int32_t* col_l1, float* val_l1,
                                  int64_t cap_l1, void* stream) {
  HLH_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && inc_rowptr && lam_node && rowptr_l0 &&
                    rowptr_l1 && cap_l0 >= 0 && cap_l1 >= 0 &&
                    (n_edges == 0 || (inc_edge && edge_index && col_l0 && val_l0 &&
                                      col_l1 && val_l1)),
                "hodge_build: bad arguments");
  BuildArgs a{inc_rowptr, inc_edge, edge_index, n_edges, n_nodes, lam_node, rowptr_l0, col_l0,
              val_l0, cap_l0, device_error_word()};
  hipStream_t s = as_stream(stream);
  if (n_nodes > 0) {
    hipLaunchKernelGGL(k_hodge_l0_rows, dim3((unsigned)ceil_div(n_nodes, (int64_t)256)),
                       dim3(256), 0, s, a);
    HLH_CHECK_LAUNCH();
  }
  if (n_edges > 0) {
    a.rp = rowptr_l1;
    a.col = col_l1;
    a.val = val_l1;
    a.cap = cap_l1;
    hipLaunchKernelGGL(k_hodge_l1_rows, dim3((unsigned)ceil_div(n_edges, (int64_t)256)),
                       dim3(256), 0, s, a);
    HLH_CHECK_LAUNCH();
  }
  return HLHGAT_OK;
}
