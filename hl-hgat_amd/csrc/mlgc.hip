// Multi-level graph coarsening (MLGC) for the attention-pooling heads: the
// graclus matching and the fine -> coarse node / edge assignment, as native
// HOST code (host pointers, no stream).  MLGC is dataset preprocessing in the
// reference (lib/Hodge_Dataset.py:241-353, run once per graph before
// training), so it sits beside the other collate-time builders
// (hlhgat_halo_tiles) rather than on the device: one pass over the edges,
// O(E log deg) for the matching and O(E) hashing for the edge map, no Python
// per-edge loops.
#include <algorithm>
#include <cstdint>
#include <limits>
#include <numeric>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace {

// (lo, hi) coarse-node pair -> one 64-bit key (both < 2^31 by the size check)
inline uint64_t pair_key(int64_t lo, int64_t hi) {
  return ((uint64_t)lo << 32) | (uint64_t)(uint32_t)hi;
}

}  // namespace

// Greedy graclus matching (torch_cluster 1.6.0 graclus_cluster, its weighted
// branch -- the reference always passes a weight, ones_like for MLGC --
// called at lib/Hodge_Dataset.py:252 and :311): self-loops dropped, every
// node's neighbours in ascending column order, nodes visited in perm order;
// an unmatched node u keeps the LAST unmatched neighbour whose weight is >=
// the best so far (best starts at 0, so zero weights match) and both get id
// min(u, v); with no unmatched neighbour u stays alone with id u.  Restated
// from torch_cluster's published graclus_cpu (not in the reference tree):
// parity unpinned.
extern "C" int hlhgat_graclus(const int64_t* edge_index, const double* weight, int64_t n_edges,
                              int64_t n_nodes, const int64_t* perm, int64_t* cluster) {
  HLH_CHECK_ARG(n_edges >= 0 && n_nodes >= 0, "graclus: bad sizes");
  HLH_CHECK_ARG(cluster && (n_nodes == 0 || perm) && (n_edges == 0 || edge_index),
                "graclus: NULL pointer");
  const int64_t* row = edge_index;
  const int64_t* col = edge_index + n_edges;
  std::vector<int64_t> deg((size_t)n_nodes + 1, 0);
  for (int64_t e = 0; e < n_edges; ++e) {
    HLH_CHECK_ARG(row[e] >= 0 && row[e] < n_nodes && col[e] >= 0 && col[e] < n_nodes,
                  "graclus: edge %lld out of range", (long long)e);
    if (row[e] != col[e]) ++deg[(size_t)row[e] + 1];
  }
  std::partial_sum(deg.begin(), deg.end(), deg.begin());
  // CSR with (col, original position) per row, so a stable sort by column
  // reproduces the (row, col) lexsort of the restatement
  std::vector<int64_t> nb((size_t)deg[(size_t)n_nodes]);
  std::vector<double> nw(nb.size());
  {
    std::vector<int64_t> fill(deg.begin(), deg.end() - 1);
    for (int64_t e = 0; e < n_edges; ++e) {
      if (row[e] == col[e]) continue;
      const int64_t p = fill[(size_t)row[e]]++;
      nb[(size_t)p] = e;
    }
    for (int64_t u = 0; u < n_nodes; ++u) {
      const int64_t b = deg[(size_t)u], f = deg[(size_t)u + 1];
      std::stable_sort(nb.begin() + b, nb.begin() + f,
                       [&](int64_t x, int64_t y) { return col[x] < col[y]; });
      for (int64_t p = b; p < f; ++p) {
        const int64_t e = nb[(size_t)p];
        nw[(size_t)p] = weight ? weight[e] : 1.0;
        nb[(size_t)p] = col[e];
      }
    }
  }
  for (int64_t u = 0; u < n_nodes; ++u) cluster[u] = -1;
  for (int64_t i = 0; i < n_nodes; ++i) {
    const int64_t u = perm[i];
    HLH_CHECK_ARG(u >= 0 && u < n_nodes, "graclus: perm[%lld] out of range", (long long)i);
    if (cluster[u] >= 0) continue;
    int64_t best = u;
    double wbest = 0.0;
    for (int64_t p = deg[(size_t)u]; p < deg[(size_t)u + 1]; ++p) {
      const int64_t v = nb[(size_t)p];
      if (cluster[v] >= 0) continue;
      if (nw[(size_t)p] >= wbest) {  // ties: the LAST such neighbour
        best = v;
        wbest = nw[(size_t)p];
      }
    }
    cluster[u] = cluster[best] = std::min(u, best);
  }
  return HLHGAT_OK;
}

// Fine -> coarse assignment of one MLGC level (lib/Hodge_Dataset.py:254-275):
// c_node = rank of the node's cluster id among the distinct ids; an edge whose
// ends share a coarse node gets +inf, the others the index of the coarse edge
// (min, max), numbered in first-seen edge order.
extern "C" int hlhgat_mlgc_map(const int64_t* cluster, int64_t n_nodes, const int64_t* edge_index,
                               int64_t n_edges, int64_t* c_node, float* c_edge,
                               int64_t* coarse_edges, int64_t* n_coarse_nodes,
                               int64_t* n_coarse_edges) {
  HLH_CHECK_ARG(n_edges >= 0 && n_nodes >= 0 && n_nodes < INT32_MAX, "mlgc_map: bad sizes");
  HLH_CHECK_ARG(n_coarse_nodes && n_coarse_edges && (n_nodes == 0 || (cluster && c_node)) &&
                    (n_edges == 0 || (edge_index && c_edge && coarse_edges)),
                "mlgc_map: NULL pointer");
  // cluster ids are node ids: rank = prefix count of the ids present
  std::vector<int64_t> rank((size_t)n_nodes + 1, 0);
  for (int64_t u = 0; u < n_nodes; ++u) {
    HLH_CHECK_ARG(cluster[u] >= 0 && cluster[u] < n_nodes, "mlgc_map: cluster id out of range");
    rank[(size_t)cluster[u] + 1] = 1;
  }
  std::partial_sum(rank.begin(), rank.end(), rank.begin());
  for (int64_t u = 0; u < n_nodes; ++u) c_node[u] = rank[(size_t)cluster[u]];
  const int64_t* row = edge_index;
  const int64_t* col = edge_index + n_edges;
  std::unordered_map<uint64_t, int64_t> key;
  key.reserve((size_t)n_edges);
  int64_t ne = 0;
  for (int64_t i = 0; i < n_edges; ++i) {
    HLH_CHECK_ARG(row[i] >= 0 && row[i] < n_nodes && col[i] >= 0 && col[i] < n_nodes,
                  "mlgc_map: edge %lld out of range", (long long)i);
    const int64_t a = c_node[row[i]], b = c_node[col[i]];
    if (a == b) {
      c_edge[i] = std::numeric_limits<float>::infinity();
      continue;
    }
    const int64_t lo = std::min(a, b), hi = std::max(a, b);
    auto it = key.emplace(pair_key(lo, hi), ne);
    if (it.second) {
      coarse_edges[ne] = lo;
      coarse_edges[n_edges + ne] = hi;
      ++ne;
    }
    c_edge[i] = (float)it.first->second;
  }
  *n_coarse_nodes = rank[(size_t)n_nodes];
  *n_coarse_edges = ne;
  return HLHGAT_OK;
}
