// Multi-level graph coarsening (MLGC) for the attention-pooling heads: the
// graclus matching and the fine -> coarse node / edge assignment, as native
// HOST code (host pointers, no stream).  MLGC is dataset preprocessing in the
// reference (lib/Hodge_Dataset.py:241-353, run once per graph before
// training), so it sits beside the other collate-time builders
// (hlhgat_halo_tiles) rather than on the device: one pass over the edges,
// O(E log deg) for the matching and O(E) hashing for the edge map, no Python
// per-edge loops.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
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

// One MLGC level for a whole batch of graphs (SuperpixelPipeline.batch, the
// reference's per-sample get(), main_cifar10SP...:67-125): per graph, graclus
// on L0's pattern (the i<j edge list both ways, unit weights, node order
// perm) and the fine -> coarse map -- hlhgat_graclus + hlhgat_mlgc_map per
// graph, the graphs spread over n_threads host threads.  All indices are
// LOCAL to their graph; graph g's nodes are [node_ptr[g], node_ptr[g+1]) of
// perm / c_node, its edges [edge_ptr[g], edge_ptr[g+1]) of edges ([2][E]) /
// c_edge, and its coarse edges are written from column edge_ptr[g] of
// coarse_edges ([2][E], row stride E), coarse_n[g] / coarse_e[g] sizes.
extern "C" int hlhgat_mlgc_batch(int64_t n_graphs, const int64_t* node_ptr,
                                 const int64_t* edge_ptr, const int64_t* edges,
                                 const int64_t* perm, int n_threads, int64_t* c_node,
                                 float* c_edge, int64_t* coarse_edges, int64_t* coarse_n,
                                 int64_t* coarse_e) {
  HLH_CHECK_ARG(n_graphs >= 0 && node_ptr && edge_ptr && coarse_n && coarse_e,
                "mlgc_batch: bad arguments");
  const int64_t N = n_graphs ? node_ptr[n_graphs] : 0, E = n_graphs ? edge_ptr[n_graphs] : 0;
  HLH_CHECK_ARG(node_ptr[0] == 0 && edge_ptr[0] == 0 && (N == 0 || (perm && c_node)) &&
                    (E == 0 || (edges && c_edge && coarse_edges)),
                "mlgc_batch: bad offsets or NULL arrays");
  for (int64_t g = 0; g < n_graphs; ++g)
    HLH_CHECK_ARG(node_ptr[g + 1] >= node_ptr[g] && edge_ptr[g + 1] >= edge_ptr[g],
                  "mlgc_batch: offsets of graph %lld decrease", (long long)g);
  std::atomic<int64_t> next{0};
  std::atomic<int> rc_first{HLHGAT_OK};
  std::mutex msg_mu;
  std::string msg;
  auto worker = [&]() {
    std::vector<int64_t> both, ei, cl, ce;
    for (;;) {
      const int64_t g = next.fetch_add(1);
      if (g >= n_graphs || rc_first.load() != HLHGAT_OK) return;
      const int64_t n0 = node_ptr[g], n = node_ptr[g + 1] - n0;
      const int64_t e0 = edge_ptr[g], m = edge_ptr[g + 1] - e0;
      ei.resize((size_t)(2 * m));
      both.resize((size_t)(4 * m));
      for (int64_t k = 0; k < m; ++k) {
        const int64_t i = edges[e0 + k], j = edges[E + e0 + k];
        ei[(size_t)k] = i;
        ei[(size_t)(m + k)] = j;
        both[(size_t)k] = i;                // rows: i then j
        both[(size_t)(m + k)] = j;
        both[(size_t)(2 * m + k)] = j;      // cols: j then i
        both[(size_t)(3 * m + k)] = i;
      }
      cl.resize((size_t)n);
      ce.resize((size_t)std::max<int64_t>(2 * m, 2));
      int64_t n1 = 0, ne = 0;
      int rc = hlhgat_graclus(both.data(), nullptr, 2 * m, n, perm + n0, cl.data());
      if (rc == HLHGAT_OK)
        rc = hlhgat_mlgc_map(cl.data(), n, ei.data(), m, c_node + n0, c_edge + e0, ce.data(),
                             &n1, &ne);
      if (rc != HLHGAT_OK) {
        int ok = HLHGAT_OK;
        if (rc_first.compare_exchange_strong(ok, rc)) {
          std::lock_guard<std::mutex> lk(msg_mu);
          msg = std::string("graph ") + std::to_string(g) + ": " + hlhgat_last_error();
        }
        return;
      }
      for (int64_t k = 0; k < ne; ++k) {
        coarse_edges[e0 + k] = ce[(size_t)k];
        coarse_edges[E + e0 + k] = ce[(size_t)(m + k)];
      }
      coarse_n[g] = n1;
      coarse_e[g] = ne;
    }
  };
  const int T = std::max(1, std::min<int>(n_threads, (int)std::min<int64_t>(n_graphs, 64)));
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  if (rc_first.load() != HLHGAT_OK) {
    hlhgat::set_error("mlgc_batch: %s", msg.c_str());
    return rc_first.load();
  }
  return HLHGAT_OK;
}
