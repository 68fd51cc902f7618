// Lane replay of a captured training step.
//
// A captured step is two chains of kernels -- the node chain and the edge
// chain of the HL blocks (lib/Hodge_ST_Model.py:608-633) -- issued on two
// streams and exchanging features once per block.  hipGraphLaunch of the
// whole two-branch graph makes the HIP runtime spread the nodes over its
// hardware queues and resolve every cross-queue edge as it writes the
// packets, ~7 us of host-side lag per node (profiles/r03_n_launch_lead.txt):
// the GPU catches up with the packet writer and waits.  A LINEAR graph takes
// the runtime's single-queue path (the whole packet list written at once).
//
// So the captured graph is split into one linear graph per lane (the stream
// each kernel was captured on: the capture stream is lane 0, every other
// stream lane 1).  Each lane keeps its kernels in a topological order of the
// whole DAG; an edge from lane A's node u to lane B's node v becomes a
// signal kernel after u in A (one thread bumps a device counter) and a wait
// kernel before v in B (one thread polls it).  The lanes replay on two
// dedicated streams, which the build checks to sit on distinct hardware
// queues (a handshake that would time out on a shared queue).
//
// Recording: while hlhgat_capture_record(1) is on, every kernel this library
// launches on a capturing stream notes (graph node, stream) -- the stream is
// not part of a graph node.  Nodes launched by others (torch's fill, memsets)
// take the lane of their latest predecessor.
#include "common.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <queue>
#include <unordered_map>
#include <vector>

namespace hlhgat {

std::atomic<int> g_capture_record{0};

namespace {
std::mutex g_rec_mu;
std::unordered_map<hipGraphNode_t, hipStream_t> g_rec;
}  // namespace

void capture_note_slow(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t n = 0;
  if (hipStreamGetCaptureInfo_v2(s, &st, &id, &g, &deps, &n) != hipSuccess) return;
  if (st != hipStreamCaptureStatusActive || n != 1 || !deps) return;
  std::lock_guard<std::mutex> lk(g_rec_mu);
  g_rec[deps[0]] = s;
}

}  // namespace hlhgat

using namespace hlhgat;

// ---------------------------------------------------------------------------
// signal / wait kernels (one thread each; plain vector-memory atomics)
// ---------------------------------------------------------------------------
// (an atomic add, as the BatchNorm grid barrier's arrivals: performed where
// every XCD's polling load sees it, not left in this XCD's L2)
__global__ void k_lane_signal(unsigned* flag) {
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// Waits until the signal counter reaches this wait's own replay count.  Gives
// up after `timeout` wall-clock ticks and raises `code` in `err` (the results
// of the step are then unusable; the counters stay in step, one increment
// per replay each, so later replays are unaffected).
__global__ void k_lane_wait(const unsigned* flag, unsigned* own, unsigned* err, unsigned code,
                            long long timeout, unsigned* timeouts) {
  if (threadIdx.x == 0) {
    const unsigned want = __hip_atomic_load(own, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_store(own, want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = wall_clock64();
    while ((int)(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
      if (wall_clock64() - t0 > timeout) {
        if (err) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}

namespace {

constexpr int kMaxLanes = 4;

struct Lanes {
  int dev = 0, n_lanes = 0;
  hipGraph_t g[kMaxLanes] = {};
  hipGraphExec_t ex[kMaxLanes] = {};
  hipStream_t st[kMaxLanes] = {};
  hipEvent_t ev_start = nullptr, ev_done[kMaxLanes] = {};
  unsigned* words = nullptr;  // [n_sig signals][n_wait own counters][n_wait timeouts]
  int n_nodes[kMaxLanes] = {}, n_sig = 0, n_wait = 0, n_virtual = 0;
};

// Dedicated lane streams per device, checked once to sit on distinct queues.
std::mutex g_lane_mu;
std::unordered_map<int, std::vector<hipStream_t>> g_lane_streams;

long long ticks_per_ms(int dev) {
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
    khz = 100000;  // gfx9 wall clock: 100 MHz
  return (long long)khz;
}

hipKernelNodeParams kparams(void* fn, void** args) {
  hipKernelNodeParams p{};
  p.func = fn;
  p.gridDim = dim3(1);
  p.blockDim = dim3(64);
  p.sharedMemBytes = 0;
  p.kernelParams = args;
  p.extra = nullptr;
  return p;
}

// Lane 0 waits for lane L on a scratch counter with a short timeout; on a
// queue shared with lane 0 the signal sits behind the wait and it times out.
int handshake(hipStream_t a, hipStream_t b, int dev, bool* ok) {
  unsigned* w = nullptr;
  HLH_CHECK_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&w), 4 * sizeof(unsigned),
                                      hipDeviceMallocUncached));
  HLH_CHECK_HIP(hipMemset(w, 0, 4 * sizeof(unsigned)));
  HLH_CHECK_HIP(hipDeviceSynchronize());
  const long long to = 50 * ticks_per_ms(dev);
  hipLaunchKernelGGL(k_lane_wait, dim3(1), dim3(64), 0, a, (const unsigned*)w, w + 1, w + 2, 1u, to,
                     w + 3);
  hipLaunchKernelGGL(k_lane_signal, dim3(1), dim3(64), 0, b, w);
  HLH_CHECK_LAUNCH();
  HLH_CHECK_HIP(hipStreamSynchronize(a));
  HLH_CHECK_HIP(hipStreamSynchronize(b));
  unsigned h[4];
  HLH_CHECK_HIP(hipMemcpy(h, w, sizeof(h), hipMemcpyDeviceToHost));
  HLH_CHECK_HIP(hipFree(w));
  *ok = h[2] == 0u && h[0] == 1u && h[1] == 1u;
  return HLHGAT_OK;
}

int lane_streams(int dev, int n, std::vector<hipStream_t>& out) {
  std::lock_guard<std::mutex> lk(g_lane_mu);
  auto it = g_lane_streams.find(dev);
  if (it != g_lane_streams.end() && (int)it->second.size() >= n) {
    out.assign(it->second.begin(), it->second.begin() + n);
    return HLHGAT_OK;
  }
  std::vector<hipStream_t> s;
  if (it != g_lane_streams.end()) s = it->second;
  // a few attempts: a stream that shares lane 0's hardware queue is kept
  // (never destroyed while other work may use it) but not used as a lane
  std::vector<hipStream_t> spare;
  for (int attempt = 0; (int)s.size() < n && attempt < 4 * kMaxLanes; ++attempt) {
    // a stream with a CU mask (all CUs) owns its hardware queue: the HIP
    // runtime maps plain streams onto its queues dynamically, and two lanes
    // mapped onto one queue would serialise (a wait in the first lane then
    // spins on a signal queued behind it)
    hipStream_t x = nullptr;
    int n_cu = 0;
    HLH_CHECK_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    std::vector<uint32_t> mask((size_t)(n_cu + 31) / 32, 0u);
    for (int c = 0; c < n_cu; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
    HLH_CHECK_HIP(hipExtStreamCreateWithCUMask(&x, (uint32_t)mask.size(), mask.data()));
    bool ok = true;
    for (hipStream_t y : s) {
      bool pair_ok = false;
      int rc = handshake(y, x, dev, &pair_ok);
      if (rc != HLHGAT_OK) return rc;
      ok = ok && pair_ok;
    }
    if (ok) s.push_back(x);
    else spare.push_back(x);
  }
  g_lane_streams[dev] = s;
  HLH_CHECK_ARG((int)s.size() >= n,
                "lanes: could not get %d streams on distinct hardware queues", n);
  out.assign(s.begin(), s.begin() + n);
  return HLHGAT_OK;
}

void destroy(Lanes* L) {
  if (!L) return;
  for (int i = 0; i < kMaxLanes; ++i) {
    if (L->ex[i]) (void)hipGraphExecDestroy(L->ex[i]);
    if (L->g[i]) (void)hipGraphDestroy(L->g[i]);
    if (L->ev_done[i]) (void)hipEventDestroy(L->ev_done[i]);
  }
  if (L->ev_start) (void)hipEventDestroy(L->ev_start);
  if (L->words) (void)hipFree(L->words);
  delete L;
}

}  // namespace

extern "C" int hlhgat_capture_record(int on) {
  if (on) {
    std::lock_guard<std::mutex> lk(g_rec_mu);
    g_rec.clear();
  }
  g_capture_record.store(on ? 1 : 0, std::memory_order_relaxed);
  return HLHGAT_OK;
}

extern "C" int hlhgat_capture_recorded(int64_t* n) {
  HLH_CHECK_ARG(n, "capture_recorded: NULL pointer");
  std::lock_guard<std::mutex> lk(g_rec_mu);
  *n = (int64_t)g_rec.size();
  return HLHGAT_OK;
}

extern "C" int hlhgat_lanes_build(void* graph, void* origin_stream, int n_lanes,
                                  hlhgat_lanes_t* out) {
  HLH_CHECK_ARG(graph && out, "lanes_build: NULL graph or output");
  HLH_CHECK_ARG(n_lanes == 2, "lanes_build: n_lanes must be 2 (got %d)", n_lanes);
  *out = nullptr;
  hipGraph_t G = reinterpret_cast<hipGraph_t>(graph);
  hipStream_t origin = as_stream(origin_stream);

  size_t n = 0;
  HLH_CHECK_HIP(hipGraphGetNodes(G, nullptr, &n));
  HLH_CHECK_ARG(n > 0, "lanes_build: empty graph");
  std::vector<hipGraphNode_t> nodes(n);
  HLH_CHECK_HIP(hipGraphGetNodes(G, nodes.data(), &n));
  std::unordered_map<hipGraphNode_t, int> id;
  for (size_t i = 0; i < n; ++i) id[nodes[i]] = (int)i;

  std::vector<hipGraphNodeType> type(n);
  std::vector<std::vector<int>> preds(n), succs(n);
  for (size_t i = 0; i < n; ++i) {
    HLH_CHECK_HIP(hipGraphNodeGetType(nodes[i], &type[i]));
    const hipGraphNodeType t = type[i];
    HLH_CHECK_ARG(t == hipGraphNodeTypeKernel || t == hipGraphNodeTypeMemcpy ||
                      t == hipGraphNodeTypeMemset || t == hipGraphNodeTypeEmpty,
                  "lanes_build: unsupported graph node type %d", (int)t);
    size_t nd = 0;
    HLH_CHECK_HIP(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd));
    std::vector<hipGraphNode_t> d(nd);
    if (nd) HLH_CHECK_HIP(hipGraphNodeGetDependencies(nodes[i], d.data(), &nd));
    for (auto x : d) {
      auto f = id.find(x);
      HLH_CHECK_ARG(f != id.end(), "lanes_build: dependency outside the graph");
      preds[i].push_back(f->second);
      succs[f->second].push_back((int)i);
    }
  }

  // topological order, ties by node order (the capture's insertion order)
  std::vector<int> indeg(n), topo;
  std::priority_queue<int, std::vector<int>, std::greater<int>> ready;
  for (size_t i = 0; i < n; ++i) {
    indeg[i] = (int)preds[i].size();
    if (!indeg[i]) ready.push((int)i);
  }
  while (!ready.empty()) {
    const int v = ready.top();
    ready.pop();
    topo.push_back(v);
    for (int w : succs[v])
      if (--indeg[w] == 0) ready.push(w);
  }
  HLH_CHECK_ARG(topo.size() == n, "lanes_build: graph has a cycle");
  std::vector<int> rank(n);
  for (size_t r = 0; r < n; ++r) rank[topo[r]] = (int)r;

  // lanes: the recorded stream, else the latest predecessor's lane
  std::vector<int> lane(n, 0);
  int n_rec = 0;
  {
    std::lock_guard<std::mutex> lk(g_rec_mu);
    for (int v : topo) {
      auto f = g_rec.find(nodes[v]);
      if (f != g_rec.end()) {
        lane[v] = f->second == origin ? 0 : 1;
        ++n_rec;
      } else if (!preds[v].empty()) {
        int best = preds[v][0];
        for (int u : preds[v])
          if (rank[u] > rank[best]) best = u;
        lane[v] = lane[best];
      }
    }
  }
  HLH_CHECK_ARG(n_rec > 0, "lanes_build: no launch was recorded during the capture");

  // real nodes per lane in topological order; empty nodes are dropped and
  // their dependencies pass through them
  const int NL = n_lanes;
  std::vector<int> pos(n, -1);
  std::vector<std::vector<int>> seq(NL);
  int n_virtual = 0;
  for (int v : topo) {
    if (type[v] == hipGraphNodeTypeEmpty) {
      ++n_virtual;
      continue;
    }
    pos[v] = (int)seq[lane[v]].size();
    seq[lane[v]].push_back(v);
  }
  // the furthest position needed in each lane by node v (through empty nodes)
  auto need_of = [&](int v, std::vector<int>& need) {
    std::fill(need.begin(), need.end(), -1);
    std::vector<int> stack(preds[v].begin(), preds[v].end());
    std::vector<char> seen;
    while (!stack.empty()) {
      const int u = stack.back();
      stack.pop_back();
      if (type[u] == hipGraphNodeTypeEmpty) {
        if (seen.empty()) seen.assign(n, 0);
        if (seen[u]) continue;
        seen[u] = 1;
        for (int x : preds[u]) stack.push_back(x);
        continue;
      }
      need[lane[u]] = std::max(need[lane[u]], pos[u]);
    }
  };

  // waits before each node, signals after each node (by lane position)
  struct Wait { int lane_from, pos_from; };
  std::vector<std::vector<std::vector<Wait>>> waits(NL);
  std::vector<std::vector<int>> sig_slot(NL);
  for (int L = 0; L < NL; ++L) {
    waits[L].resize(seq[L].size());
    sig_slot[L].assign(seq[L].size(), -1);
  }
  int n_sig = 0, n_wait = 0;
  std::vector<int> need(NL);
  for (int L = 0; L < NL; ++L) {
    std::vector<int> done(NL, -1);
    for (size_t p = 0; p < seq[L].size(); ++p) {
      need_of(seq[L][p], need);
      for (int M = 0; M < NL; ++M) {
        if (M == L || need[M] <= done[M]) continue;
        waits[L][p].push_back(Wait{M, need[M]});
        done[M] = need[M];
        ++n_wait;
      }
    }
  }
  for (int L = 0; L < NL; ++L)
    for (auto& wl : waits[L])
      for (auto& w : wl)
        if (sig_slot[w.lane_from][w.pos_from] < 0) sig_slot[w.lane_from][w.pos_from] = n_sig++;

  int dev = 0;
  HLH_CHECK_HIP(hipGetDevice(&dev));
  Lanes* Lx = new Lanes();
  Lx->dev = dev;
  Lx->n_lanes = NL;
  Lx->n_sig = n_sig;
  Lx->n_wait = n_wait;
  Lx->n_virtual = n_virtual;
  auto fail = [&](int rc) {
    destroy(Lx);
    return rc;
  };
  {
    const size_t words = (size_t)std::max(1, n_sig + 2 * n_wait);
    // uncached device memory: the counters are written by one XCD and polled
    // by another; no L2 may hold a stale copy (a counter in cached memory was
    // observed to stay invisible to the polling XCD for seconds)
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&Lx->words), words * sizeof(unsigned),
                              hipDeviceMallocUncached) != hipSuccess ||
        hipMemset(Lx->words, 0, words * sizeof(unsigned)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      set_error("lanes_build: counter allocation failed");
      return fail(HLHGAT_EHIP);
    }
  }
  unsigned* err = device_error_word();
  const long long timeout = 2000 * ticks_per_ms(dev);  // 2 s
  const unsigned code = HLHGAT_DEVERR_LANE_WAIT;
  unsigned* sig_words = Lx->words;
  unsigned* own_words = Lx->words + n_sig;
  unsigned* tmo_words = own_words + n_wait;
  int wait_k = 0;
  // kernel-node arguments stay alive until every graph is instantiated
  struct NodeArgs {
    const unsigned* f;
    unsigned* own;
    unsigned* err;
    unsigned code;
    long long timeout;
    unsigned* tmo;
    void* args[6];
  };
  std::vector<NodeArgs> argstore((size_t)(n_sig + n_wait) + 1);
  size_t argk = 0;

  for (int L = 0; L < NL; ++L) {
    hipGraph_t C = nullptr;
    if (hipGraphClone(&C, G) != hipSuccess) {
      set_error("lanes_build: hipGraphClone failed");
      return fail(HLHGAT_EHIP);
    }
    Lx->g[L] = C;
    // the clone's copies of this lane's nodes; every other node goes
    std::vector<hipGraphNode_t> mine(seq[L].size()), drop;
    for (size_t p = 0; p < seq[L].size(); ++p)
      if (hipGraphNodeFindInClone(&mine[p], nodes[seq[L][p]], C) != hipSuccess) {
        set_error("lanes_build: hipGraphNodeFindInClone failed");
        return fail(HLHGAT_EHIP);
      }
    for (size_t i = 0; i < n; ++i) {
      if (type[i] != hipGraphNodeTypeEmpty && lane[i] == L) continue;
      hipGraphNode_t c = nullptr;
      if (hipGraphNodeFindInClone(&c, nodes[i], C) != hipSuccess) {
        set_error("lanes_build: hipGraphNodeFindInClone failed");
        return fail(HLHGAT_EHIP);
      }
      drop.push_back(c);
    }
    for (auto c : drop)
      if (hipGraphDestroyNode(c) != hipSuccess) {
        set_error("lanes_build: hipGraphDestroyNode failed");
        return fail(HLHGAT_EHIP);
      }
    size_t ne = 0;
    if (hipGraphGetEdges(C, nullptr, nullptr, &ne) != hipSuccess) {
      set_error("lanes_build: hipGraphGetEdges failed");
      return fail(HLHGAT_EHIP);
    }
    if (ne) {
      std::vector<hipGraphNode_t> from(ne), to(ne);
      if (hipGraphGetEdges(C, from.data(), to.data(), &ne) != hipSuccess ||
          hipGraphRemoveDependencies(C, from.data(), to.data(), ne) != hipSuccess) {
        set_error("lanes_build: removing the captured edges failed");
        return fail(HLHGAT_EHIP);
      }
    }
    // the lane as one chain: [waits] node [signal] ...
    hipGraphNode_t prev = nullptr;
    auto link = [&](hipGraphNode_t x) -> bool {
      if (prev && hipGraphAddDependencies(C, &prev, &x, 1) != hipSuccess) return false;
      prev = x;
      return true;
    };
    for (size_t p = 0; p < seq[L].size(); ++p) {
      for (const Wait& w : waits[L][p]) {
        const int slot = sig_slot[w.lane_from][w.pos_from];
        NodeArgs& A = argstore.at(argk++);
        A.f = sig_words + slot;
        A.tmo = tmo_words + wait_k;
        A.own = own_words + wait_k++;
        A.err = err;
        A.code = code;
        A.timeout = timeout;
        A.args[0] = &A.f;
        A.args[1] = &A.own;
        A.args[2] = &A.err;
        A.args[3] = &A.code;
        A.args[4] = &A.timeout;
        A.args[5] = &A.tmo;
        hipKernelNodeParams kp = kparams(reinterpret_cast<void*>(k_lane_wait), A.args);
        hipGraphNode_t wn = nullptr;
        if (hipGraphAddKernelNode(&wn, C, prev ? &prev : nullptr, prev ? 1 : 0, &kp) !=
            hipSuccess) {
          set_error("lanes_build: adding a wait node failed");
          return fail(HLHGAT_EHIP);
        }
        prev = wn;
      }
      if (!link(mine[p])) {
        set_error("lanes_build: linking the lane failed");
        return fail(HLHGAT_EHIP);
      }
      const int slot = sig_slot[L][p];
      if (slot >= 0) {
        NodeArgs& A = argstore.at(argk++);
        A.own = sig_words + slot;
        A.args[0] = &A.own;
        hipKernelNodeParams kp = kparams(reinterpret_cast<void*>(k_lane_signal), A.args);
        hipGraphNode_t sn = nullptr;
        if (hipGraphAddKernelNode(&sn, C, &prev, 1, &kp) != hipSuccess) {
          set_error("lanes_build: adding a signal node failed");
          return fail(HLHGAT_EHIP);
        }
        prev = sn;
      }
    }
    Lx->n_nodes[L] = (int)seq[L].size();
    if (hipGraphInstantiate(&Lx->ex[L], C, nullptr, nullptr, 0) != hipSuccess) {
      set_error("lanes_build: hipGraphInstantiate failed");
      return fail(HLHGAT_EHIP);
    }
  }
  std::vector<hipStream_t> st;
  int rc = lane_streams(dev, NL, st);
  if (rc != HLHGAT_OK) return fail(rc);
  for (int L = 0; L < NL; ++L) {
    Lx->st[L] = st[L];
    // the runtime's per-exec launch resources are prepared here, not at the
    // first launch: a lane whose first launch stalls the host (e.g. on an
    // allocation that waits for the device) while the other lane already
    // spins on its signal would hold that wait until its timeout
    if (hipGraphUpload(Lx->ex[L], st[L]) != hipSuccess ||
        hipStreamSynchronize(st[L]) != hipSuccess) {
      set_error("lanes_build: hipGraphUpload failed");
      return fail(HLHGAT_EHIP);
    }
    if (hipEventCreateWithFlags(&Lx->ev_done[L], hipEventDisableTiming) != hipSuccess) {
      set_error("lanes_build: hipEventCreate failed");
      return fail(HLHGAT_EHIP);
    }
  }
  if (hipEventCreateWithFlags(&Lx->ev_start, hipEventDisableTiming) != hipSuccess) {
    set_error("lanes_build: hipEventCreate failed");
    return fail(HLHGAT_EHIP);
  }
  *out = reinterpret_cast<hlhgat_lanes_t>(Lx);
  return HLHGAT_OK;
}

extern "C" int hlhgat_graph_kernel_count(void* graph, const char* name_part, int64_t* kernels,
                                         int64_t* matching) {
  HLH_CHECK_ARG(graph && name_part && kernels && matching, "graph_kernel_count: NULL argument");
  hipGraph_t G = reinterpret_cast<hipGraph_t>(graph);
  size_t n = 0;
  HLH_CHECK_HIP(hipGraphGetNodes(G, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  if (n) HLH_CHECK_HIP(hipGraphGetNodes(G, nodes.data(), &n));
  *kernels = 0;
  *matching = 0;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    HLH_CHECK_HIP(hipGraphNodeGetType(nd, &t));
    if (t != hipGraphNodeTypeKernel) continue;
    ++*kernels;
    hipKernelNodeParams kp{};
    if (hipGraphKernelNodeGetParams(nd, &kp) != hipSuccess || !kp.func) continue;
    const char* nm = hipKernelNameRefByPtr(kp.func, nullptr);
    if (nm && std::strstr(nm, name_part)) ++*matching;
  }
  return HLHGAT_OK;
}

extern "C" int hlhgat_lanes_info(hlhgat_lanes_t h, int64_t* info, int n_info) {
  HLH_CHECK_ARG(h && info && n_info >= 0, "lanes_info: NULL handle or output");
  const Lanes* L = reinterpret_cast<const Lanes*>(h);
  int64_t v[8] = {L->n_lanes, L->n_nodes[0], L->n_nodes[1], L->n_sig, L->n_wait, L->n_virtual,
                  0, 0};
  for (int i = 0; i < n_info && i < 8; ++i) info[i] = v[i];
  return HLHGAT_OK;
}

extern "C" int hlhgat_lanes_counters(hlhgat_lanes_t h, unsigned* out, int n) {
  HLH_CHECK_ARG(h && out, "lanes_counters: NULL handle or output");
  Lanes* L = reinterpret_cast<Lanes*>(h);
  HLH_CHECK_ARG(n == L->n_sig + 2 * L->n_wait, "lanes_counters: expected %d words, got %d",
                L->n_sig + 2 * L->n_wait, n);
  for (int i = 0; i < L->n_lanes; ++i) HLH_CHECK_HIP(hipStreamSynchronize(L->st[i]));
  if (n) HLH_CHECK_HIP(hipMemcpy(out, L->words, sizeof(unsigned) * n, hipMemcpyDeviceToHost));
  return HLHGAT_OK;
}

extern "C" int hlhgat_lanes_launch(hlhgat_lanes_t h, void* stream) {
  HLH_CHECK_ARG(h, "lanes_launch: NULL handle");
  Lanes* L = reinterpret_cast<Lanes*>(h);
  hipStream_t s = as_stream(stream);
  HLH_CHECK_HIP(hipEventRecord(L->ev_start, s));
  for (int i = 0; i < L->n_lanes; ++i) {
    HLH_CHECK_HIP(hipStreamWaitEvent(L->st[i], L->ev_start, 0));
    HLH_CHECK_HIP(hipGraphLaunch(L->ex[i], L->st[i]));
    HLH_CHECK_HIP(hipEventRecord(L->ev_done[i], L->st[i]));
  }
  for (int i = 0; i < L->n_lanes; ++i) HLH_CHECK_HIP(hipStreamWaitEvent(s, L->ev_done[i], 0));
  return HLHGAT_OK;
}

extern "C" int hlhgat_lanes_destroy(hlhgat_lanes_t h) {
  if (!h) return HLHGAT_OK;
  Lanes* L = reinterpret_cast<Lanes*>(h);
  // the lanes may still run a replay: wait for it before freeing the counters
  for (int i = 0; i < L->n_lanes; ++i)
    if (L->st[i]) (void)hipStreamSynchronize(L->st[i]);
  destroy(L);
  return HLHGAT_OK;
}
