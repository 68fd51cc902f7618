// Host-side torch binding of the hot path: C++ autograd nodes over the C-ABI
// of include/hlhgat.h.
//
// Python autograd Functions + ctypes cost 20-70 us of host time per op, which
// made the ZINC-scale training step host-bound.  Here each
// composite layer is ONE C++ autograd node whose forward / backward issue the
// whole launch sequence from C++:
//   conv_bn     HodgeLaguerreConv / HodgeChebConv (+ BatchNorm (+ ReLU))
//               lib/Hodge_Cheb_Conv.py:480-515 / :394-439, lib/Hodge_ST_Model.py:556-566
//   bn_act      gnn.BatchNorm / BatchNorm1d (+ ReLU), training statistics
//   linear      Linear over a split reduction axis (Linear(cat[a, b]))
//   mlp2        NodeEdgeInt WV_*: Linear->BN->ReLU->Linear->BN->ReLU
//               lib/Hodge_Cheb_Conv.py:276-289,307-308
//   node_from_edges / edge_from_nodes   (1/D)|B1| x_s and |B1|^T x_t / 2
//               lib/Hodge_Cheb_Conv.py:294-295
// Every kernel runs on torch's current HIP stream; no CPU fallback exists.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <algorithm>
#include <mutex>
#include <optional>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/hlhgat.h"

namespace {

using torch::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;
using OptT = std::optional<Tensor>;

inline void* stream_of(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.get_device()).stream();
}
inline const int32_t* iptr(const std::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr<int32_t>() : nullptr;
}
inline void chk(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "hlhgat: ", what, " failed: ", hlhgat_last_error());
}
inline int64_t ld_of(const Tensor& t) {
  return std::max<int64_t>({t.stride(0), t.size(1), (int64_t)1});
}
inline bool has(const OptT& t) { return t.has_value() && t->defined(); }
inline const float* fptr(const OptT& t) { return has(t) ? t->data_ptr<float>() : nullptr; }
inline float* mfptr(const OptT& t) { return has(t) ? t->data_ptr<float>() : nullptr; }
inline Tensor rows2d(const Tensor& t) {
  if (t.stride(1) != 1 || t.stride(0) < t.size(1)) return t.contiguous();
  return t;
}
inline void req(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "hlhgat: ", name, " must be on a ROCm device (no CPU fallback)");
  TORCH_CHECK(t.scalar_type() == at::kFloat, "hlhgat: ", name, " must be float32");
}

// Argument position -> autograd edge index.  In C++ custom functions
// needs_input_grad() indexes EDGES: a Tensor argument is always an edge, an
// optional<Tensor> only when defined, each TensorList element is one, and any
// other argument none.  Backward still returns one gradient per position.
struct EdgeMap {
  std::vector<int64_t> e;
  int64_t n = 0;
  void tensor() { e.push_back(n++); }
  void opt(const OptT& t) { e.push_back(has(t) ? n++ : -1); }
  void list(at::TensorList l) {
    for (size_t i = 0; i < l.size(); ++i) e.push_back(n++);
  }
  void other() { e.push_back(-1); }
};
inline bool need(AutogradContext* ctx, int64_t pos) {
  const auto em = ctx->saved_data["edges"].toIntVector();
  return pos < (int64_t)em.size() && em[pos] >= 0 && ctx->needs_input_grad(em[pos]);
}

// ---------------------------------------------------------------------------
// raw launches
// ---------------------------------------------------------------------------
struct Csr {
  Tensor rowptr, col;
  OptT val;
  int64_t nnz;
};

// hlhgat_halo_t over the halo-tile tensors of an operator (see hlhgat.h);
// bounds = {max_halo, max_rows, max_nnz}
hlhgat_halo_t make_halo(const Tensor& tile, const Tensor& ptr, const Tensor& cols,
                        const Tensor& srp, const Tensor& lcol, const Tensor& sval,
                        const std::vector<int64_t>& bounds, const Tensor& hdr) {
  hlhgat_halo_t h{};
  if (!lcol.defined()) return h;
  TORCH_CHECK(tile.scalar_type() == at::kInt && ptr.scalar_type() == at::kInt &&
                  cols.scalar_type() == at::kInt && srp.scalar_type() == at::kInt &&
                  lcol.element_size() == 2 && bounds.size() == 3 && hdr.defined() &&
                  hdr.scalar_type() == at::kInt,
              "hlhgat: halo tiles must be int32 (tile_ptr, halo_ptr, halo, srp), 16-bit lcol "
              "and 3 bounds");
  h.hdr = hdr.data_ptr<int>();
  h.tile_ptr = tile.data_ptr<int>();
  h.halo_ptr = ptr.data_ptr<int>();
  h.halo = cols.data_ptr<int>();
  h.srp = srp.data_ptr<int>();
  h.lcol = reinterpret_cast<const uint16_t*>(lcol.data_ptr());
  h.sval = sval.defined() ? sval.data_ptr<float>() : nullptr;
  h.n_tiles = tile.numel() - 1;
  h.max_halo = (int32_t)bounds[0];
  h.max_rows = (int32_t)bounds[1];
  h.max_nnz = (int32_t)bounds[2];
  return h;
}

// hlhgat_hodge_factor_t over the factor tensors of an L1 operator
// (hlhgat.ops.set_hodge_factor): {node_rowptr, node_edge, node_sign,
// node_order, ends, alpha, edge_order}; an undefined / empty order = natural.
hlhgat_hodge_factor_t make_factor(at::TensorList f, int64_t n_nodes, int64_t n_edges) {
  hlhgat_hodge_factor_t h{};
  TORCH_CHECK(f.size() == 7, "hlhgat: hodge factor needs 7 tensors");
  auto opt_i = [](const Tensor& t) -> const int32_t* {
    return (t.defined() && t.numel() > 0) ? t.data_ptr<int>() : nullptr;
  };
  TORCH_CHECK(f[0].scalar_type() == at::kInt && f[1].scalar_type() == at::kInt &&
                  f[2].scalar_type() == at::kFloat && f[4].scalar_type() == at::kInt &&
                  f[5].scalar_type() == at::kFloat && f[0].numel() == n_nodes + 1 &&
                  f[4].numel() == 2 * n_edges && f[5].numel() == n_edges,
              "hlhgat: bad hodge factor tensors");
  h.node_rowptr = f[0].data_ptr<int>();
  h.node_edge = n_edges ? f[1].data_ptr<int>() : nullptr;
  h.node_sign = n_edges ? f[2].data_ptr<float>() : nullptr;
  h.node_order = opt_i(f[3]);
  h.n_nodes = n_nodes;
  h.ends = f[4].data_ptr<int>();
  h.alpha = f[5].data_ptr<float>();
  h.edge_order = opt_i(f[6]);
  h.n_edges = n_edges;
  return h;
}

// One BN workspace per (device, stream): its arrival counters must not be
// shared by launches that can run concurrently (node / edge chains run on two
// streams, see hlhgat.ops.fork).  Stream-ordered reuse on one stream is safe.
// A workspace that is outgrown is RETIRED, never freed: a hipGraph captured
// earlier on that stream still holds its address, and a replay must not write
// BN counters into memory the caching allocator has handed to another tensor.
// (Sizes grow geometrically, so at most a handful are ever retired.)
// The block is allocated FROM THE KEYED STREAM's pool and zero-filled on that
// stream: a block taken from another stream's pool (the current one, when
// TrainStep reserves a workspace for its capture streams) may still be written
// by kernels queued on that stream after the fill, which would leave counter
// words non-zero and every later launch on the workspace waiting for an
// arrival count it can never reach.
Tensor bn_workspace_for(void* stream, int device, int64_t need) {
  static auto* cache = new std::unordered_map<uintptr_t, Tensor>();  // leaked: outlives HIP teardown
  static auto* retired = new std::vector<Tensor>();
  const uintptr_t key = reinterpret_cast<uintptr_t>(stream) * 64 + device;
  auto it = cache->find(key);
  if (it == cache->end() || it->second.numel() < need) {
    int64_t bytes = std::max<int64_t>(need, 1 << 20);
    if (it != cache->end()) {
      bytes = std::max<int64_t>(bytes, 2 * it->second.numel());
      retired->push_back(it->second);
    }
    Tensor ws;
    {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA g(
          c10::hip::getStreamFromExternalMasqueradingAsCUDA(
              reinterpret_cast<hipStream_t>(stream), (c10::DeviceIndex)device));
      ws = at::empty({bytes}, at::TensorOptions()
                                  .device(at::kCUDA, (c10::DeviceIndex)device)
                                  .dtype(at::kByte));
    }
    chk(hlhgat_zero_fill(ws.data_ptr(), (size_t)ws.numel(), stream), "zero_fill");
    (*cache)[key] = ws;
  }
  return (*cache)[key];
}

Tensor bn_workspace(const Tensor& like, int64_t n, int64_t C) {
  return bn_workspace_for(stream_of(like), like.get_device(), hlhgat_bn_workspace_bytes(n, C));
}

// A workspace for `stream` big enough for C channels, zero-filled and
// synchronised NOW: hlhgat.train.TrainStep calls it before a capture, so the
// zero fill of a workspace first met during the capture is not recorded into
// the graph (and replayed every step; the counters reset themselves).
void bn_workspace_reserve(int64_t stream, int64_t device, int64_t C) {
  void* s = reinterpret_cast<void*>(stream);
  bn_workspace_for(s, (int)device, hlhgat_bn_workspace_bytes(1, C));
  TORCH_CHECK(hipStreamSynchronize((hipStream_t)s) == hipSuccess, "hlhgat: hipStreamSynchronize");
}

// ---------------------------------------------------------------------------
// Gradient bucket (hlhgat.train.TrainStep): parameters are views of one flat
// buffer and their gradients go to the same offsets of one flat gradient
// buffer.  A node computing a parameter gradient writes it straight into a
// FRESH view of that bucket region and returns the view; autograd's
// AccumulateGrad then adopts it as .grad without a copy or an add kernel (it
// steals a gradient whose only reference it holds).  A region is handed out
// once per backward; a second request (a parameter used twice) gets a plain
// tensor so AccumulateGrad's sum stays correct.
// ---------------------------------------------------------------------------
struct BucketEntry {
  Tensor flat;
  int64_t offset;
  int64_t numel;
  bool claimed;
  bool double_use = false;  // claimed twice in one backward (a parameter used twice)
};
std::unordered_map<const void*, BucketEntry>& bucket() {
  static auto* m = new std::unordered_map<const void*, BucketEntry>();
  return *m;
}

void double_claim_hook(const BucketEntry& e);

Tensor grad_like(const Tensor& p) {
  if (!p.defined()) return Tensor();
  auto& m = bucket();
  auto it = m.find(p.data_ptr());
  if (it != m.end() && !it->second.claimed && it->second.numel == p.numel() &&
      it->second.flat.device() == p.device()) {
    it->second.claimed = true;
    return it->second.flat.narrow(0, it->second.offset, p.numel()).view(p.sizes());
  }
  if (it != m.end() && it->second.claimed) {
    it->second.double_use = true;  // never deferred again (deferred_ok)
    double_claim_hook(it->second);
  }
  return at::empty(p.sizes(), p.options());
}
Tensor grad_like(const OptT& p) { return has(p) ? grad_like(*p) : Tensor(); }

void grad_bucket_set(std::vector<Tensor> params, Tensor flat_grad, std::vector<int64_t> offsets) {
  TORCH_CHECK(params.size() == offsets.size(), "hlhgat: grad bucket: params / offsets differ");
  auto& m = bucket();
  m.clear();
  for (size_t i = 0; i < params.size(); ++i)
    m[params[i].data_ptr()] = BucketEntry{flat_grad, offsets[i], params[i].numel(), false};
}
void grad_bucket_begin() {
  for (auto& kv : bucket()) kv.second.claimed = false;
}
// the bucket entry whose gradient region starts at p (nullptr: not in the bucket)
const BucketEntry* bucket_entry_at(const void* p) {
  for (const auto& kv : bucket()) {
    const auto& e = kv.second;
    if (static_cast<const char*>(e.flat.data_ptr()) + e.offset * e.flat.element_size() == p)
      return &e;
  }
  return nullptr;
}
void grad_bucket_clear() { bucket().clear(); }
// parameters whose gradient is not ONE contribution of a HIP node (found by
// TrainStep's first step): never deferred
void grad_bucket_no_defer(std::vector<Tensor> params) {
  auto& m = bucket();
  for (const auto& p : params) {
    auto it = m.find(p.data_ptr());
    if (it != m.end()) it->second.double_use = true;
  }
}

// out[M, N] = sum_b A_b W_b^T + bias
void proj_fwd(const std::vector<const float*>& A, const std::vector<int64_t>& lda,
              const std::vector<const float*>& W, const std::vector<int64_t>& ldw,
              const std::vector<int64_t>& kb, int64_t M, int64_t N, const float* bias,
              Tensor& out, void* s) {
  chk(hlhgat_proj_fwd((int)A.size(), A.data(), lda.data(), W.data(), ldw.data(), kb.data(), M, N,
                      bias, out.data_ptr<float>(), ld_of(out), 0, s),
      "proj_fwd");
}

void proj_bwd_weight(const Tensor& G, const std::vector<const float*>& A,
                     const std::vector<int64_t>& lda, const std::vector<int64_t>& kb,
                     std::vector<float*>& dW, const std::vector<int64_t>& lddw, float* db,
                     void* s) {
  const int nb = (int)A.size();
  const int64_t M = G.size(0), N = G.size(1);
  const int64_t wsf =
      hlhgat_proj_bwd_weight_workspace_floats(nb, kb.data(), M, N, db != nullptr);
  Tensor ws = at::empty({std::max<int64_t>(wsf, 1)}, G.options());
  chk(hlhgat_proj_bwd_weight(nb, G.data_ptr<float>(), ld_of(G), A.data(), lda.data(), kb.data(),
                             M, N, dW.data(), lddw.data(), db, 0, ws.data_ptr<float>(), wsf, s),
      "proj_bwd_weight");
}

// set_fused_bwd(false) (tests): weight and data gradients as separate
// launches instead of hlhgat_proj_bwd's single launch (bitwise the same).
bool& fused_bwd_flag() {
  static bool on = true;
  return on;
}
void set_fused_bwd(bool on) { fused_bwd_flag() = on; }


// One launch for a set of strided rectangles (hlhgat_copy2d_batched);
// src == nullptr zero-fills.
struct CopyBlocks {
  std::vector<const float*> src;
  std::vector<float*> dst;
  std::vector<int64_t> lds, ldd, rows, cols;
  void add(const float* s, int64_t ls, float* d, int64_t ld, int64_t r, int64_t c) {
    src.push_back(s);
    lds.push_back(ls);
    dst.push_back(d);
    ldd.push_back(ld);
    rows.push_back(r);
    cols.push_back(c);
  }
  void run(void* stream) {
    if (src.empty()) return;
    chk(hlhgat_copy2d_batched((int)src.size(), src.data(), lds.data(), dst.data(), ldd.data(),
                              rows.data(), cols.data(), stream),
        "copy2d_batched");
  }
};

// ---------------------------------------------------------------------------
// Deferred split reductions (hlhgat_proj_bwd_defer; hlhgat.train.TrainStep
// turns this on around its backward): a Linear backward whose gradients land
// in the gradient bucket hands its split reduction to the NEXT Linear
// backward on the same stream, which runs it as extra workgroups of its own
// launch, so each backward chain loses one dependent launch per layer.  The
// last one per stream is launched by reduce_flush() after the backward,
// before anything reads the bucket.  Only bucket destinations are deferred:
// autograd adopts those views without reading them (AccumulateGrad steals),
// and nothing else reads the bucket before the flush.
// ---------------------------------------------------------------------------
struct PendingReduce {
  hlhgat_reduce_desc_t desc;
  Tensor ws;  // the split slab the reduction reads: alive until it has run
  void* stream = nullptr;
};
struct DeferState {
  bool on = false;
  std::mutex mu;
  std::unordered_map<void*, PendingReduce> pending;  // by stream
  std::unordered_set<const void*> dests;             // deferred gradient destinations
  bool violation = false;  // a deferred destination was claimed a second time
  std::unordered_set<void*> streams;  // streams that deferred or merged a reduction
  struct Copies {
    CopyBlocks cb;
    std::vector<Tensor> keep;  // the sources, alive until the copies have run
  };
  std::unordered_map<void*, Copies> copies;  // by stream
};
DeferState& defer_state() {
  static auto* d = new DeferState();
  return *d;
}

// a destination that may be deferred: a bucket region of a parameter that is
// not used twice (a second use adds into .grad through AccumulateGrad, which
// must not run before the deferred reduction; TrainStep's first, eager step
// runs without deferral and finds those parameters)
bool deferred_ok(const void* p) {
  if (!p) return true;
  const BucketEntry* e = bucket_entry_at(p);
  return e && !e->double_use;
}

// Gradient copies into the bucket (the NodeEdgeInt unpack) joining the
// deferred work: false (run them now) unless every destination may be deferred.
bool defer_copies(const CopyBlocks& cb, std::initializer_list<Tensor> dests,
                  std::initializer_list<Tensor> keep, void* stream) {
  auto& d = defer_state();
  std::lock_guard<std::mutex> g(d.mu);
  if (!d.on || cb.src.empty()) return false;
  for (const auto& t : dests)
    if (t.defined() && !deferred_ok(t.data_ptr())) return false;
  auto& c = d.copies[stream];
  for (size_t i = 0; i < cb.src.size(); ++i)
    c.cb.add(cb.src[i], cb.lds[i], cb.dst[i], cb.ldd[i], cb.rows[i], cb.cols[i]);
  for (const auto& t : keep)
    if (t.defined()) c.keep.push_back(t);
  for (const auto& t : dests)
    if (t.defined()) d.dests.insert(t.data_ptr());
  return true;
}

// may the gradient of parameter p (not yet claimed in this backward) be deferred?
bool param_deferrable(const Tensor& p) {
  if (!p.defined() || !defer_state().on) return false;
  auto& m = bucket();
  auto it = m.find(p.data_ptr());
  return it != m.end() && !it->second.claimed && !it->second.double_use &&
         it->second.numel == p.numel();
}

void double_claim_hook(const BucketEntry& e) {
  auto& d = defer_state();
  std::lock_guard<std::mutex> g(d.mu);
  const void* p = static_cast<const char*>(e.flat.data_ptr()) + e.offset * e.flat.element_size();
  if (d.on && d.dests.count(p)) d.violation = true;
}

void reduce_defer(bool on) {
  auto& d = defer_state();
  std::lock_guard<std::mutex> g(d.mu);
  TORCH_CHECK(d.pending.empty() && d.copies.empty(),
              "hlhgat: reduce_defer: deferred work still pending (call reduce_flush first)");
  d.on = on;
  d.dests.clear();
  d.streams.clear();
  d.violation = false;
}

// Run every pending reduction on the current stream (after its own stream's
// work); returns the gradient destinations that were deferred this backward.
std::vector<int64_t> reduce_flush(int64_t device) {
  auto& d = defer_state();
  std::lock_guard<std::mutex> g(d.mu);
  auto main = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)device);
  static std::vector<hipEvent_t> events;  // reused: recorded and waited at once
  size_t k = 0;
  // main waits for every stream that deferred, merged or queued copies: a
  // merged reduction (on its own stream) may feed a copy queued on another
  std::unordered_set<void*> waits = d.streams;
  for (auto& kv : d.copies) waits.insert(kv.first);
  for (void* st : waits) {
    if (st == (void*)main.stream()) continue;
    if (k == events.size()) {
      events.emplace_back();
      TORCH_CHECK(hipEventCreateWithFlags(&events.back(), hipEventDisableTiming) == hipSuccess,
                  "hlhgat: hipEventCreate");
    }
    hipEvent_t e = events[k++];
    TORCH_CHECK(hipEventRecord(e, (hipStream_t)st) == hipSuccess, "hlhgat: hipEventRecord");
    TORCH_CHECK(hipStreamWaitEvent(main.stream(), e, 0) == hipSuccess,
                "hlhgat: hipStreamWaitEvent");
  }
  d.streams.clear();
  for (auto& kv : d.pending) {
    chk(hlhgat_reduce_run(&kv.second.desc, main.stream()), "reduce_run");
    kv.second.ws.record_stream(main);
  }
  d.pending.clear();
  CopyBlocks all;
  for (auto& kv : d.copies) {
    const auto& c = kv.second.cb;
    for (size_t i = 0; i < c.src.size(); ++i) {
      if (all.src.size() == (size_t)HLHGAT_MAX_COPY_BLOCKS) {
        all.run(main.stream());
        all = CopyBlocks();
      }
      all.add(c.src[i], c.lds[i], c.dst[i], c.ldd[i], c.rows[i], c.cols[i]);
    }
    for (auto& t : kv.second.keep) t.record_stream(main);
  }
  all.run(main.stream());
  d.copies.clear();
  std::vector<int64_t> out;
  for (const void* p : d.dests) out.push_back(reinterpret_cast<int64_t>(p));
  d.dests.clear();
  const bool bad = d.violation;
  d.violation = false;
  TORCH_CHECK(!bad, "hlhgat: a parameter whose split reduction was deferred received a second "
                    "gradient in the same backward (set hlhgat.train.DEFER_REDUCE = False)");
  return out;
}

// weight (+bias) and data gradients of one Linear: hlhgat_proj_bwd (weight
// partials and data gradient in one launch, then the split reduction)
void proj_bwd_both(const Tensor& G, const std::vector<const float*>& A,
                   const std::vector<int64_t>& lda, const std::vector<int64_t>& kbw,
                   std::vector<float*>& dW, const std::vector<int64_t>& lddw, float* db,
                   const std::vector<const float*>& W, const std::vector<int64_t>& ldw,
                   const std::vector<int64_t>& kbd, std::vector<float*>& dA,
                   const std::vector<int64_t>& ldda, void* s, int acc_d = 0,
                   bool force_defer = false) {
  const int nbw = (int)A.size(), nbd = (int)W.size();
  const int64_t M = G.size(0), N = G.size(1);
  const int64_t wsf =
      nbw ? hlhgat_proj_bwd_weight_workspace_floats(nbw, kbw.data(), M, N, db != nullptr) : 0;
  Tensor ws = at::empty({std::max<int64_t>(wsf, 1)}, G.options());
  auto& d = defer_state();
  std::unique_lock<std::mutex> g(d.mu);
  // force_defer: private gradient buffers read only by deferred copies (the
  // NodeEdgeInt unpack), which the flush runs after every reduction
  bool defer = d.on && nbw > 0 && (force_defer || deferred_ok(db));
  for (int b = 0; b < nbw && defer && !force_defer; ++b) defer = deferred_ok(dW[b]);
  auto it = d.pending.find(s);
  PendingReduce prev;
  const bool merge = it != d.pending.end();
  if (merge) {
    prev = it->second;
    d.pending.erase(it);
  }
  hlhgat_reduce_desc_t out;
  int deferred = 0;
  chk(hlhgat_proj_bwd_defer(M, N, G.data_ptr<float>(), ld_of(G), nbw, A.data(), lda.data(),
                              kbw.data(), dW.data(), lddw.data(), db, nbd, W.data(), ldw.data(),
                              kbd.data(), dA.data(), ldda.data(), acc_d, ws.data_ptr<float>(),
                              wsf, merge ? &prev.desc : nullptr, defer ? &out : nullptr,
                              &deferred, s),
        "proj_bwd");
  if (merge || deferred) d.streams.insert(s);
  if (deferred) {
    d.pending[s] = PendingReduce{out, ws, s};
    for (int b = 0; b < nbw; ++b) d.dests.insert(dW[b]);
    if (db) d.dests.insert(db);
  }
}

void proj_bwd_data(const Tensor& G, const std::vector<const float*>& W,
                   const std::vector<int64_t>& ldw, const std::vector<int64_t>& kb,
                   std::vector<float*>& dA, const std::vector<int64_t>& ldda, void* s,
                   int acc = 0) {
  chk(hlhgat_proj_bwd_data((int)W.size(), G.data_ptr<float>(), ld_of(G), W.data(), ldw.data(),
                           kb.data(), G.size(0), G.size(1), dA.data(), ldda.data(), acc, s),
      "proj_bwd_data");
}

struct BnState {
  OptT w, b, rm, rv, nbt;
  double momentum = 0.1, eps = 1e-5;
  OptT valid;  // device int32 [1]: rows >= *valid are static-shape padding
};

Tensor bn_forward(const Tensor& x, const BnState& st, bool relu, Tensor& mean, Tensor& invstd,
                  const Tensor* y_into = nullptr) {
  const int64_t n = x.size(0), C = x.size(1);
  Tensor y = y_into ? *y_into : at::empty({n, C}, x.options());
  TORCH_CHECK(y.size(0) == n && y.size(1) == C && y.stride(1) == 1, "hlhgat: bad BN output view");
  mean = at::empty({C}, x.options());
  invstd = at::empty({C}, x.options());
  Tensor ws = bn_workspace(x, n, C);
  int64_t* nbt = has(st.nbt) ? st.nbt->data_ptr<int64_t>() : nullptr;
  chk(hlhgat_bn_fwd_train(x.data_ptr<float>(), ld_of(x), n, iptr(st.valid), C, fptr(st.w),
                          fptr(st.b),
                          mfptr(st.rm), mfptr(st.rv), nbt, (float)st.momentum, (float)st.eps,
                          relu ? 1 : 0, y.data_ptr<float>(), ld_of(y), mean.data_ptr<float>(),
                          invstd.data_ptr<float>(), ws.data_ptr(), ws.numel(), stream_of(x)),
      "bn_fwd_train");
  return y;
}

// x = sum_b A_b W_b^T + bias, then BatchNorm (+ReLU) of x into y: one launch
// where the grid fits (hlhgat_proj_bn_fwd), else the projection then
// bn_forward's kernels.  x must be a fresh [M, N] tensor (kept for backward).
Tensor proj_bn_forward(const std::vector<const float*>& A, const std::vector<int64_t>& lda,
                       const std::vector<const float*>& W, const std::vector<int64_t>& ldw,
                       const std::vector<int64_t>& kb, int64_t M, int64_t N, const float* bias,
                       Tensor& x, const BnState& st, bool relu, Tensor& mean, Tensor& invstd,
                       const Tensor* y_into = nullptr) {
  Tensor y = y_into ? *y_into : at::empty({M, N}, x.options());
  TORCH_CHECK(y.size(0) == M && y.size(1) == N && y.stride(1) == 1, "hlhgat: bad BN output view");
  mean = at::empty({N}, x.options());
  invstd = at::empty({N}, x.options());
  Tensor ws = bn_workspace(x, M, N);
  int64_t* nbt = has(st.nbt) ? st.nbt->data_ptr<int64_t>() : nullptr;
  chk(hlhgat_proj_bn_fwd((int)A.size(), A.data(), lda.data(), W.data(), ldw.data(), kb.data(), M,
                         N, bias, x.data_ptr<float>(), ld_of(x), iptr(st.valid), fptr(st.w),
                         fptr(st.b), mfptr(st.rm), mfptr(st.rv), nbt, (float)st.momentum,
                         (float)st.eps, relu ? 1 : 0, y.data_ptr<float>(), ld_of(y),
                         mean.data_ptr<float>(), invstd.data_ptr<float>(), ws.data_ptr(),
                         ws.numel(), stream_of(x)),
      "proj_bn_fwd");
  return y;
}

// returns dx; fills dw/db when requested
// dx_into: optional [n, C] row-strided destination (e.g. a column slice)
Tensor bn_backward(const Tensor& x, const OptT& y, const Tensor& dy, const OptT& w,
                   const Tensor& mean, const Tensor& invstd, bool need_w, bool need_b,
                   Tensor& dw, Tensor& db, const Tensor* dx_into = nullptr,
                   const Tensor* b_param = nullptr, const Tensor& valid = Tensor()) {
  const int64_t n = x.size(0), C = x.size(1);
  Tensor dyc = rows2d(dy);
  Tensor dx = dx_into ? *dx_into : at::empty({n, C}, x.options());
  TORCH_CHECK(dx.size(0) == n && dx.size(1) == C && dx.stride(1) == 1, "hlhgat: bad dx view");
  dw = (need_w && has(w)) ? grad_like(w) : Tensor();
  db = need_b ? ((b_param && b_param->defined()) ? grad_like(*b_param)
                                                 : at::empty({C}, x.options()))
              : Tensor();
  Tensor ws = bn_workspace(x, n, C);
  chk(hlhgat_bn_bwd_train(x.data_ptr<float>(), ld_of(x), fptr(y), has(y) ? ld_of(*y) : 0,
                          dyc.data_ptr<float>(), ld_of(dyc), n,
                          valid.defined() ? valid.data_ptr<int32_t>() : nullptr, C, fptr(w),
                          mean.data_ptr<float>(), invstd.data_ptr<float>(), dx.data_ptr<float>(),
                          ld_of(dx), dw.defined() ? dw.data_ptr<float>() : nullptr,
                          db.defined() ? db.data_ptr<float>() : nullptr, ws.data_ptr(),
                          ws.numel(), stream_of(x)),
      "bn_bwd_train");
  return dx;
}

inline bool al4(const void* p, int64_t ld) {
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0;
}

// Two-stream fork inside one autograd node: the node (current) stream and a
// persistent side stream per device, ordered by hipEvents (captured into a
// hipGraph as branch dependencies).  Tensors allocated while the side stream
// is current and then used on the node stream are record_stream()-ed.
// (PyTorch-ROCm exposes HIP streams to torch as "cuda" streams: the
// MasqueradingAsCUDA wrappers are the ones its allocator and guards accept.)
using TStream = c10::hip::HIPStreamMasqueradingAsCUDA;
using TStreamGuard = c10::hip::HIPStreamGuardMasqueradingAsCUDA;
struct Fork {
  TStream main, side;
  explicit Fork(int dev)
      : main(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA((c10::DeviceIndex)dev)),
        side(side_of(dev)) {}
  static std::unordered_map<int, TStream>& registry() {
    static auto* streams = new std::unordered_map<int, TStream>();
    return *streams;
  }
  static TStream side_of(int dev) {
    auto& streams = registry();
    auto it = streams.find(dev);
    if (it == streams.end()) {
      // a stream of its own, not one of torch's round-robin pool: a pool
      // stream is handed out again after 32 requests, e.g. as a user's copy
      // stream, whose uploads would then land inside a capture this side
      // stream has joined
      c10::hip::HIPGuardMasqueradingAsCUDA g((c10::DeviceIndex)dev);
      hipStream_t raw = nullptr;
      TORCH_CHECK(hipStreamCreateWithFlags(&raw, hipStreamNonBlocking) == hipSuccess,
                  "hlhgat: hipStreamCreateWithFlags");
      it = streams.emplace(dev, c10::hip::getStreamFromExternalMasqueradingAsCUDA(
                                    raw, (c10::DeviceIndex)dev)).first;
    }
    return it->second;
  }
  static hipEvent_t next_event() {
    static thread_local std::vector<hipEvent_t> pool;
    static thread_local size_t k = 0;
    if (pool.empty()) {
      pool.resize(64);
      for (auto& e : pool) TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == 0);
    }
    return pool[k++ % pool.size()];
  }
  static void order(const TStream& from, const TStream& to) {
    hipEvent_t e = next_event();
    TORCH_CHECK(hipEventRecord(e, from.stream()) == hipSuccess, "hlhgat: hipEventRecord");
    TORCH_CHECK(hipStreamWaitEvent(to.stream(), e, 0) == hipSuccess, "hlhgat: hipStreamWaitEvent");
  }
  void side_waits_main() { order(main, side); }
  void main_waits_side() { order(side, main); }
  void escape(std::initializer_list<Tensor> ts) {
    for (const auto& t : ts)
      if (t.defined()) t.record_stream(main);
  }
};

// ---------------------------------------------------------------------------
// conv (+ BN (+ ReLU))
// ---------------------------------------------------------------------------
// One side's conv (+ BN (+ ReLU)) arguments (the conv_bn signature below).
struct ConvArgs {
  Tensor x, a_rowptr, a_col;
  OptT a_val;
  Tensor t_rowptr, t_col;
  OptT t_val;
  int64_t nnz = 0, kind = 0;
  std::vector<Tensor> W;
  OptT bias, bn_w, bn_b, bn_rm, bn_rv, bn_nbt;
  double momentum = 0.1, eps = 1e-5;
  int64_t bn_mode = 0;
  OptT out_buf, a_order, t_order;
  OptT valid, h_tile, h_ptr, h_cols, h_srp, h_lcol, h_sval;
  std::vector<int64_t> h_bounds;
  OptT h_hdr;
  std::vector<Tensor> fac;
  int64_t fac_nodes = 0;
};

// What one side's backward needs: the tensors (kSavedFixed, then W[0..K),
// then the factor) and the sizes.
constexpr size_t kSavedFixed = 21;
struct ConvSaved {
  std::vector<Tensor> t;
  std::vector<int64_t> dims;  // N, Cin, F, M, dout, K, kind, nnz, bn_mode, has_bias
  std::vector<int64_t> xshape, h_bounds;
  int64_t fac_nodes = 0;
  void to_ctx(AutogradContext* ctx, const std::string& p) const {
    ctx->saved_data[p + "dims"] = dims;
    ctx->saved_data[p + "xshape"] = xshape;
    ctx->saved_data[p + "h_bounds"] = h_bounds;
    ctx->saved_data[p + "misc"] = std::vector<int64_t>{fac_nodes, (int64_t)t.size()};
  }
  static ConvSaved from_ctx(AutogradContext* ctx, const std::string& p,
                            const std::vector<Tensor>& all, size_t first) {
    ConvSaved s;
    s.dims = ctx->saved_data[p + "dims"].toIntVector();
    s.xshape = ctx->saved_data[p + "xshape"].toIntVector();
    s.h_bounds = ctx->saved_data[p + "h_bounds"].toIntVector();
    const auto m = ctx->saved_data[p + "misc"].toIntVector();
    s.fac_nodes = m[0];
    s.t.assign(all.begin() + first, all.begin() + first + m[1]);
    return s;
  }
};

// Which gradients one side's backward must produce.
struct ConvNeeds {
  bool x = false;
  std::vector<bool> w;
  bool bias = false, bn_w = false, bn_b = false;
};
struct ConvGrads {
  Tensor dx, dbias, dbn_w, dbn_b;
  std::vector<Tensor> dW;
};

// HodgeLaguerreConv / HodgeChebConv forward (+ BN (+ ReLU)) of one side.
Tensor conv_forward(const ConvArgs& c, ConvSaved& sv) {
  const Tensor& x = c.x;
  req(x, "x");
  const int64_t N = x.size(0);
  const int64_t Cin = x.size(-1);
  const int64_t K = (int64_t)c.W.size();
  Tensor x2 = x.dim() == 2 ? rows2d(x) : x.contiguous().view({N, -1});
  const int64_t F = x2.size(1);
  const int64_t M = N * (F / Cin);
  const int64_t dout = c.W[0].size(0);
  void* s = stream_of(x);
  Tensor T = at::empty({std::max<int64_t>(K - 1, 0), N, F}, x.options());
  // halo tiles describe A; they serve the adjoint only when A^T is A
  const bool use_halo = has(c.h_lcol) && has(c.h_tile) && has(c.h_ptr) && has(c.h_cols) &&
                        has(c.h_srp) && has(c.h_hdr);
  const hlhgat_halo_t halo =
      use_halo ? make_halo(*c.h_tile, *c.h_ptr, *c.h_cols, *c.h_srp, *c.h_lcol,
                           has(c.h_sval) ? *c.h_sval : Tensor(), c.h_bounds, *c.h_hdr)
               : hlhgat_halo_t{};
  const bool factored = !c.fac.empty();
  if (factored && K > 1 && N > 0) {
    const hlhgat_hodge_factor_t hf = make_factor(c.fac, c.fac_nodes, N);
    Tensor work = at::empty({hlhgat_hodge_factor_work_floats(c.fac_nodes, F)}, x.options());
    chk(hlhgat_poly_basis_fwd_factored((int)c.kind, &hf, x2.data_ptr<float>(), ld_of(x2), F,
                                       (int)K, T.data_ptr<float>(), work.data_ptr<float>(), s),
        "poly_basis_fwd_factored");
  } else if (K > 1 && N > 0) {
    chk(hlhgat_poly_basis_fwd((int)c.kind, c.a_rowptr.data_ptr<int>(),
                              c.nnz ? c.a_col.data_ptr<int>() : nullptr,
                              c.nnz ? fptr(c.a_val) : nullptr, N, c.nnz, iptr(c.a_order),
                              use_halo ? &halo : nullptr, x2.data_ptr<float>(), ld_of(x2), F, (int)K, T.data_ptr<float>(), s),
        "poly_basis_fwd");
  }
  std::vector<const float*> Ap(K), Wp(K);
  std::vector<int64_t> lda(K), ldw(K), kb(K, Cin);
  Ap[0] = x2.data_ptr<float>();
  lda[0] = x.dim() == 2 ? ld_of(x2) : Cin;
  for (int64_t k = 1; k < K; ++k) {
    Ap[k] = T.data_ptr<float>() + (k - 1) * N * F;
    lda[k] = Cin;
  }
  for (int64_t k = 0; k < K; ++k) {
    req(c.W[k], "lins[k].weight");
    TORCH_CHECK(c.W[k].stride(1) == 1, "hlhgat: weights need unit inner stride");
    Wp[k] = c.W[k].data_ptr<float>();
    ldw[k] = c.W[k].stride(0);
  }
  // out_buf: caller-owned [M, dout] destination (a column block of the dense
  // concatenation slab, hlhgat.ops.DenseConcat); the final output lands there
  const bool sink = has(c.out_buf);
  if (sink)
    TORCH_CHECK(c.out_buf->size(0) == M && c.out_buf->size(1) == dout &&
                    c.out_buf->stride(1) == 1 && c.out_buf->device() == x.device(),
                "hlhgat: conv output buffer must be a row-major [", M, ", ", dout, "] view");
  Tensor pre = (sink && c.bn_mode == 0) ? *c.out_buf : at::empty({M, dout}, x.options());
  Tensor out = pre, mean, invstd;
  if (M > 0 && c.bn_mode > 0) {
    BnState st{c.bn_w, c.bn_b, c.bn_rm, c.bn_rv, c.bn_nbt, c.momentum, c.eps, c.valid};
    out = proj_bn_forward(Ap, lda, Wp, ldw, kb, M, dout, fptr(c.bias), pre, st, c.bn_mode == 2,
                          mean, invstd, sink ? &*c.out_buf : nullptr);
  } else {
    if (M > 0) {
      proj_fwd(Ap, lda, Wp, ldw, kb, M, dout, fptr(c.bias), pre, s);
    } else if (has(c.bias)) {
      pre.copy_(c.bias->expand_as(pre));
    }
    if (c.bn_mode > 0) {
      BnState st{c.bn_w, c.bn_b, c.bn_rm, c.bn_rv, c.bn_nbt, c.momentum, c.eps, c.valid};
      out = bn_forward(pre, st, c.bn_mode == 2, mean, invstd, sink ? &*c.out_buf : nullptr);
    }
  }
  sv.dims = {N, Cin, F, M, dout, K, c.kind, c.nnz, c.bn_mode, has(c.bias) ? 1 : 0};
  sv.fac_nodes = c.fac_nodes;
  sv.h_bounds = c.h_bounds;
  sv.xshape = x.sizes().vec();
  const bool halo_bwd = use_halo && c.t_rowptr.data_ptr() == c.a_rowptr.data_ptr();
  sv.t = {x2,
          T,
          has(c.t_order) ? *c.t_order : Tensor(),
          has(c.valid) ? *c.valid : Tensor(),
          c.t_rowptr,
          c.t_col,
          has(c.t_val) ? *c.t_val : Tensor(),
          c.bn_mode > 0 ? pre : Tensor(),
          c.bn_mode == 2 ? out : Tensor(),
          mean,
          invstd,
          has(c.bn_w) ? *c.bn_w : Tensor(),
          has(c.bias) ? *c.bias : Tensor(),
          has(c.bn_b) ? *c.bn_b : Tensor(),
          halo_bwd ? *c.h_tile : Tensor(),
          halo_bwd ? *c.h_ptr : Tensor(),
          halo_bwd ? *c.h_cols : Tensor(),
          halo_bwd ? *c.h_srp : Tensor(),
          halo_bwd ? *c.h_lcol : Tensor(),
          (halo_bwd && has(c.h_sval)) ? *c.h_sval : Tensor(),
          halo_bwd ? *c.h_hdr : Tensor()};
  for (const auto& w : c.W) sv.t.push_back(w);
  for (const auto& t : c.fac) sv.t.push_back(t);
  std::vector<int64_t> oshape = x.sizes().vec();
  oshape.back() = dout;
  return out.view(oshape);
}

ConvGrads conv_backward(const ConvSaved& sv, const Tensor& grad, const ConvNeeds& nd) {
  const auto& d = sv.dims;
  const int64_t N = d[0], Cin = d[1], F = d[2], M = d[3], dout = d[4], K = d[5], kind = d[6],
                nnz = d[7], bn_mode = d[8];
  const bool has_bias = d[9] != 0;
  const auto& t = sv.t;
  Tensor x2 = t[0], T = t[1], t_order = t[2], valid = t[3], t_rowptr = t[4], t_col = t[5],
         t_val = t[6], pre = t[7], yout = t[8], mean = t[9], invstd = t[10], bn_w = t[11],
         bias_p = t[12], bn_b = t[13], h_tile = t[14], h_ptr = t[15], h_cols = t[16],
         h_srp = t[17], h_lcol = t[18], h_sval = t[19], h_hdr = t[20];
  std::vector<Tensor> W(t.begin() + kSavedFixed, t.begin() + kSavedFixed + K);
  std::vector<Tensor> fac(t.begin() + kSavedFixed + K, t.end());
  const bool use_halo = h_lcol.defined();
  const hlhgat_halo_t halo =
      use_halo ? make_halo(h_tile, h_ptr, h_cols, h_srp, h_lcol, h_sval, sv.h_bounds, h_hdr)
               : hlhgat_halo_t{};
  void* s = stream_of(x2);
  // row-strided is fine (e.g. a column block of the gradient slab)
  Tensor G = rows2d(grad.reshape({M, dout}));
  ConvGrads out;
  out.dW.resize(K);
  std::vector<const float*> Ap(K);
  std::vector<int64_t> lda(K), kb(K, Cin);
  Ap[0] = x2.data_ptr<float>();
  lda[0] = (int64_t)sv.xshape.size() == 2 ? ld_of(x2) : Cin;
  for (int64_t k = 1; k < K; ++k) {
    Ap[k] = T.data_ptr<float>() + (k - 1) * N * F;
    lda[k] = Cin;
  }
  bool need_w = false;
  for (int64_t k = 0; k < K; ++k) need_w = need_w || nd.w[k];
  const bool need_b = has_bias && nd.bias;
  struct {
    std::vector<float*> dWp;
    std::vector<int64_t> lddw;
    float* db = nullptr;
  } wdef;  // weight gradient deferred into the data gradient's launch
  if (bn_mode > 0) {
    const OptT bn_y = bn_mode == 2 ? OptT(yout) : OptT();
    OptT w = bn_w.defined() ? OptT(bn_w) : OptT();
    G = bn_backward(pre, bn_y, G, w, mean, invstd, nd.bn_w, nd.bn_b, out.dbn_w, out.dbn_b,
                    nullptr, &bn_b, valid);
  }
  if (need_w || need_b) {
    std::vector<Tensor> dW(K);
    std::vector<float*> dWp(K);
    std::vector<int64_t> lddw(K);
    for (int64_t k = 0; k < K; ++k) {
      dW[k] = nd.w[k] ? grad_like(W[k]) : at::empty({dout, Cin}, x2.options());
      dWp[k] = dW[k].data_ptr<float>();
      lddw[k] = Cin;
    }
    Tensor db = need_b ? grad_like(bias_p) : Tensor();
    if (M > 0 && nd.x && fused_bwd_flag()) {
      wdef.dWp = dWp;  // launched with the data gradient
      wdef.lddw = lddw;
      wdef.db = need_b ? db.data_ptr<float>() : nullptr;
    } else if (M > 0) {  // weight only: the one-launch path with no data items
      std::vector<const float*> noW;
      std::vector<int64_t> noL;
      std::vector<float*> noD;
      proj_bwd_both(G, Ap, lda, kb, dWp, lddw, need_b ? db.data_ptr<float>() : nullptr, noW, noL,
                    noL, noD, noL, s, 0, false);
    } else {
      for (auto& tt : dW) tt.zero_();
      if (need_b) db.zero_();
    }
    for (int64_t k = 0; k < K; ++k)
      if (nd.w[k]) out.dW[k] = dW[k];
    if (need_b) out.dbias = db;
  }
  if (nd.x) {
    Tensor Gs = at::empty({K, N, F}, x2.options());
    if (M > 0) {
      std::vector<const float*> Wp(K);
      std::vector<int64_t> ldw(K), ldda(K, Cin);
      std::vector<float*> dA(K);
      for (int64_t k = 0; k < K; ++k) {
        Wp[k] = W[k].data_ptr<float>();
        ldw[k] = W[k].stride(0);
        dA[k] = Gs.data_ptr<float>() + k * N * F;
      }
      if (!wdef.dWp.empty())
        proj_bwd_both(G, Ap, lda, kb, wdef.dWp, wdef.lddw, wdef.db, Wp, ldw, kb, dA, ldda, s, 0,
                      false);
      else
        proj_bwd_data(G, Wp, ldw, kb, dA, ldda, s);
      if (K > 1 && !fac.empty()) {  // L1 symmetric: the adjoint uses the same factor
        const hlhgat_hodge_factor_t hf = make_factor(fac, sv.fac_nodes, N);
        Tensor work = at::empty({hlhgat_hodge_factor_work_floats(sv.fac_nodes, F)}, x2.options());
        chk(hlhgat_poly_basis_bwd_factored((int)kind, &hf, F, (int)K, Gs.data_ptr<float>(),
                                           work.data_ptr<float>(), s),
            "poly_basis_bwd_factored");
      } else if (K > 1) {
        chk(hlhgat_poly_basis_bwd((int)kind, t_rowptr.data_ptr<int>(),
                                  nnz ? t_col.data_ptr<int>() : nullptr,
                                  (nnz && t_val.defined()) ? t_val.data_ptr<float>() : nullptr, N,
                                  nnz, t_order.defined() ? t_order.data_ptr<int>() : nullptr,
                                  use_halo ? &halo : nullptr, F, (int)K, Gs.data_ptr<float>(), s),
            "poly_basis_bwd");
      }
    } else {
      Gs.zero_();
    }
    out.dx = Gs[0].view(sv.xshape);
  }
  return out;
}

// argument positions of conv_bn (needs_input_grad / gradient slots)
constexpr int64_t kConvPosW = 9;  // W[0..K), then bias, bn_w, bn_b

ConvNeeds conv_needs(AutogradContext* ctx, int64_t K, int64_t base) {
  ConvNeeds nd;
  nd.x = need(ctx, base);
  nd.w.resize(K);
  for (int64_t k = 0; k < K; ++k) nd.w[k] = need(ctx, base + kConvPosW + k);
  nd.bias = need(ctx, base + kConvPosW + K);
  nd.bn_w = need(ctx, base + kConvPosW + K + 1);
  nd.bn_b = need(ctx, base + kConvPosW + K + 2);
  return nd;
}

void edge_map_conv(EdgeMap& em, const ConvArgs& c) {
  em.tensor();  // x
  em.tensor();
  em.tensor();
  em.opt(c.a_val);
  em.tensor();
  em.tensor();
  em.opt(c.t_val);
  em.other();
  em.other();
  em.list(c.W);
  em.opt(c.bias);
  em.opt(c.bn_w);
  em.opt(c.bn_b);
  em.opt(c.bn_rm);
  em.opt(c.bn_rv);
  em.opt(c.bn_nbt);
  em.other();
  em.other();
  em.other();
  em.opt(c.out_buf);
  em.opt(c.a_order);
  em.opt(c.t_order);
  em.opt(c.valid);
  em.opt(c.h_tile);
  em.opt(c.h_ptr);
  em.opt(c.h_cols);
  em.opt(c.h_srp);
  em.opt(c.h_lcol);
  em.opt(c.h_sval);
  em.other();
  em.opt(c.h_hdr);
  em.list(c.fac);
  em.other();
}
constexpr int64_t conv_positions(int64_t K, int64_t n_fac) { return 30 + K + n_fac + 1; }

void put_grads(variable_list& out, int64_t base, int64_t K, const ConvGrads& g) {
  out[base] = g.dx;
  for (int64_t k = 0; k < K; ++k) out[base + kConvPosW + k] = g.dW[k];
  out[base + kConvPosW + K] = g.dbias;
  out[base + kConvPosW + K + 1] = g.dbn_w;
  out[base + kConvPosW + K + 2] = g.dbn_b;
}

class ConvBNFn : public torch::autograd::Function<ConvBNFn> {
 public:
  // x: [N, C] or [N, T, C]; A/At: CSR of L and L^T; W: K weights [dout, C]
  static Tensor forward(AutogradContext* ctx, Tensor x, Tensor a_rowptr, Tensor a_col,
                        OptT a_val, Tensor t_rowptr, Tensor t_col, OptT t_val, int64_t nnz,
                        int64_t kind, at::TensorList W, OptT bias, OptT bn_w, OptT bn_b,
                        OptT bn_rm, OptT bn_rv, OptT bn_nbt, double momentum, double eps,
                        int64_t bn_mode, OptT out_buf, OptT a_order, OptT t_order, OptT valid,
                        OptT h_tile, OptT h_ptr, OptT h_cols, OptT h_srp, OptT h_lcol,
                        OptT h_sval, std::vector<int64_t> h_bounds, OptT h_hdr,
                        at::TensorList fac, int64_t fac_nodes) {
    ConvArgs c{x, a_rowptr, a_col, a_val, t_rowptr, t_col, t_val, nnz, kind, W.vec(), bias,
               bn_w, bn_b, bn_rm, bn_rv, bn_nbt, momentum, eps, bn_mode, out_buf, a_order,
               t_order, valid, h_tile, h_ptr, h_cols, h_srp, h_lcol, h_sval, h_bounds, h_hdr,
               fac.vec(), fac_nodes};
    ConvSaved sv;
    Tensor y = conv_forward(c, sv);
    EdgeMap em;
    edge_map_conv(em, c);
    ctx->saved_data["edges"] = em.e;
    sv.to_ctx(ctx, "");
    ctx->save_for_backward(sv.t);
    return y;
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    ConvSaved sv = ConvSaved::from_ctx(ctx, "", ctx->get_saved_variables(), 0);
    const int64_t K = sv.dims[5];
    const int64_t n_fac = (int64_t)sv.t.size() - (int64_t)kSavedFixed - K;
    variable_list out(conv_positions(K, n_fac));
    put_grads(out, 0, K, conv_backward(sv, grads[0], conv_needs(ctx, K, 0)));
    return out;
  }
};

// ---------------------------------------------------------------------------
// BatchNorm (+ ReLU)
// ---------------------------------------------------------------------------
class BNActFn : public torch::autograd::Function<BNActFn> {
 public:
  static Tensor forward(AutogradContext* ctx, Tensor x, OptT w, OptT b, OptT rm, OptT rv,
                        OptT nbt, double momentum, double eps, bool relu, OptT valid) {
    req(x, "x");
    Tensor xc = rows2d(x);
    Tensor mean, invstd;
    BnState st{w, b, rm, rv, nbt, momentum, eps, valid};
    Tensor y = bn_forward(xc, st, relu, mean, invstd);
    ctx->saved_data["relu"] = relu;
    EdgeMap em;
    em.tensor();
    em.opt(w);
    em.opt(b);
    em.opt(rm);
    em.opt(rv);
    em.opt(nbt);
    ctx->saved_data["edges"] = em.e;
    ctx->save_for_backward({xc, relu ? y : Tensor(), has(w) ? *w : Tensor(), mean, invstd,
                            has(b) ? *b : Tensor(), has(valid) ? *valid : Tensor()});
    return y;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    Tensor dw, db;
    OptT y = sv[1].defined() ? OptT(sv[1]) : OptT();
    OptT w = sv[2].defined() ? OptT(sv[2]) : OptT();
    Tensor dx = bn_backward(sv[0], y, grads[0], w, sv[3], sv[4], need(ctx, 1), need(ctx, 2), dw,
                           db, nullptr, &sv[5], sv[6]);
    return {dx, dw, db, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

// ---------------------------------------------------------------------------
// Linear over blocks: out = cat(As, -1) @ W^T + b, W column-split per block
// ---------------------------------------------------------------------------
struct LinearOperands {
  std::vector<const float*> Ap, Wp;
  std::vector<int64_t> lda, ldw, kb;
};
LinearOperands linear_operands(const std::vector<Tensor>& As, const Tensor& W) {
  const int nb = (int)As.size();
  LinearOperands o;
  o.Ap.resize(nb);
  o.Wp.resize(nb);
  o.lda.resize(nb);
  o.ldw.resize(nb);
  o.kb.resize(nb);
  int64_t off = 0;
  for (int i = 0; i < nb; ++i) {
    o.Ap[i] = As[i].data_ptr<float>();
    o.lda[i] = ld_of(As[i]);
    o.kb[i] = As[i].size(1);
    o.Wp[i] = W.data_ptr<float>() + off;
    o.ldw[i] = W.stride(0);
    off += o.kb[i];
  }
  TORCH_CHECK(off == W.size(1), "hlhgat: Linear expects ", W.size(1), " input features, got ",
              off);
  return o;
}

Tensor linear_forward(const std::vector<Tensor>& As, const Tensor& W, const OptT& b) {
  const int64_t M = As[0].size(0), N = W.size(0);
  LinearOperands o = linear_operands(As, W);
  Tensor out = at::empty({M, N}, W.options());
  if (M > 0) proj_fwd(o.Ap, o.lda, o.Wp, o.ldw, o.kb, M, N, fptr(b), out, stream_of(W));
  return out;
}

// Linear(blocks) -> BatchNorm (+ReLU): h (the BN input) is returned through
// `h`, the activation as the result (one launch where it fits).
Tensor linear_bn_forward(const std::vector<Tensor>& As, const Tensor& W, const OptT& b,
                         const BnState& st, bool relu, Tensor& h, Tensor& mean, Tensor& invstd) {
  const int64_t M = As[0].size(0), N = W.size(0);
  if (M == 0) {
    h = linear_forward(As, W, b);
    return bn_forward(h, st, relu, mean, invstd);
  }
  LinearOperands o = linear_operands(As, W);
  h = at::empty({M, N}, W.options());
  return proj_bn_forward(o.Ap, o.lda, o.Wp, o.ldw, o.kb, M, N, fptr(b), h, st, relu, mean,
                         invstd);
}

// grads of linear_forward; dAs[i] only where need_a[i]
// dA_into (optional, one per block, undefined = fresh): row-strided views the
// data gradient is written (into_acc = 0) or ADDED (1) into and returned as
// dAs (a DenseConcat gradient sink)
void linear_backward(const Tensor& Gin, const std::vector<Tensor>& As, const Tensor& W,
                     bool need_w, bool need_b, const std::vector<bool>& need_a, Tensor& dW,
                     Tensor& db, std::vector<Tensor>& dAs, const Tensor* b_param = nullptr,
                     const std::vector<Tensor>* dA_into = nullptr, int into_acc = 1,
                     bool force_defer = false) {
  Tensor G = rows2d(Gin);
  const int64_t M = G.size(0), N = G.size(1);
  const int nb = (int)As.size();
  void* s = stream_of(W);
  std::vector<int64_t> kb(nb), offs(nb);
  int64_t off = 0;
  for (int i = 0; i < nb; ++i) {
    kb[i] = As[i].size(1);
    offs[i] = off;
    off += kb[i];
  }
  dW = Tensor();
  db = Tensor();
  bool any_a = false;
  for (int i = 0; i < nb; ++i) any_a = any_a || need_a[i];
  std::vector<const float*> wAp;  // weight gradient deferred into the data gradient's launch
  std::vector<int64_t> wlda, wlddw;
  std::vector<float*> wdWp;
  float* wdb = nullptr;
  Tensor wkeep, wkeep_b;  // the gradient buffers stay allocated until the launch
  if (need_w || need_b) {
    Tensor gw = need_w ? grad_like(W) : at::empty_like(W, at::MemoryFormat::Contiguous);
    Tensor gb = need_b ? ((b_param && b_param->defined()) ? grad_like(*b_param)
                                                          : at::empty({N}, W.options()))
                       : Tensor();
    if (M > 0) {
      std::vector<const float*> Ap(nb);
      std::vector<int64_t> lda(nb), lddw(nb, W.size(1));
      std::vector<float*> dWp(nb);
      for (int i = 0; i < nb; ++i) {
        Ap[i] = As[i].data_ptr<float>();
        lda[i] = ld_of(As[i]);
        dWp[i] = gw.data_ptr<float>() + offs[i];
      }
      if (any_a && fused_bwd_flag()) {
        wAp = Ap;
        wlda = lda;
        wlddw = lddw;
        wdWp = dWp;
        wdb = need_b ? gb.data_ptr<float>() : nullptr;
        wkeep = gw;
        wkeep_b = gb;
      } else {  // weight only: the one-launch path with no data items
        std::vector<const float*> noW;
        std::vector<int64_t> noL;
        std::vector<float*> noD;
        proj_bwd_both(G, Ap, lda, kb, dWp, lddw, need_b ? gb.data_ptr<float>() : nullptr, noW,
                      noL, noL, noD, noL, s, 0, false);
      }
    } else {
      gw.zero_();
      if (need_b) gb.zero_();
    }
    if (need_w) dW = gw;
    if (need_b) db = gb;
  }
  dAs.assign(nb, Tensor());
  std::vector<int> idx;
  for (int i = 0; i < nb; ++i)
    if (need_a[i]) idx.push_back(i);
  if (!idx.empty()) {
    std::vector<const float*> Wp;
    std::vector<int64_t> ldw, kbs, ldda;
    std::vector<float*> dA;
    // accumulate into the given destinations only when every block has one
    bool into = dA_into != nullptr;
    for (int i : idx)
      into = into && (int)dA_into->size() > i && (*dA_into)[i].defined() &&
             (*dA_into)[i].size(0) == M && (*dA_into)[i].size(1) == kb[i] &&
             (*dA_into)[i].stride(1) == 1;
    for (int i : idx) {
      dAs[i] = into ? (*dA_into)[i] : at::empty({M, kb[i]}, W.options());
      Wp.push_back(W.data_ptr<float>() + offs[i]);
      ldw.push_back(W.stride(0));
      kbs.push_back(kb[i]);
      dA.push_back(dAs[i].data_ptr<float>());
      ldda.push_back(into ? dAs[i].stride(0) : kb[i]);
    }
    if (M > 0) {
      const int acc = into ? into_acc : 0;
      if (!wAp.empty())
        proj_bwd_both(G, wAp, wlda, kb, wdWp, wlddw, wdb, Wp, ldw, kbs, dA, ldda, s, acc,
                      force_defer);
      else
        proj_bwd_data(G, Wp, ldw, kbs, dA, ldda, s, acc);
    }
  }
}

class LinearFn : public torch::autograd::Function<LinearFn> {
 public:
  static Tensor forward(AutogradContext* ctx, Tensor W, OptT b, at::TensorList As_in) {
    req(W, "weight");
    std::vector<Tensor> As;
    for (const auto& a : As_in) {
      req(a, "input");
      As.push_back(rows2d(a));
    }
    Tensor Wc = W.stride(1) == 1 ? W : W.contiguous();
    Tensor out = linear_forward(As, Wc, b);
    ctx->saved_data["has_b"] = has(b);
    EdgeMap em;
    em.tensor();
    em.opt(b);
    em.list(As_in);
    ctx->saved_data["edges"] = em.e;
    std::vector<Tensor> save = {Wc, has(b) ? *b : Tensor()};
    save.insert(save.end(), As.begin(), As.end());
    ctx->save_for_backward(save);
    return out;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    Tensor W = sv[0], b = sv[1];
    std::vector<Tensor> As(sv.begin() + 2, sv.end());
    std::vector<bool> need_a(As.size());
    for (size_t i = 0; i < As.size(); ++i) need_a[i] = need(ctx, 2 + (int64_t)i);
    Tensor dW, db;
    std::vector<Tensor> dAs;
    linear_backward(grads[0], As, W, need(ctx, 0), need(ctx, 1), need_a, dW, db, dAs, &b);
    variable_list out = {dW, db};
    out.insert(out.end(), dAs.begin(), dAs.end());
    return out;
  }
};

// Activation tap (test infrastructure, hlhgat.nn.TAP): while on, the
// NodeEdgeInt value node and the two-layer MLP node keep a copy of their
// hidden post-ReLU activations (NodeEdgeInt: node side, then edge side) for
// the frozen-mask gradient checks.
struct TapState {
  bool on = false;
  std::vector<Tensor> taken;
};
TapState& tap_state() {
  static auto* t = new TapState();
  return *t;
}
void set_tap(bool on) {
  tap_state().on = on;
  tap_state().taken.clear();
}
std::vector<Tensor> take_tap() {
  std::vector<Tensor> out;
  out.swap(tap_state().taken);
  return out;
}

// ---------------------------------------------------------------------------
// Linear(blocks) -> BN -> ReLU -> Linear -> BN -> ReLU (NodeEdgeInt WV_*, two
// layers of a readout MLP)
// ---------------------------------------------------------------------------
class MLP2Fn : public torch::autograd::Function<MLP2Fn> {
 public:
  static Tensor forward(AutogradContext* ctx, at::TensorList blocks_in, Tensor W0, OptT b0,
                        OptT g1, OptT be1, OptT rm1, OptT rv1, OptT nbt1, Tensor W3, OptT b3,
                        OptT g4, OptT be4, OptT rm4, OptT rv4, OptT nbt4, double mom1, double eps1,
                        double mom4, double eps4) {
    std::vector<Tensor> blocks;
    for (const auto& a : blocks_in) {
      req(a, "input");
      blocks.push_back(rows2d(a));
    }
    Tensor W0c = W0.stride(1) == 1 ? W0 : W0.contiguous();
    Tensor W3c = W3.stride(1) == 1 ? W3 : W3.contiguous();
    Tensor h1, h2, m1, i1, m4, i4;
    Tensor a1 = linear_bn_forward(blocks, W0c, b0, BnState{g1, be1, rm1, rv1, nbt1, mom1, eps1},
                                  true, h1, m1, i1);
    Tensor y = linear_bn_forward({a1}, W3c, b3, BnState{g4, be4, rm4, rv4, nbt4, mom4, eps4},
                                 true, h2, m4, i4);
    if (tap_state().on) tap_state().taken.push_back(a1.clone());  // the hidden ReLU
    ctx->saved_data["nb"] = (int64_t)blocks.size();
    {
      EdgeMap em;
      em.list(blocks_in);
      em.tensor();  // W0
      em.opt(b0);
      em.opt(g1);
      em.opt(be1);
      em.opt(rm1);
      em.opt(rv1);
      em.opt(nbt1);
      em.tensor();  // W3
      em.opt(b3);
      em.opt(g4);
      em.opt(be4);
      em.opt(rm4);
      em.opt(rv4);
      em.opt(nbt4);
      for (int i = 0; i < 4; ++i) em.other();
      ctx->saved_data["edges"] = em.e;
    }
    ctx->saved_data["has_b0"] = has(b0);
    ctx->saved_data["has_b3"] = has(b3);
    std::vector<Tensor> save = {W0c, h1, a1, m1, i1, has(g1) ? *g1 : Tensor(), W3c, h2, y, m4, i4,
                                has(g4) ? *g4 : Tensor(), has(b0) ? *b0 : Tensor(),
                                has(be1) ? *be1 : Tensor(), has(b3) ? *b3 : Tensor(),
                                has(be4) ? *be4 : Tensor()};
    save.insert(save.end(), blocks.begin(), blocks.end());
    ctx->save_for_backward(save);
    return y;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    const int64_t nb = ctx->saved_data["nb"].toInt();
    Tensor W0 = sv[0], h1 = sv[1], a1 = sv[2], m1 = sv[3], i1 = sv[4], g1 = sv[5], W3 = sv[6],
           h2 = sv[7], y = sv[8], m4 = sv[9], i4 = sv[10], g4 = sv[11];
    Tensor b0 = sv[12], be1 = sv[13], b3 = sv[14], be4 = sv[15];
    std::vector<Tensor> blocks(sv.begin() + 16, sv.end());
    // positions: blocks[0..nb), W0, b0, g1, be1, rm1, rv1, nbt1, W3, b3, g4, be4, rm4, rv4,
    //            nbt4, mom1, eps1, mom4, eps4
    const int64_t P = nb;
    variable_list out(nb + 18);
    Tensor dg4, dbe4, dg1, dbe1;
    Tensor dh2 = bn_backward(h2, OptT(y), grads[0], g4.defined() ? OptT(g4) : OptT(), m4, i4,
                             need(ctx, P + 9), need(ctx, P + 10), dg4,
                             dbe4, nullptr, &be4);
    out[P + 9] = dg4;
    out[P + 10] = dbe4;
    Tensor dW3, db3, dW0, db0;
    std::vector<Tensor> da1;
    linear_backward(dh2, {a1}, W3, need(ctx, P + 7), need(ctx, P + 8), {true},
                    dW3, db3, da1, &b3);
    out[P + 7] = dW3;
    out[P + 8] = db3;
    Tensor dh1 = bn_backward(h1, OptT(a1), da1[0], g1.defined() ? OptT(g1) : OptT(), m1, i1,
                             need(ctx, P + 2), need(ctx, P + 3), dg1,
                             dbe1, nullptr, &be1);
    out[P + 2] = dg1;
    out[P + 3] = dbe1;
    std::vector<bool> need_a(nb);
    for (int64_t i = 0; i < nb; ++i) need_a[i] = need(ctx, i);
    std::vector<Tensor> dblocks;
    linear_backward(dh1, blocks, W0, need(ctx, P), need(ctx, P + 1), need_a,
                    dW0, db0, dblocks, &b0);
    out[P] = dW0;
    out[P + 1] = db0;
    for (int64_t i = 0; i < nb; ++i) out[i] = dblocks[i];
    return out;
  }
};

// ---------------------------------------------------------------------------
// boundary operator gathers
// ---------------------------------------------------------------------------
Tensor node_segment(const Tensor& rowptr, const Tensor& eids, int64_t n_nodes, int64_t n_edges,
                    const Tensor& x, const float* rs, float alpha) {
  Tensor out = at::empty({n_nodes, x.size(1)}, x.options());
  if (n_nodes > 0) {
    chk(hlhgat_incidence_step(rowptr.data_ptr<int>(), n_edges ? eids.data_ptr<int>() : nullptr,
                              nullptr, rs, n_nodes, 2 * n_edges, n_edges, x.data_ptr<float>(),
                              ld_of(x), x.size(1), nullptr, 0, alpha, 0.f,
                              out.data_ptr<float>(), ld_of(out), stream_of(x)),
        "incidence_step");
  }
  return out;
}

Tensor edge_gather(const Tensor& ei, int64_t n_edges, const Tensor& x, const float* sa,
                   const float* sb, float ca, float cb) {
  Tensor out = at::empty({n_edges, x.size(1)}, x.options());
  if (n_edges > 0) {
    chk(hlhgat_edge_gather2(ei.data_ptr<int64_t>(), n_edges, x.data_ptr<float>(), ld_of(x),
                            x.size(1), sa, sb, ca, cb, nullptr, 0, out.data_ptr<float>(),
                            ld_of(out), 0, stream_of(x)),
        "edge_gather2");
  }
  return out;
}

class NodeFromEdgesFn : public torch::autograd::Function<NodeFromEdgesFn> {
 public:
  // (1/D) |B1| x_s
  static Tensor forward(AutogradContext* ctx, Tensor x_s, Tensor rowptr, Tensor eids, Tensor ei,
                        Tensor rD, int64_t n_nodes) {
    req(x_s, "x_s");
    Tensor xs = rows2d(x_s);
    const int64_t E = ei.size(1);
    TORCH_CHECK(xs.size(0) == E, "hlhgat: x_s rows != |B1| edges");
    ctx->saved_data["n"] = n_nodes;
    ctx->save_for_backward({ei, rD});
    return node_segment(rowptr, eids, n_nodes, E, xs, rD.data_ptr<float>(), 1.f);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    Tensor g = rows2d(grads[0]);
    const float* rD = sv[1].data_ptr<float>();
    Tensor gx = edge_gather(sv[0], sv[0].size(1), g, rD, rD, 1.f, 1.f);
    return {gx, Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

class EdgeFromNodesFn : public torch::autograd::Function<EdgeFromNodesFn> {
 public:
  // |B1|^T x_t / 2
  static Tensor forward(AutogradContext* ctx, Tensor x_t, Tensor rowptr, Tensor eids, Tensor ei) {
    req(x_t, "x_t");
    Tensor xt = rows2d(x_t);
    ctx->saved_data["n"] = xt.size(0);
    ctx->save_for_backward({rowptr, eids, ei});
    return edge_gather(ei, ei.size(1), xt, nullptr, nullptr, 0.5f, 0.5f);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    Tensor g = rows2d(grads[0]);
    const int64_t n = ctx->saved_data["n"].toInt();
    Tensor gx = node_segment(sv[0], sv[1], n, sv[2].size(1), g, nullptr, 0.5f);
    return {gx, Tensor(), Tensor(), Tensor()};
  }
};

// ---------------------------------------------------------------------------
// NodeEdgeInt value path, both sides in one node, projected BEFORE the
// boundary-operator gathers (lib/Hodge_Cheb_Conv.py:293-295,307-308):
//
//   WV_Node(cat[(1/D)|B1| x_s, x_t]) first Linear
//     = x_t Wn_b^T + b_n + (1/D) |B1| (x_s Wn_a^T)
//   WV_Edge(cat[|B1|^T x_t / 2, x_s]) first Linear
//     = x_s We_b^T + b_e + |B1|^T (x_t We_a^T) / 2
//
// (W = [W_a | W_b] split at column d).  The gathers then run at the latent
// width dl = 64 instead of the growing input width d (64..384 in cfg2), the
// d-wide x_s2t / x_t2s are never materialised, and the two first-layer GEMMs
// become ONE per input with N = 2*dl:
//   Yt = x_t [Wn_b; We_a]^T  ->  [Qt | P2]      Ys = x_s [We_b; Wn_a]^T -> [Qs | P1]
//   h1_t = Qt + rD * |B1| P1                    h1_s = Qs + (P2[i] + P2[j]) / 2
// then BN -> ReLU -> Linear -> BN -> ReLU per side as in the reference.
// Same fp32 arithmetic up to summation order (1e-5 relative, tests).
// ---------------------------------------------------------------------------
// Rejoin every side stream that joined the capture of the current stream
// (hlhgat.train.TrainStep calls this as the last captured operation): a
// stream forked from the capture stream -- e.g. inside an autograd backward
// node, which runs on autograd's device thread -- and never waited on again
// leaves the capture "unjoined" at hipStreamEndCapture.  For each candidate
// stream (the C++ Fork side streams of `device` + `extra`, raw hipStream_t
// handles) whose capture id equals the current stream's, record an event on
// it and make the capture stream wait for it.  Returns the number rejoined.
int64_t join_capture_streams(int64_t device, std::vector<int64_t> extra) {
  hipStream_t cur = c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream();
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long cur_id = 0;
  TORCH_CHECK(hipStreamGetCaptureInfo(cur, &st, &cur_id) == hipSuccess,
              "hlhgat: hipStreamGetCaptureInfo");
  if (st != hipStreamCaptureStatusActive) return 0;
  std::vector<hipStream_t> cand;
  auto& reg = Fork::registry();
  auto it = reg.find((int)device);
  if (it != reg.end()) cand.push_back(it->second.stream());
  for (int64_t h : extra) cand.push_back(reinterpret_cast<hipStream_t>(h));
  int64_t n = 0;
  for (hipStream_t sd : cand) {
    if (sd == cur) continue;
    hipStreamCaptureStatus ss = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    if (hipStreamGetCaptureInfo(sd, &ss, &id) != hipSuccess) continue;
    if (ss != hipStreamCaptureStatusActive || id != cur_id) continue;
    hipEvent_t e = Fork::next_event();
    TORCH_CHECK(hipEventRecord(e, sd) == hipSuccess, "hlhgat: hipEventRecord (capture join)");
    TORCH_CHECK(hipStreamWaitEvent(cur, e, 0) == hipSuccess,
                "hlhgat: hipStreamWaitEvent (capture join)");
    ++n;
  }
  return n;
}

// Is `stream` (raw handle) still part of an active capture?
bool stream_capturing(int64_t stream) {
  hipStreamCaptureStatus ss = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  TORCH_CHECK(hipStreamGetCaptureInfo(reinterpret_cast<hipStream_t>(stream), &ss, &id) ==
                  hipSuccess,
              "hlhgat: hipStreamGetCaptureInfo");
  return ss == hipStreamCaptureStatusActive;
}

int64_t fork_side_stream(int64_t device) {
  return reinterpret_cast<int64_t>(Fork::side_of((int)device).stream());
}

struct SideMlp {  // [W0, b0, g1, be1, rm1, rv1, nbt1, W3, b3, g4, be4, rm4, rv4, nbt4]
  Tensor h1, a1, m1, i1, h2, y, m4, i4;
};

// Wt = [Wn_b; We_a], Ws = [We_b; Wn_a], bt = [b_n; 0], bs = [b_e; 0]
// (W0 = [W_a | W_b], lib/Hodge_Cheb_Conv.py:307-308) into one flat tensor
// [Wt | Ws | bt | bs]: both sides' first Linear on x_t (x_s) is ONE GEMM.
void pack_nei(CopyBlocks& cb, const Tensor& Wn, const Tensor& bn0, const Tensor& We,
              const Tensor& be0, int64_t d, int64_t dn, int64_t de, Tensor& pk) {
  const int64_t P = dn + de;
  float* base = pk.data_ptr<float>();
  float *Wt = base, *Ws = base + P * d, *bt = base + 2 * P * d, *bs = bt + P;
  const float *pwn = Wn.data_ptr<float>(), *pwe = We.data_ptr<float>();
  cb.add(pwn + d, Wn.stride(0), Wt, d, dn, d);
  cb.add(pwe, We.stride(0), Wt + dn * d, d, de, d);
  cb.add(pwe + d, We.stride(0), Ws, d, de, d);
  cb.add(pwn, Wn.stride(0), Ws + de * d, d, dn, d);
  cb.add(bn0.data_ptr<float>(), dn, bt, dn, 1, dn);
  cb.add(nullptr, 0, bt + dn, de, 1, de);
  cb.add(be0.data_ptr<float>(), de, bs, de, 1, de);
  cb.add(nullptr, 0, bs + de, dn, 1, dn);
}

// Every NodeEdgeInt's pack of one forward in one launch (hlhgat.ops.nei_prepack):
// groups[i] = {W0n, b0n, W0e, b0e}.
std::vector<Tensor> nei_prepack(std::vector<std::vector<Tensor>> groups) {
  std::vector<Tensor> out;
  CopyBlocks cb;
  void* s = nullptr;  // the current stream (nullptr is the legacy default stream)
  for (auto& g : groups) {
    TORCH_CHECK(g.size() == 4, "hlhgat: nei_prepack: {W0n, b0n, W0e, b0e} per module");
    Tensor Wn = g[0].stride(1) == 1 ? g[0] : g[0].contiguous();
    Tensor We = g[2].stride(1) == 1 ? g[2] : g[2].contiguous();
    Tensor bn0 = g[1].contiguous(), be0 = g[3].contiguous();
    req(Wn, "W0n");
    const int64_t d = Wn.size(1) / 2, dn = Wn.size(0), de = We.size(0);
    TORCH_CHECK(We.size(1) == 2 * d, "hlhgat: nei_prepack: W0n / W0e widths differ");
    Tensor pk = at::empty({2 * (dn + de) * d + 2 * (dn + de)}, Wn.options());
    if (cb.src.size() + 8 > (size_t)HLHGAT_MAX_COPY_BLOCKS) {
      cb.run(stream_of(Wn));
      cb = CopyBlocks();
    }
    pack_nei(cb, Wn, bn0, We, be0, d, dn, de, pk);
    s = stream_of(Wn);
    out.push_back(pk);
  }
  if (!groups.empty()) cb.run(s);
  return out;
}

// The DenseConcat gradient slab's host flag: 0 until a gradient has landed
// in the slab.  Returns the accumulate mode for this writer and marks the
// slab written (host-side, at backward issue: a captured graph replays the
// same sequence).
int sink_accumulate(AutogradContext* ctx, const char* key) {
  Tensor f = ctx->saved_data[key].toTensor();
  TORCH_CHECK(f.device().is_cpu() && f.scalar_type() == at::kInt && f.numel() == 1,
              "hlhgat: gradient-sink flag must be a CPU int32 [1]");
  int* w = f.data_ptr<int>();
  const int acc = *w != 0 ? 1 : 0;
  *w = 1;
  return acc;
}


// Chain mode (hlhgat.ops.Chains): the HL blocks' node and edge chains stay on
// their two streams for the whole block section of a forward, so the
// NodeEdgeInt forward neither waits for the main stream before its edge-side
// GEMM (its inputs come from the edge chain itself) nor joins the main stream
// at its end (the edge outputs feed the edge chain); only the exchange of the
// two first-layer GEMM results remains a cross-stream dependency.
bool& chain_flag() {
  static bool on = false;
  return on;
}
void set_chain(bool on) { chain_flag() = on; }
// the backward half of chain mode (test / A-B hook; on by default)
bool& chain_bwd_flag() {
  static bool on = true;
  return on;
}
void set_chain_bwd(bool on) { chain_bwd_flag() = on; }

class NEIntValueFn : public torch::autograd::Function<NEIntValueFn> {
 public:
  static variable_list forward(AutogradContext* ctx, Tensor x_t, Tensor x_s, Tensor rowptr,
                               Tensor eids, Tensor ei, Tensor rD, at::TensorList pn,
                               at::TensorList pe, double mom1n, double eps1n, double mom4n,
                               double eps4n, double mom1e, double eps1e, double mom4e,
                               double eps4e, OptT valid_t, OptT valid_s, OptT gsink_t,
                               OptT gsink_s, OptT gflag_t, OptT gflag_s, OptT packed) {
    req(x_t, "x_t");
    req(x_s, "x_s");
    TORCH_CHECK(pn.size() == 14 && pe.size() == 14, "hlhgat: nei_value expects 14+14 params");
    Tensor xt = rows2d(x_t), xs = rows2d(x_s);
    const int64_t N = xt.size(0), E = xs.size(0), d = xt.size(1);
    TORCH_CHECK(xs.size(1) == d, "hlhgat: NodeEdgeInt x_t / x_s widths differ");
    TORCH_CHECK(ei.size(1) == E, "hlhgat: x_s rows != |B1| edges");
    TORCH_CHECK(rD.numel() == N, "hlhgat: D has ", rD.numel(), " entries, x_t has ", N, " rows");
    const Tensor &W0n = pn[0], &W0e = pe[0];
    TORCH_CHECK(W0n.size(1) == 2 * d && W0e.size(1) == 2 * d, "hlhgat: WV first Linear expects ",
                2 * d, " input features");
    const int64_t dn = W0n.size(0), de = W0e.size(0);
    // Wt = [Wn_b; We_a], Ws = [We_b; Wn_a], bt = [b_n; 0], bs = [b_e; 0]: one launch
    Tensor Wn = W0n.stride(1) == 1 ? W0n : W0n.contiguous();
    Tensor We = W0e.stride(1) == 1 ? W0e : W0e.contiguous();
    Tensor bn0 = pn[1].contiguous(), be0 = pe[1].contiguous();
    const int64_t P = dn + de;
    Tensor Wt, Ws, bt, bs;
    if (has(packed)) {  // built for the whole forward by nei_prepack
      TORCH_CHECK(packed->numel() == 2 * P * d + 2 * P && packed->is_contiguous(),
                  "hlhgat: nei_value: packed weights have the wrong size");
      Wt = packed->narrow(0, 0, P * d).view({P, d});
      Ws = packed->narrow(0, P * d, P * d).view({P, d});
      bt = packed->narrow(0, 2 * P * d, P);
      bs = packed->narrow(0, 2 * P * d + P, P);
    } else {
      Tensor pk = at::empty({2 * P * d + 2 * P}, xt.options());
      CopyBlocks cb;
      pack_nei(cb, Wn, bn0, We, be0, d, dn, de, pk);
      cb.run(stream_of(xt));
      Wt = pk.narrow(0, 0, P * d).view({P, d});
      Ws = pk.narrow(0, P * d, P * d).view({P, d});
      bt = pk.narrow(0, 2 * P * d, P);
      bs = pk.narrow(0, 2 * P * d + P, P);
    }
    Fork fk(xt.get_device());
    const bool chain = chain_flag();
    // the edge GEMM needs this node's own weight pack (built on the main
    // stream above) unless a forward-wide pack (nei_prepack) was ordered before
    // the chains began; outside chain mode this also makes the side stream
    // part of a capture before anything is allocated on it
    if (!chain || !has(packed)) fk.side_waits_main();
    Tensor Yt = at::empty({N, dn + de}, xt.options());  // [Qt | P2]
    Tensor h1t = at::empty({N, dn}, xt.options());
    // Ys / h1s are first written on the side stream, which in chain mode does
    // not wait for the main stream: their blocks come from the side stream's
    // pool (a block main freed may still be read by main's queued kernels)
    Tensor Ys, h1s;
    {
      TStreamGuard g(fk.side);
      Ys = at::empty({E, de + dn}, xt.options());  // [Qs | P1]
      h1s = at::empty({E, de}, xt.options());
    }
    Ys.record_stream(fk.main);  // read by the node side's gather on main
    // the hidden layer's input rows: edge rows h1_s = Qs + (P2[i] + P2[j]) / 2
    // (hlhgat_edge_gather2), node rows h1_t = Qt + rD * |B1| P1 (hlhgat_poly_step
    // over the binary incidence), then its BatchNorm
    struct Producer {
      bool edge;
      const float* p;
      int64_t ldp;
      const float* z;
      int64_t ldz;
      float ca, cb;
    };
    auto side = [&](const at::TensorList& p, const Tensor& h1, double m1, double e1, double m4,
                    double e4, const OptT& valid, SideMlp& o, const Producer* pr) {
      o.h1 = h1;
      const BnState bst{p[2], p[3], p[4], p[5], p[6], m1, e1, valid};
      if (pr) {
        const int64_t n = h1.size(0), C = h1.size(1);
        if (pr->edge)
          chk(hlhgat_edge_gather2(ei.data_ptr<int64_t>(), n, pr->p, pr->ldp, (int)C, nullptr,
                                  nullptr, pr->ca, pr->cb, pr->z, pr->ldz, h1.data_ptr<float>(),
                                  ld_of(h1), 0, stream_of(h1)),
              "edge_gather2");
        else
          chk(hlhgat_incidence_step(rowptr.data_ptr<int>(), E ? eids.data_ptr<int>() : nullptr,
                                    nullptr, rD.data_ptr<float>(), n, 2 * E, E, pr->p, pr->ldp,
                                    (int)C, pr->z, pr->ldz, 1.f, 1.f, h1.data_ptr<float>(),
                                    ld_of(h1), stream_of(h1)),
              "incidence_step");
      }
      o.a1 = bn_forward(h1, bst, true, o.m1, o.i1);
      Tensor W3 = p[7].stride(1) == 1 ? p[7] : p[7].contiguous();
      o.y = linear_bn_forward({o.a1}, W3, p[8],
                              BnState{p[9], p[10], p[11], p[12], p[13], m4, e4, valid}, true,
                              o.h2, o.m4, o.i4);
    };
    auto lin_into = [](const Tensor& A, const Tensor& W, const Tensor& b, Tensor& out) {
      if (A.size(0) > 0)
        proj_fwd({A.data_ptr<float>()}, {ld_of(A)}, {W.data_ptr<float>()}, {W.stride(0)},
                 {A.size(1)}, A.size(0), W.size(0), b.data_ptr<float>(), out, stream_of(A));
    };
    SideMlp tn, te;
    // Yt is read on the side stream after the exchange (no join at the end in
    // chain mode): keep its block for the side stream
    if (chain) Yt.record_stream(fk.side);
    {  // edge side: first-layer GEMM on the side stream
      TStreamGuard g(fk.side);
      lin_into(xs, Ws, bs, Ys);
    }
    lin_into(xt, Wt, bt, Yt);
    fk.side_waits_main();  // side needs Yt
    fk.main_waits_side();  // main needs Ys
    {  // edge side: h1_s = Qs + (P2[i] + P2[j]) / 2, then its MLP
      TStreamGuard g(fk.side);
      const Producer pr{true, Yt.data_ptr<float>() + dn, dn + de,
                        Ys.data_ptr<float>(), de + dn, 0.5f, 0.5f};
      side(pe, h1s, mom1e, eps1e, mom4e, eps4e, valid_s, te, E > 0 ? &pr : nullptr);
    }
    {  // node side: h1_t = Qt + rD * |B1| P1, then its MLP
      const Producer pr{false, Ys.data_ptr<float>() + de, de + dn,
                        Yt.data_ptr<float>(), dn + de, 1.f, 1.f};
      side(pn, h1t, mom1n, eps1n, mom4n, eps4n, valid_t, tn, N > 0 ? &pr : nullptr);
    }
    if (!chain || tap_state().on) fk.main_waits_side();
    if (tap_state().on) {
      tap_state().taken.push_back(tn.a1.clone());
      tap_state().taken.push_back(te.a1.clone());
    }
    fk.escape({te.a1, te.m1, te.i1, te.h2, te.y, te.m4, te.i4});
    {
      EdgeMap em;
      for (int i = 0; i < 6; ++i) em.tensor();
      em.list(pn);
      em.list(pe);
      for (int i = 0; i < 8; ++i) em.other();
      em.opt(valid_t);
      em.opt(valid_s);
      em.opt(gsink_t);
      em.opt(gsink_s);
      em.opt(gflag_t);
      em.opt(gflag_s);
      em.opt(packed);
      ctx->saved_data["edges"] = em.e;
    }
    ctx->saved_data["dims"] = std::vector<int64_t>{N, E, d, dn, de};
    if (chain && chain_bwd_flag()) ctx->saved_data["chain"] = true;
    ctx->save_for_backward({xt, xs, rowptr, eids, ei, rD, Wt, Ws, pn[2], pn[7], pn[9], pe[2],
                            pe[7], pe[9], tn.h1, tn.a1, tn.m1, tn.i1, tn.h2, tn.y, tn.m4, tn.i4,
                            te.h1, te.a1, te.m1, te.i1, te.h2, te.y, te.m4, te.i4,
                            // 30..: W0, b0, be1, b3, be4 per side (gradient bucket targets)
                            pn[0], pn[1], pn[3], pn[8], pn[10], pe[0], pe[1], pe[3], pe[8],
                            pe[10],
                            // 40, 41: valid-row counts of the node / edge sides
                            has(valid_t) ? *valid_t : Tensor(), has(valid_s) ? *valid_s : Tensor()});
    // gradient sinks of x_t / x_s (DenseConcat slab views): kept outside the
    // saved variables -- other views' backwards add into the same slab in
    // place before this node's backward runs, which is the point
    // with a host int32 flag each ("slab written yet"): the first gradient to
    // land in a slab overwrites, the later ones add (no zero fill of the slab)
    if (has(gsink_t) && has(gflag_t)) {
      ctx->saved_data["gsink_t"] = *gsink_t;
      ctx->saved_data["gflag_t"] = *gflag_t;
    }
    if (has(gsink_s) && has(gflag_s)) {
      ctx->saved_data["gsink_s"] = *gsink_s;
      ctx->saved_data["gflag_s"] = *gflag_s;
    }
    return {tn.y, te.y};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    const auto dims = ctx->saved_data["dims"].toIntVector();
    const int64_t N = dims[0], E = dims[1], d = dims[2], dn = dims[3], de = dims[4];
    Tensor xt = sv[0], xs = sv[1], rowptr = sv[2], eids = sv[3], ei = sv[4], rD = sv[5],
           Wt = sv[6], Ws = sv[7];
    // positions: x_t 0, x_s 1, rowptr 2, eids 3, ei 4, rD 5, pn 6..19, pe 20..33, hyper 34..41,
    //            valid_t 42, valid_s 43, gsink_t 44, gsink_s 45, gflag_t 46, gflag_s 47,
    //            packed 48 (no gradient: the weights' gradients go to pn / pe)
    variable_list out(49);
    const int64_t PN = 6, PE = 20;
    auto side_bwd = [&](const Tensor& gy, int64_t P, const Tensor& g1, const Tensor& W3,
                        const Tensor& g4, int o0, Tensor dest, int q0, const Tensor& valid) {
      const Tensor &be1 = sv[q0 + 2], &b3 = sv[q0 + 3], &be4 = sv[q0 + 4];
      Tensor h1 = sv[o0], a1 = sv[o0 + 1], m1 = sv[o0 + 2], i1 = sv[o0 + 3], h2 = sv[o0 + 4],
             y = sv[o0 + 5], m4 = sv[o0 + 6], i4 = sv[o0 + 7];
      Tensor dg4, dbe4, dg1, dbe1, dW3, db3;
      Tensor gyc = gy.defined() ? gy : at::zeros_like(y);
      Tensor dh2 = bn_backward(h2, OptT(y), gyc, OptT(g4), m4, i4, need(ctx, P + 9),
                               need(ctx, P + 10), dg4, dbe4, nullptr, &be4, valid);
      std::vector<Tensor> da1;
      linear_backward(dh2, {a1}, W3, need(ctx, P + 7), need(ctx, P + 8), {true}, dW3, db3, da1,
                      &b3, nullptr, 1, false);
      bn_backward(h1, OptT(a1), da1[0], OptT(g1), m1, i1, need(ctx, P + 2), need(ctx, P + 3), dg1,
                  dbe1, &dest, &be1, valid);
      out[P + 2] = dg1;
      out[P + 3] = dbe1;
      out[P + 7] = dW3;
      out[P + 8] = db3;
      out[P + 9] = dg4;
      out[P + 10] = dbe4;
    };
    const bool nW = need(ctx, PN) || need(ctx, PE), nB = need(ctx, PN + 1) || need(ctx, PE + 1);
    // TrainStep: every unpack destination deferrable -> the Wt / Ws split
    // reductions are deferred too (their only reader is the deferred unpack)
    const bool fdef = need(ctx, PN) && need(ctx, PE) && need(ctx, PN + 1) &&
                      need(ctx, PE + 1) && param_deferrable(sv[30]) && param_deferrable(sv[35]) &&
                      param_deferrable(sv[31]) && param_deferrable(sv[36]);
    // chain mode (forward under ops.Chains) with every gradient deferred to the
    // flush: the edge half starts without waiting for the main stream (its
    // output gradient comes from the edge chain) and is not joined at the end
    // (its consumers are the edge chain and the flush, which waits for every
    // deferring stream); only the exchange stays
    const bool chain_b = fdef && ctx->saved_data.count("chain") > 0;
    Fork fk(xt.get_device());
    // outside chain mode the side stream waits for main first (which also
    // makes it part of a capture before anything is allocated on it)
    if (!chain_b) fk.side_waits_main();
    Tensor dYt = at::empty({N, dn + de}, xt.options());
    // dYs is first written on the side stream (which in chain mode does not
    // wait for main): a block of the side stream's pool, kept for main's read
    Tensor dYs;
    {
      TStreamGuard g(fk.side);
      dYs = at::empty({E, de + dn}, xt.options());
    }
    dYs.record_stream(fk.main);
    if (chain_b) dYt.record_stream(fk.side);
    {  // edge side MLP backward on the side stream -> dYs[:, :de]
      TStreamGuard g(fk.side);
      side_bwd(grads[1], PE, sv[11], sv[12], sv[13], 22, dYs.narrow(1, 0, de), 35, sv[41]);
    }
    side_bwd(grads[0], PN, sv[8], sv[9], sv[10], 14, dYt.narrow(1, 0, dn), 30, sv[40]);
    fk.side_waits_main();  // side needs dh1_t
    fk.main_waits_side();  // main needs dh1_s
    {  // dP1[e] = rD[i] dh1_t[i] + rD[j] dh1_t[j] -> dYs[:, de:], then the edge GEMM grads
      TStreamGuard g(fk.side);
      if (E > 0) {
        const float* r = rD.data_ptr<float>();
        chk(hlhgat_edge_gather2(ei.data_ptr<int64_t>(), E, dYt.data_ptr<float>(), dn + de, dn, r,
                                r, 1.f, 1.f, nullptr, 0, dYs.data_ptr<float>() + de, de + dn, 0,
                                fk.side.stream()),
            "edge_gather2(nei edge bwd)");
      }
    }
    // dP2[v] = 1/2 sum_{e ni v} dh1_s[e]  -> dYt[:, dn:]
    if (N > 0) {
      chk(hlhgat_incidence_step(rowptr.data_ptr<int>(), E ? eids.data_ptr<int>() : nullptr,
                                nullptr, nullptr, N, 2 * E, E, dYs.data_ptr<float>(), de + dn, de,
                                nullptr, 0, 0.5f, 0.f, dYt.data_ptr<float>() + dn, dn + de,
                                fk.main.stream()),
          "incidence_step(nei node bwd)");
    }
    Tensor dWt, dbt, dWs, dbs;
    std::vector<Tensor> dxt, dxs;
    {
      TStreamGuard g(fk.side);
      // x_s's gradient added straight into the dense slab's gradient (sink)
      const bool hs = ctx->saved_data.count("gsink_s") > 0;
      const std::vector<Tensor> into_s{hs ? ctx->saved_data["gsink_s"].toTensor() : Tensor()};
      linear_backward(dYs, {xs}, Ws, nW, nB, {need(ctx, 1)}, dWs, dbs, dxs, nullptr,
                      hs ? &into_s : nullptr, hs ? sink_accumulate(ctx, "gflag_s") : 0, fdef);
    }
    const bool ht = ctx->saved_data.count("gsink_t") > 0;
    const std::vector<Tensor> into_t{ht ? ctx->saved_data["gsink_t"].toTensor() : Tensor()};
    linear_backward(dYt, {xt}, Wt, nW, nB, {need(ctx, 0)}, dWt, dbt, dxt, nullptr,
                    ht ? &into_t : nullptr, ht ? sink_accumulate(ctx, "gflag_t") : 0, fdef);
    if (!chain_b) fk.main_waits_side();
    fk.escape({dWs, dbs, dxs[0], out[PE + 2], out[PE + 3], out[PE + 7], out[PE + 8], out[PE + 9],
               out[PE + 10]});
    out[0] = dxt[0];
    out[1] = dxs[0];
    {
      // Wt = [Wn_b; We_a], Ws = [We_b; Wn_a]  (W0 = [W_a | W_b]): unpack the
      // gradients (into the flat bucket when one is set) in one launch
      CopyBlocks cb;
      auto rows_into = [&](Tensor& g, const Tensor& src, int64_t r0, int64_t rows, int64_t c0) {
        cb.add(src.data_ptr<float>() + r0 * src.stride(0), src.stride(0),
               g.data_ptr<float>() + c0, g.stride(0), rows, d);
      };
      if (nW && need(ctx, PN)) {
        out[PN] = grad_like(sv[30]);
        TORCH_CHECK(out[PN].stride(1) == 1, "hlhgat: gradient of WV_Node[0] not row-major");
        rows_into(out[PN], dWs, de, dn, 0);
        rows_into(out[PN], dWt, 0, dn, d);
      }
      if (nW && need(ctx, PE)) {
        out[PE] = grad_like(sv[35]);
        TORCH_CHECK(out[PE].stride(1) == 1, "hlhgat: gradient of WV_Edge[0] not row-major");
        rows_into(out[PE], dWt, dn, de, 0);
        rows_into(out[PE], dWs, 0, de, d);
      }
      if (nB && need(ctx, PN + 1)) {
        out[PN + 1] = grad_like(sv[31]);
        cb.add(dbt.data_ptr<float>(), dn, out[PN + 1].data_ptr<float>(), dn, 1, dn);
      }
      if (nB && need(ctx, PE + 1)) {
        out[PE + 1] = grad_like(sv[36]);
        cb.add(dbs.data_ptr<float>(), de, out[PE + 1].data_ptr<float>(), de, 1, de);
      }
      // TrainStep: the unpack joins the deferred work flushed after the backward
      if (!defer_copies(cb, {out[PN], out[PE], out[PN + 1], out[PE + 1]},
                        {dWt, dWs, dbt, dbs}, stream_of(xt))) {
        TORCH_CHECK(!fdef, "hlhgat: NodeEdgeInt gradient reductions deferred but the unpack "
                           "could not be (set HLHGAT_DEFER_REDUCE=0)");
        cb.run(stream_of(xt));
      }
    }
    (void)d;
    return out;
  }
};

// ---------------------------------------------------------------------------
// python entry points
// ---------------------------------------------------------------------------
Tensor conv_bn(Tensor x, Tensor a_rowptr, Tensor a_col, OptT a_val, Tensor t_rowptr, Tensor t_col,
               OptT t_val, int64_t nnz, int64_t kind, std::vector<Tensor> W, OptT bias, OptT bn_w,
               OptT bn_b, OptT bn_rm, OptT bn_rv, OptT bn_nbt, double momentum, double eps,
               int64_t bn_mode, OptT out_buf, OptT a_order, OptT t_order, OptT valid,
               OptT h_tile, OptT h_ptr, OptT h_cols, OptT h_srp, OptT h_lcol, OptT h_sval,
               std::vector<int64_t> h_bounds, OptT h_hdr, std::vector<Tensor> fac,
               int64_t fac_nodes) {
  return ConvBNFn::apply(x, a_rowptr, a_col, a_val, t_rowptr, t_col, t_val, nnz, kind,
                         at::TensorList(W), bias, bn_w, bn_b, bn_rm, bn_rv, bn_nbt, momentum, eps,
                         bn_mode, out_buf, a_order, t_order, valid, h_tile, h_ptr, h_cols, h_srp, h_lcol, h_sval, h_bounds,
                         h_hdr, at::TensorList(fac), fac_nodes);
}

Tensor bn_act(Tensor x, OptT w, OptT b, OptT rm, OptT rv, OptT nbt, double momentum, double eps,
              bool relu, OptT valid) {
  return BNActFn::apply(x, w, b, rm, rv, nbt, momentum, eps, relu, valid);
}

Tensor linear(std::vector<Tensor> As, Tensor W, OptT b) {
  return LinearFn::apply(W, b, at::TensorList(As));
}

Tensor mlp2(std::vector<Tensor> blocks, Tensor W0, OptT b0, OptT g1, OptT be1, OptT rm1, OptT rv1,
            OptT nbt1, Tensor W3, OptT b3, OptT g4, OptT be4, OptT rm4, OptT rv4, OptT nbt4,
            double mom1, double eps1, double mom4, double eps4) {
  return MLP2Fn::apply(at::TensorList(blocks), W0, b0, g1, be1, rm1, rv1, nbt1, W3, b3, g4, be4,
                       rm4, rv4, nbt4, mom1, eps1, mom4, eps4);
}

Tensor node_from_edges(Tensor x_s, Tensor rowptr, Tensor eids, Tensor ei, Tensor rD,
                       int64_t n_nodes) {
  return NodeFromEdgesFn::apply(x_s, rowptr, eids, ei, rD, n_nodes);
}

Tensor edge_from_nodes(Tensor x_t, Tensor rowptr, Tensor eids, Tensor ei) {
  return EdgeFromNodesFn::apply(x_t, rowptr, eids, ei);
}

std::vector<Tensor> nei_value(Tensor x_t, Tensor x_s, Tensor rowptr, Tensor eids, Tensor ei,
                              Tensor rD, std::vector<Tensor> pn, std::vector<Tensor> pe,
                              double mom1n, double eps1n, double mom4n, double eps4n,
                              double mom1e, double eps1e, double mom4e, double eps4e,
                              OptT valid_t, OptT valid_s, OptT gsink_t, OptT gsink_s,
                              OptT gflag_t, OptT gflag_s, OptT packed) {
  auto r = NEIntValueFn::apply(x_t, x_s, rowptr, eids, ei, rD, at::TensorList(pn),
                               at::TensorList(pe), mom1n, eps1n, mom4n, eps4n, mom1e, eps1e,
                               mom4e, eps4e, valid_t, valid_s, gsink_t, gsink_s, gflag_t,
                               gflag_s, packed);
  return {r[0], r[1]};
}


// ---------------------------------------------------------------------------
// torch.ops.hlhgat: the native op boundary of SURVEY.md §8(b), registered with
// the dispatcher (schemas, HIP kernels under the CUDA key -- PyTorch-ROCm's
// key for device tensors --, Meta kernels for FakeTensor / torch.compile
// tracing, and Autograd kernels whose backward is itself a registered op).
// Contract: fp32 features, int32 CSR, outputs allocated on x's device, the
// current stream, errors as RuntimeError (TORCH_CHECK), no host sync.
//
//   spmm(rowptr, col, val?, x, t_rowptr?, t_col?, t_val?) -> y = A x
//       PyG propagate over a CSR keyed by edge_index[1] (lib/Hodge_Cheb_Conv.py:
//       442-443,518-519); the backward multiplies by A^T, given as the t_*
//       CSR or, when omitted, A itself (every Hodge Laplacian is symmetric).
//       Edge weights are data (no gradient), as in the reference models.
//   poly_basis(rowptr, col, val?, x, K, kind, t_*?) -> T [K-1, n, F]
//       T_1..T_{K-1} of the Laguerre (kind 0, :480-515), Chebyshev (1,
//       :394-439) or DEMO (2) recurrence; backward = the adjoint recurrence.
//   proj(A[], W, bias?) -> F.linear(cat(A, -1), W, bias) on fp32 MFMA
//       (the HodgeLaguerreConv projections and Linear(cat[..]), :307-308).
//   att_score(Qc, Qs, K, w_cross, w_self, sqrt_dk, sigma) -> a [n, 1]
//       NodeEdgeInt only_att (:297-305), sigma 0 = Sigmoid, 1 = ReLU.
//   segment_mean(x, seg_ptr, seg_rows?, n_seg) -> [n_seg, d]
//       global_mean_pool / scatter_mean.
//   csr_from_coo(row, col, val?, n_rows, sorted) -> (rowptr, col, val)
// ---------------------------------------------------------------------------
inline void req_i32(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.dim() == 1 && t.is_contiguous(),
              "hlhgat: ", name, " must be a contiguous int32 1-D ROCm tensor");
}
inline void req_csr(const Tensor& rowptr, const Tensor& col, const OptT& val) {
  req_i32(rowptr, "rowptr");
  req_i32(col, "col");
  TORCH_CHECK(rowptr.numel() >= 1, "hlhgat: rowptr needs n_rows + 1 >= 1 entries");
  TORCH_CHECK(col.numel() < ((int64_t)1 << 31), "hlhgat: nnz must be < 2^31");
  if (has(val))
    TORCH_CHECK(val->is_cuda() && val->scalar_type() == at::kFloat && val->is_contiguous() &&
                    val->numel() == col.numel(),
                "hlhgat: val must be contiguous fp32 with one entry per column index");
}
inline void req_x(const Tensor& x, const char* name) {
  req(x, name);
  TORCH_CHECK(x.dim() == 2, "hlhgat: ", name, " must be 2-D");
}

Tensor spmm_hip(const Tensor& rowptr, const Tensor& col, const OptT& val, const Tensor& x,
                const OptT& t_rowptr, const OptT& t_col, const OptT& t_val) {
  (void)t_rowptr, (void)t_col, (void)t_val;
  req_csr(rowptr, col, val);
  req_x(x, "x");
  const int64_t n = rowptr.numel() - 1, nnz = col.numel();
  Tensor xc = rows2d(x);
  Tensor y = at::empty({n, xc.size(1)}, xc.options());
  if (n > 0 && xc.size(1) > 0)
    chk(hlhgat_spmm(rowptr.data_ptr<int>(), nnz ? col.data_ptr<int>() : nullptr,
                    nnz ? fptr(val) : nullptr, n, nnz, nullptr, nullptr, xc.data_ptr<float>(),
                    ld_of(xc), xc.size(1), y.data_ptr<float>(), ld_of(y), stream_of(xc)),
        "spmm");
  return y;
}
Tensor spmm_meta(const Tensor& rowptr, const Tensor& col, const OptT& val, const Tensor& x,
                 const OptT&, const OptT&, const OptT&) {
  (void)col, (void)val;
  return at::empty_symint({rowptr.sym_size(0) - 1, x.sym_size(1)}, x.options());
}

Tensor poly_basis_hip(const Tensor& rowptr, const Tensor& col, const OptT& val, const Tensor& x,
                      int64_t K, int64_t kind, const OptT&, const OptT&, const OptT&) {
  req_csr(rowptr, col, val);
  req_x(x, "x");
  TORCH_CHECK(K >= 1 && kind >= 0 && kind <= 2, "hlhgat: poly_basis needs K >= 1, kind 0..2");
  const int64_t n = rowptr.numel() - 1, nnz = col.numel();
  TORCH_CHECK(x.size(0) == n, "hlhgat: x has ", x.size(0), " rows, the operator ", n);
  Tensor xc = rows2d(x);
  const int64_t F = xc.size(1);
  Tensor T = at::empty({K - 1, n, F}, xc.options());
  if (K > 1 && n > 0 && F > 0)
    chk(hlhgat_poly_basis_fwd((int)kind, rowptr.data_ptr<int>(),
                              nnz ? col.data_ptr<int>() : nullptr, nnz ? fptr(val) : nullptr, n,
                              nnz, nullptr, nullptr, xc.data_ptr<float>(),
                              ld_of(xc), F, (int)K, T.data_ptr<float>(), stream_of(xc)),
        "poly_basis_fwd");
  return T;
}
Tensor poly_basis_meta(const Tensor& rowptr, const Tensor&, const OptT&, const Tensor& x,
                       int64_t K, int64_t, const OptT&, const OptT&, const OptT&) {
  return at::empty_symint({c10::SymInt(K - 1), rowptr.sym_size(0) - 1, x.sym_size(1)},
                          x.options());
}

// gx of poly_basis given dT [K-1, n, F] (the adjoint recurrence over A^T)
Tensor poly_basis_backward_hip(const Tensor& grad, const Tensor& rowptr, const Tensor& col,
                               const OptT& val, int64_t K, int64_t kind) {
  req_csr(rowptr, col, val);
  const int64_t n = rowptr.numel() - 1, nnz = col.numel();
  TORCH_CHECK(grad.dim() == 3 && grad.size(0) == K - 1 && grad.size(1) == n,
              "hlhgat: poly_basis_backward: grad must be [K-1, n, F]");
  const int64_t F = grad.size(2);
  Tensor Gs = at::empty({K, n, F}, grad.options());
  Gs[0].zero_();
  if (K > 1) Gs.narrow(0, 1, K - 1).copy_(grad);
  if (K > 1 && n > 0 && F > 0)
    chk(hlhgat_poly_basis_bwd((int)kind, rowptr.data_ptr<int>(),
                              nnz ? col.data_ptr<int>() : nullptr, nnz ? fptr(val) : nullptr, n,
                              nnz, nullptr, nullptr, F, (int)K,
                              Gs.data_ptr<float>(), stream_of(grad)),
        "poly_basis_bwd");
  return Gs[0].clone();
}
Tensor poly_basis_backward_meta(const Tensor& grad, const Tensor&, const Tensor&, const OptT&,
                                int64_t, int64_t) {
  return at::empty_symint({grad.sym_size(1), grad.sym_size(2)}, grad.options());
}

Tensor proj_hip(at::TensorList A, const Tensor& W, const OptT& bias) {
  TORCH_CHECK(!A.empty() && (int64_t)A.size() <= HLHGAT_MAX_BLOCKS, "hlhgat: proj takes 1..",
              HLHGAT_MAX_BLOCKS, " operand blocks");
  req(W, "W");
  TORCH_CHECK(W.dim() == 2, "hlhgat: W must be [N, sum K_b]");
  std::vector<Tensor> As;
  for (const auto& a : A) {
    req_x(a, "A_b");
    TORCH_CHECK(a.size(0) == A[0].size(0), "hlhgat: proj blocks must have equal rows");
    As.push_back(rows2d(a));
  }
  if (has(bias)) req(*bias, "bias");
  Tensor Wc = W.stride(1) == 1 ? W : W.contiguous();
  return linear_forward(As, Wc, bias);
}
Tensor proj_meta(at::TensorList A, const Tensor& W, const OptT&) {
  return at::empty_symint({A[0].sym_size(0), W.sym_size(0)}, W.options());
}
std::tuple<Tensor, Tensor, std::vector<Tensor>> proj_backward_hip(const Tensor& grad,
                                                                   at::TensorList A,
                                                                   const Tensor& W,
                                                                   bool has_bias) {
  std::vector<Tensor> As;
  for (const auto& a : A) As.push_back(rows2d(a));
  Tensor Wc = W.stride(1) == 1 ? W : W.contiguous();
  Tensor dW, db;
  std::vector<Tensor> dAs;
  linear_backward(grad, As, Wc, true, has_bias, std::vector<bool>(As.size(), true), dW, db, dAs);
  if (!db.defined()) db = at::empty({0}, W.options());
  return {dW, db, dAs};
}
std::tuple<Tensor, Tensor, std::vector<Tensor>> proj_backward_meta(const Tensor& grad,
                                                                    at::TensorList A,
                                                                    const Tensor& W,
                                                                    bool has_bias) {
  std::vector<Tensor> dAs;
  for (const auto& a : A) dAs.push_back(at::empty_symint(a.sym_sizes(), a.options()));
  return {at::empty_symint(W.sym_sizes(), W.options()),
          at::empty_symint({has_bias ? W.sym_size(0) : c10::SymInt(0)}, W.options()), dAs};
}

Tensor att_score_hip(const Tensor& Qc, const Tensor& Qs, const Tensor& K, double w_cross,
                     double w_self, double sqrt_dk, int64_t sigma) {
  req_x(Qc, "Qc");
  req_x(Qs, "Qs");
  req_x(K, "K");
  TORCH_CHECK(Qc.sizes() == K.sizes() && Qs.sizes() == K.sizes(),
              "hlhgat: att_score: Qc, Qs and K must have one shape [n, dk]");
  Tensor qc = rows2d(Qc), qs = rows2d(Qs), k = rows2d(K);
  Tensor a = at::empty({k.size(0), 1}, k.options());
  if (k.size(0) > 0)
    chk(hlhgat_att_score_fwd(k.size(0), k.size(1), qc.data_ptr<float>(), ld_of(qc),
                             qs.data_ptr<float>(), ld_of(qs), k.data_ptr<float>(), ld_of(k),
                             (float)w_cross, (float)w_self, (float)sqrt_dk, (int)sigma,
                             a.data_ptr<float>(), stream_of(k)),
        "att_score_fwd");
  return a;
}
Tensor att_score_meta(const Tensor&, const Tensor&, const Tensor& K, double, double, double,
                      int64_t) {
  return at::empty_symint({K.sym_size(0), c10::SymInt(1)}, K.options());
}
std::tuple<Tensor, Tensor, Tensor> att_score_backward_hip(const Tensor& grad, const Tensor& Qc,
                                                          const Tensor& Qs, const Tensor& K,
                                                          const Tensor& a, double w_cross,
                                                          double w_self, double sqrt_dk,
                                                          int64_t sigma) {
  Tensor qc = rows2d(Qc), qs = rows2d(Qs), k = rows2d(K);
  Tensor ga = grad.contiguous();
  const int64_t n = k.size(0), dk = k.size(1);
  Tensor g = at::empty({3, n, dk}, k.options());
  if (n > 0)
    chk(hlhgat_att_score_bwd(n, dk, qc.data_ptr<float>(), ld_of(qc), qs.data_ptr<float>(),
                             ld_of(qs), k.data_ptr<float>(), ld_of(k), (float)w_cross,
                             (float)w_self, (float)sqrt_dk, (int)sigma, a.data_ptr<float>(),
                             ga.data_ptr<float>(), g[0].data_ptr<float>(), g[1].data_ptr<float>(),
                             g[2].data_ptr<float>(), dk, stream_of(k)),
        "att_score_bwd");
  return {g[0], g[1], g[2]};
}
std::tuple<Tensor, Tensor, Tensor> att_score_backward_meta(const Tensor&, const Tensor& Qc,
                                                           const Tensor& Qs, const Tensor& K,
                                                           const Tensor&, double, double, double,
                                                           int64_t) {
  return {at::empty_symint(Qc.sym_sizes(), Qc.options()),
          at::empty_symint(Qs.sym_sizes(), Qs.options()),
          at::empty_symint(K.sym_sizes(), K.options())};
}

Tensor segment_mean_hip(const Tensor& x, const Tensor& seg_ptr, const OptT& seg_rows,
                        int64_t n_seg) {
  req_x(x, "x");
  req_i32(seg_ptr, "seg_ptr");
  TORCH_CHECK(seg_ptr.numel() == n_seg + 1, "hlhgat: seg_ptr must have n_seg + 1 entries");
  if (has(seg_rows)) req_i32(*seg_rows, "seg_rows");
  Tensor xc = rows2d(x);
  Tensor out = at::empty({n_seg, xc.size(1)}, xc.options());
  if (n_seg > 0)
    chk(hlhgat_segment_mean_fwd(seg_ptr.data_ptr<int>(), iptr(seg_rows), n_seg,
                                xc.data_ptr<float>(), ld_of(xc), xc.size(1),
                                out.data_ptr<float>(), ld_of(out), stream_of(xc)),
        "segment_mean_fwd");
  return out;
}
Tensor segment_mean_meta(const Tensor& x, const Tensor&, const OptT&, int64_t n_seg) {
  return at::empty_symint({c10::SymInt(n_seg), x.sym_size(1)}, x.options());
}
Tensor segment_mean_backward_hip(const Tensor& grad, const Tensor& seg_ptr, const OptT& seg_rows,
                                 int64_t n_rows) {
  Tensor g = rows2d(grad);
  const int64_t n_seg = seg_ptr.numel() - 1;
  Tensor gx = has(seg_rows) ? at::zeros({n_rows, g.size(1)}, g.options())
                            : at::empty({n_rows, g.size(1)}, g.options());
  if (n_rows > 0)
    chk(hlhgat_segment_mean_bwd(seg_ptr.data_ptr<int>(), iptr(seg_rows), n_seg,
                                g.data_ptr<float>(), ld_of(g), g.size(1), gx.data_ptr<float>(),
                                ld_of(gx), n_rows, stream_of(g)),
        "segment_mean_bwd");
  return gx;
}
Tensor segment_mean_backward_meta(const Tensor& grad, const Tensor&, const OptT&,
                                  int64_t n_rows) {
  return at::empty_symint({c10::SymInt(n_rows), grad.sym_size(1)}, grad.options());
}

std::tuple<Tensor, Tensor, Tensor> csr_from_coo_hip(const Tensor& row, const Tensor& col,
                                                    const OptT& val, int64_t n_rows,
                                                    bool sorted) {
  TORCH_CHECK(row.is_cuda() && col.is_cuda() && row.scalar_type() == at::kLong &&
                  col.scalar_type() == at::kLong && row.dim() == 1 && row.sizes() == col.sizes(),
              "hlhgat: csr_from_coo needs int64 ROCm row / col of one length");
  const int64_t nnz = row.numel();
  TORCH_CHECK(nnz < ((int64_t)1 << 31), "hlhgat: nnz must be < 2^31");
  Tensor r = row.contiguous(), c = col.contiguous();
  OptT v = has(val) ? OptT(val->contiguous()) : OptT();
  if (has(v)) req(*v, "val");
  Tensor rowptr = at::empty({n_rows + 1}, r.options().dtype(at::kInt));
  Tensor col32 = at::empty({nnz}, r.options().dtype(at::kInt));
  Tensor val32 = at::empty({has(v) ? nnz : 0}, r.options().dtype(at::kFloat));
  void* s = stream_of(r);
  if (sorted) {
    chk(hlhgat_csr_from_sorted_coo(r.data_ptr<int64_t>(), c.data_ptr<int64_t>(), fptr(v), nnz,
                                   n_rows, rowptr.data_ptr<int>(), col32.data_ptr<int>(),
                                   has(v) ? val32.data_ptr<float>() : nullptr, s),
        "csr_from_sorted_coo");
  } else {
    const int64_t wsb = (int64_t)hlhgat_csr_workspace_bytes(nnz);
    Tensor ws = at::empty({std::max<int64_t>(wsb, 1)}, r.options().dtype(at::kByte));
    int64_t n_cols = 1;  // only bounds the sort key: any value > max(col) works
    if (nnz) n_cols = c.max().item<int64_t>() + 1;  // host sync: general (unsorted) path only
    chk(hlhgat_csr_from_coo(nnz ? r.data_ptr<int64_t>() : nullptr,
                            nnz ? c.data_ptr<int64_t>() : nullptr, fptr(v), nnz, n_rows, n_cols,
                            rowptr.data_ptr<int>(), nnz ? col32.data_ptr<int>() : nullptr,
                            (has(v) && nnz) ? val32.data_ptr<float>() : nullptr, nullptr,
                            ws.data_ptr(), (size_t)wsb, s),
        "csr_from_coo");
  }
  return {rowptr, col32, val32};
}
std::tuple<Tensor, Tensor, Tensor> csr_from_coo_meta(const Tensor& row, const Tensor&,
                                                     const OptT& val, int64_t n_rows, bool) {
  auto o = row.options();
  return {at::empty({n_rows + 1}, o.dtype(at::kInt)), at::empty_symint(row.sym_sizes(),
                                                                       o.dtype(at::kInt)),
          at::empty_symint({has(val) ? row.sym_size(0) : c10::SymInt(0)}, o.dtype(at::kFloat))};
}

// --- autograd over the dispatcher ---------------------------------------------
template <typename Sig>
c10::TypedOperatorHandle<Sig> op_handle(const char* name) {
  return c10::Dispatcher::singleton().findSchemaOrThrow(name, "").typed<Sig>();
}
using SpmmSig = Tensor(const Tensor&, const Tensor&, const OptT&, const Tensor&, const OptT&,
                       const OptT&, const OptT&);
using BasisSig = Tensor(const Tensor&, const Tensor&, const OptT&, const Tensor&, int64_t, int64_t,
                        const OptT&, const OptT&, const OptT&);
using BasisBwdSig = Tensor(const Tensor&, const Tensor&, const Tensor&, const OptT&, int64_t,
                           int64_t);
using ProjSig = Tensor(at::TensorList, const Tensor&, const OptT&);
using ProjBwdSig = std::tuple<Tensor, Tensor, std::vector<Tensor>>(const Tensor&, at::TensorList,
                                                                   const Tensor&, bool);
using AttSig = Tensor(const Tensor&, const Tensor&, const Tensor&, double, double, double,
                      int64_t);
using AttBwdSig = std::tuple<Tensor, Tensor, Tensor>(const Tensor&, const Tensor&, const Tensor&,
                                                     const Tensor&, const Tensor&, double, double,
                                                     double, int64_t);
using SegSig = Tensor(const Tensor&, const Tensor&, const OptT&, int64_t);
using SegBwdSig = Tensor(const Tensor&, const Tensor&, const OptT&, int64_t);

inline Tensor opt_or_undef(const OptT& t) { return has(t) ? *t : Tensor(); }
inline OptT undef_to_opt(const Tensor& t) { return t.defined() ? OptT(t) : OptT(); }

class SpmmOp : public torch::autograd::Function<SpmmOp> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& rowptr, const Tensor& col,
                        const OptT& val, const Tensor& x, const OptT& t_rowptr, const OptT& t_col,
                        const OptT& t_val) {
    at::AutoDispatchBelowADInplaceOrView g;
    const bool t = has(t_rowptr);
    ctx->save_for_backward({t ? *t_rowptr : rowptr, t ? *t_col : col,
                            t ? opt_or_undef(t_val) : opt_or_undef(val)});
    static auto op = op_handle<SpmmSig>("hlhgat::spmm");
    return op.call(rowptr, col, val, x, t_rowptr, t_col, t_val);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    static auto op = op_handle<SpmmSig>("hlhgat::spmm");
    Tensor gx = op.call(sv[0], sv[1], undef_to_opt(sv[2]), grads[0], OptT(), OptT(), OptT());
    return {Tensor(), Tensor(), Tensor(), gx, Tensor(), Tensor(), Tensor()};
  }
};

class BasisOp : public torch::autograd::Function<BasisOp> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& rowptr, const Tensor& col,
                        const OptT& val, const Tensor& x, int64_t K, int64_t kind,
                        const OptT& t_rowptr, const OptT& t_col, const OptT& t_val) {
    at::AutoDispatchBelowADInplaceOrView g;
    const bool t = has(t_rowptr);
    ctx->save_for_backward({t ? *t_rowptr : rowptr, t ? *t_col : col,
                            t ? opt_or_undef(t_val) : opt_or_undef(val)});
    ctx->saved_data["K"] = K;
    ctx->saved_data["kind"] = kind;
    static auto op = op_handle<BasisSig>("hlhgat::poly_basis");
    return op.call(rowptr, col, val, x, K, kind, t_rowptr, t_col, t_val);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    static auto op = op_handle<BasisBwdSig>("hlhgat::poly_basis_backward");
    Tensor gx = op.call(grads[0].contiguous(), sv[0], sv[1], undef_to_opt(sv[2]),
                        ctx->saved_data["K"].toInt(), ctx->saved_data["kind"].toInt());
    return {Tensor(), Tensor(), Tensor(), gx, Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

class ProjOp : public torch::autograd::Function<ProjOp> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& W, const OptT& bias,
                        at::TensorList A) {
    at::AutoDispatchBelowADInplaceOrView g;
    std::vector<Tensor> save(A.begin(), A.end());
    save.push_back(W);
    ctx->save_for_backward(save);
    ctx->saved_data["has_b"] = has(bias);
    static auto op = op_handle<ProjSig>("hlhgat::proj");
    return op.call(A, W, bias);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    Tensor W = sv.back();
    std::vector<Tensor> A(sv.begin(), sv.end() - 1);
    const bool hb = ctx->saved_data["has_b"].toBool();
    static auto op = op_handle<ProjBwdSig>("hlhgat::proj_backward");
    auto r = op.call(grads[0], A, W, hb);
    variable_list out = {std::get<0>(r), hb ? std::get<1>(r) : Tensor()};
    for (auto& t : std::get<2>(r)) out.push_back(t);
    return out;
  }
};

class AttOp : public torch::autograd::Function<AttOp> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& Qc, const Tensor& Qs, const Tensor& K,
                        double wc, double ws, double sq, int64_t sigma) {
    at::AutoDispatchBelowADInplaceOrView g;
    static auto op = op_handle<AttSig>("hlhgat::att_score");
    Tensor a = op.call(Qc, Qs, K, wc, ws, sq, sigma);
    ctx->save_for_backward({Qc, Qs, K, a});
    ctx->saved_data["c"] = std::vector<double>{wc, ws, sq};
    ctx->saved_data["sigma"] = sigma;
    return a;
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    auto c = ctx->saved_data["c"].toDoubleVector();
    static auto op = op_handle<AttBwdSig>("hlhgat::att_score_backward");
    auto r = op.call(grads[0], sv[0], sv[1], sv[2], sv[3], c[0], c[1], c[2],
                     ctx->saved_data["sigma"].toInt());
    return {std::get<0>(r), std::get<1>(r), std::get<2>(r), Tensor(), Tensor(), Tensor(),
            Tensor()};
  }
};

class SegOp : public torch::autograd::Function<SegOp> {
 public:
  static Tensor forward(AutogradContext* ctx, const Tensor& x, const Tensor& seg_ptr,
                        const OptT& seg_rows, int64_t n_seg) {
    at::AutoDispatchBelowADInplaceOrView g;
    ctx->save_for_backward({seg_ptr, opt_or_undef(seg_rows)});
    ctx->saved_data["n"] = x.sym_size(0).guard_int(__FILE__, __LINE__);
    static auto op = op_handle<SegSig>("hlhgat::segment_mean");
    return op.call(x, seg_ptr, seg_rows, n_seg);
  }
  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    auto sv = ctx->get_saved_variables();
    static auto op = op_handle<SegBwdSig>("hlhgat::segment_mean_backward");
    return {op.call(grads[0], sv[0], undef_to_opt(sv[1]), ctx->saved_data["n"].toInt()),
            Tensor(), Tensor(), Tensor()};
  }
};

Tensor spmm_ad(const Tensor& rowptr, const Tensor& col, const OptT& val, const Tensor& x,
               const OptT& tr, const OptT& tc, const OptT& tv) {
  return SpmmOp::apply(rowptr, col, val, x, tr, tc, tv);
}
Tensor poly_basis_ad(const Tensor& rowptr, const Tensor& col, const OptT& val, const Tensor& x,
                     int64_t K, int64_t kind, const OptT& tr, const OptT& tc, const OptT& tv) {
  return BasisOp::apply(rowptr, col, val, x, K, kind, tr, tc, tv);
}
Tensor proj_ad(at::TensorList A, const Tensor& W, const OptT& bias) {
  return ProjOp::apply(W, bias, A);
}
Tensor att_score_ad(const Tensor& Qc, const Tensor& Qs, const Tensor& K, double wc, double ws,
                    double sq, int64_t sigma) {
  return AttOp::apply(Qc, Qs, K, wc, ws, sq, sigma);
}
Tensor segment_mean_ad(const Tensor& x, const Tensor& seg_ptr, const OptT& seg_rows,
                       int64_t n_seg) {
  return SegOp::apply(x, seg_ptr, seg_rows, n_seg);
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "hlhgat C++ autograd nodes over the libhlhgat C-ABI";
  m.def("conv_bn", &conv_bn);
  m.def("set_fused_bwd", &set_fused_bwd);
  m.def("set_tap", &set_tap);
  m.def("take_tap", &take_tap);
  m.def("join_capture_streams", &join_capture_streams);
  m.def("stream_capturing", &stream_capturing);
  m.def("fork_side_stream", &fork_side_stream);
  m.def("bn_act", &bn_act);
  m.def("linear", &linear);
  m.def("mlp2", &mlp2);
  m.def("nei_value", &nei_value);
  m.def("set_chain", &set_chain);
  m.def("bn_workspace_reserve", &bn_workspace_reserve);
  m.def("set_chain_bwd", &set_chain_bwd);
  m.def("nei_prepack", &nei_prepack);
  m.def("grad_bucket_set", &grad_bucket_set);
  m.def("grad_bucket_begin", &grad_bucket_begin);
  m.def("grad_bucket_clear", &grad_bucket_clear);
  m.def("grad_bucket_no_defer", &grad_bucket_no_defer);
  m.def("reduce_defer", &reduce_defer);
  m.def("reduce_flush", &reduce_flush);
  m.def("node_from_edges", &node_from_edges);
  m.def("edge_from_nodes", &edge_from_nodes);
  m.def("version", []() { return hlhgat_version(); });
}

TORCH_LIBRARY(hlhgat, m) {
  m.def("spmm(Tensor rowptr, Tensor col, Tensor? val, Tensor x, Tensor? t_rowptr=None, "
        "Tensor? t_col=None, Tensor? t_val=None) -> Tensor");
  m.def("poly_basis(Tensor rowptr, Tensor col, Tensor? val, Tensor x, int K, int kind, "
        "Tensor? t_rowptr=None, Tensor? t_col=None, Tensor? t_val=None) -> Tensor");
  m.def("poly_basis_backward(Tensor grad, Tensor rowptr, Tensor col, Tensor? val, int K, "
        "int kind) -> Tensor");
  m.def("proj(Tensor[] A, Tensor W, Tensor? bias) -> Tensor");
  m.def("proj_backward(Tensor grad, Tensor[] A, Tensor W, bool has_bias) -> "
        "(Tensor, Tensor, Tensor[])");
  m.def("att_score(Tensor Qc, Tensor Qs, Tensor K, float w_cross, float w_self, float sqrt_dk, "
        "int sigma) -> Tensor");
  m.def("att_score_backward(Tensor grad, Tensor Qc, Tensor Qs, Tensor K, Tensor a, "
        "float w_cross, float w_self, float sqrt_dk, int sigma) -> (Tensor, Tensor, Tensor)");
  m.def("segment_mean(Tensor x, Tensor seg_ptr, Tensor? seg_rows, int n_seg) -> Tensor");
  m.def("segment_mean_backward(Tensor grad, Tensor seg_ptr, Tensor? seg_rows, int n_rows) -> "
        "Tensor");
  m.def("csr_from_coo(Tensor row, Tensor col, Tensor? val, int n_rows, bool sorted) -> "
        "(Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(hlhgat, CUDA, m) {  // PyTorch-ROCm dispatches HIP tensors under CUDA
  m.impl("spmm", &spmm_hip);
  m.impl("poly_basis", &poly_basis_hip);
  m.impl("poly_basis_backward", &poly_basis_backward_hip);
  m.impl("proj", &proj_hip);
  m.impl("proj_backward", &proj_backward_hip);
  m.impl("att_score", &att_score_hip);
  m.impl("att_score_backward", &att_score_backward_hip);
  m.impl("segment_mean", &segment_mean_hip);
  m.impl("segment_mean_backward", &segment_mean_backward_hip);
  m.impl("csr_from_coo", &csr_from_coo_hip);
}

TORCH_LIBRARY_IMPL(hlhgat, Meta, m) {
  m.impl("spmm", &spmm_meta);
  m.impl("poly_basis", &poly_basis_meta);
  m.impl("poly_basis_backward", &poly_basis_backward_meta);
  m.impl("proj", &proj_meta);
  m.impl("proj_backward", &proj_backward_meta);
  m.impl("att_score", &att_score_meta);
  m.impl("att_score_backward", &att_score_backward_meta);
  m.impl("segment_mean", &segment_mean_meta);
  m.impl("segment_mean_backward", &segment_mean_backward_meta);
  m.impl("csr_from_coo", &csr_from_coo_meta);
}

TORCH_LIBRARY_IMPL(hlhgat, Autograd, m) {
  m.impl("spmm", &spmm_ad);
  m.impl("poly_basis", &poly_basis_ad);
  m.impl("proj", &proj_ad);
  m.impl("att_score", &att_score_ad);
  m.impl("segment_mean", &segment_mean_ad);
}
