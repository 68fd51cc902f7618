// Library-level state: error messages, version, live kernel timing.
#include "common.h"

#include <cstring>
#include <mutex>
#include <vector>

namespace hlhgat {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

// --- live timing -----------------------------------------------------------
// A fixed pool of hipEvent pairs per kernel class, stamped by
// hipExtLaunchKernel at kernel start / end (common.h: launch()).  Records are
// appended in launch order; hlhgat_prof_read() synchronises them and sums the
// kernel durations.
namespace {
constexpr int kPoolSize = 1 << 14;
struct ProfClass {
  bool enabled = false;
  std::vector<hipEvent_t> start, stop;
  std::vector<double> bytes, flops;
  int used = 0;
  int64_t dropped = 0;
};
std::mutex g_prof_mu;
ProfClass g_prof[HLHGAT_PROF_NCLASS];
}  // namespace

ProfScope::ProfScope(int kernel_class, hipStream_t s, double b, double f)
    : cls(kernel_class), bytes(b), flops(f) {
  (void)s;
  if (kernel_class < 0 || kernel_class >= HLHGAT_PROF_NCLASS) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  ProfClass& pc = g_prof[kernel_class];
  if (!pc.enabled) return;
  if (pc.used >= (int)pc.start.size()) {
    pc.dropped++;
    return;
  }
  slot = pc.used++;
  pc.bytes[slot] = b;
  pc.flops[slot] = f;
  start_ev = pc.start[slot];
  stop_ev = pc.stop[slot];
}

// --- device error word -------------------------------------------------------
// One pinned, mapped, coherent host word shared by all devices: kernels store
// an HLHGAT_DEVERR_* code into it with plain system-scope stores (no PCIe
// atomics; reporters of different codes may overwrite each other, so any
// nonzero value means "do not use these results"), the host reads it without
// synchronising.
namespace {
std::mutex g_err_mu;
unsigned* g_err_word = nullptr;
}  // namespace

unsigned* device_error_word() {
  std::lock_guard<std::mutex> lk(g_err_mu);
  if (!g_err_word) {
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, 64, hipHostMallocPortable | hipHostMallocMapped |
                                             hipHostMallocCoherent);
    if (e != hipSuccess) {
      set_error("hipHostMalloc(device error word) failed: %s", hipGetErrorString(e));
      return nullptr;
    }
    *static_cast<volatile unsigned*>(p) = 0u;
    g_err_word = static_cast<unsigned*>(p);
  }
  return g_err_word;
}

}  // namespace hlhgat

using namespace hlhgat;

extern "C" int hlhgat_version(void) { return 101; }

extern "C" int hlhgat_device_errors(unsigned* out) {
  HLH_CHECK_ARG(out, "device_errors: NULL pointer");
  unsigned* w = device_error_word();
  HLH_CHECK_ARG(w, "device_errors: %s", hlhgat_last_error());
  *out = *static_cast<volatile unsigned*>(w);
  return HLHGAT_OK;
}

extern "C" int hlhgat_clear_device_errors(void) {
  unsigned* w = device_error_word();
  HLH_CHECK_ARG(w, "clear_device_errors: %s", hlhgat_last_error());
  *static_cast<volatile unsigned*>(w) = 0u;
  return HLHGAT_OK;
}

extern "C" const char* hlhgat_last_error(void) { return g_last_error.c_str(); }

extern "C" int hlhgat_stream_create(int device, unsigned flags, int priority,
                                    const uint32_t* cu_mask, int cu_mask_words, void** out) {
  HLH_CHECK_ARG(out && device >= 0 && cu_mask_words >= 0 && (cu_mask_words == 0 || cu_mask) &&
                    (cu_mask_words == 0 || priority == 0),
                "stream_create: bad arguments (a CU-masked stream has the default priority)");
  int prev = 0;
  HLH_CHECK_HIP(hipGetDevice(&prev));
  HLH_CHECK_HIP(hipSetDevice(device));
  hipStream_t s = nullptr;
  hipError_t e;
  if (cu_mask_words > 0) {
    int cus = 0;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    int on = 0;
    for (int w = 0; w < cu_mask_words; ++w) on += __builtin_popcount(cu_mask[w]);
    if (e == hipSuccess && (on == 0 || cu_mask_words * 32 < cus)) {
      (void)hipSetDevice(prev);
      HLH_CHECK_ARG(false, "stream_create: the CU mask must cover all %d CUs (%d words given) "
                    "and enable at least one", cus, cu_mask_words);
    }
    if (e == hipSuccess) e = hipExtStreamCreateWithCUMask(&s, (uint32_t)cu_mask_words, cu_mask);
    // (a CU-masked stream is blocking w.r.t. the null stream; the library's
    // streams only ever synchronise through events)
  } else if (priority != 0) {
    e = hipStreamCreateWithPriority(&s, flags, priority);
  } else {
    e = hipStreamCreateWithFlags(&s, flags);
  }
  (void)hipSetDevice(prev);
  HLH_CHECK_HIP(e);
  *out = s;
  return HLHGAT_OK;
}

extern "C" int hlhgat_stream_cu_mask(void* stream, uint32_t* cu_mask, int cu_mask_words) {
  HLH_CHECK_ARG(stream && cu_mask && cu_mask_words > 0, "stream_cu_mask: bad arguments");
  HLH_CHECK_HIP(hipExtStreamGetCUMask(as_stream(stream), (uint32_t)cu_mask_words, cu_mask));
  return HLHGAT_OK;
}

extern "C" int hlhgat_prof_enable(int kernel_class, int enable) {
  HLH_CHECK_ARG(kernel_class >= 0 && kernel_class < HLHGAT_PROF_NCLASS,
                "prof_enable: bad kernel class %d", kernel_class);
  std::lock_guard<std::mutex> lk(g_prof_mu);
  ProfClass& pc = g_prof[kernel_class];
  if (enable && pc.start.empty()) {
    pc.start.resize(kPoolSize);
    pc.stop.resize(kPoolSize);
    pc.bytes.resize(kPoolSize);
    pc.flops.resize(kPoolSize);
    for (int i = 0; i < kPoolSize; ++i) {
      HLH_CHECK_HIP(hipEventCreate(&pc.start[i]));
      HLH_CHECK_HIP(hipEventCreate(&pc.stop[i]));
    }
  }
  pc.enabled = enable != 0;
  return HLHGAT_OK;
}

extern "C" int hlhgat_prof_reset(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& pc : g_prof) {
    pc.used = 0;
    pc.dropped = 0;
  }
  return HLHGAT_OK;
}

extern "C" int hlhgat_prof_read(int kernel_class, int64_t* launches,
                                double* total_ms, double* total_bytes,
                                double* total_flops) {
  HLH_CHECK_ARG(kernel_class >= 0 && kernel_class < HLHGAT_PROF_NCLASS,
                "prof_read: bad kernel class %d", kernel_class);
  std::lock_guard<std::mutex> lk(g_prof_mu);
  ProfClass& pc = g_prof[kernel_class];
  double ms = 0, b = 0, f = 0;
  for (int i = 0; i < pc.used; ++i) {
    HLH_CHECK_HIP(hipEventSynchronize(pc.stop[i]));
    float t = 0.f;
    HLH_CHECK_HIP(hipEventElapsedTime(&t, pc.start[i], pc.stop[i]));
    ms += t;
    b += pc.bytes[i];
    f += pc.flops[i];
  }
  if (launches) *launches = pc.used;
  if (total_ms) *total_ms = ms;
  if (total_bytes) *total_bytes = b;
  if (total_flops) *total_flops = f;
  return HLHGAT_OK;
}

// --- workspace initialisation ------------------------------------------------
namespace {
__global__ void k_zero_words(uint32_t* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0u;
}
}  // namespace

extern "C" int hlhgat_zero_fill(void* p, size_t bytes, void* stream) {
  HLH_CHECK_ARG(bytes % 4 == 0 && (bytes == 0 || p) && (reinterpret_cast<uintptr_t>(p) & 3) == 0,
                "zero_fill: pointer / size must be 4-byte aligned");
  const int64_t n = (int64_t)(bytes / 4);
  if (n == 0) return HLHGAT_OK;
  int64_t g = ceil_div(n, 256);
  if (g > 1024) g = 1024;
  k_zero_words<<<(unsigned)g, 256, 0, as_stream(stream)>>>(static_cast<uint32_t*>(p), n);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// --- batched 2-D strided copies (parameter packing) -------------------------
// Up to HLHGAT_MAX_COPY_BLOCKS rectangles dst[r][c] = src ? src[r][c] : 0 in
// ONE launch: the NodeEdgeInt value path repacks its first-Linear weights and
// biases (and unpacks their gradients) every step; one launch replaces the
// cat / zeros / narrow-copy kernels that would otherwise sit on the critical
// stream.
namespace {
struct CopyArgs {
  int n;
  const float* src[HLHGAT_MAX_COPY_BLOCKS];
  float* dst[HLHGAT_MAX_COPY_BLOCKS];
  int64_t lds[HLHGAT_MAX_COPY_BLOCKS];
  int64_t ldd[HLHGAT_MAX_COPY_BLOCKS];
  int64_t cols[HLHGAT_MAX_COPY_BLOCKS];
  int64_t start[HLHGAT_MAX_COPY_BLOCKS + 1];  // element offsets of the blocks
};

__global__ __launch_bounds__(256) void k_copy2d_batched(CopyArgs a) {
  const int64_t total = a.start[a.n];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = a.n - 1;  // the block holding element e (binary search)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (e >= a.start[mid]) lo = mid; else hi = mid - 1;
    }
    const int b = lo;
    const int64_t loc = e - a.start[b];
    const int64_t r = loc / a.cols[b], c = loc % a.cols[b];
    a.dst[b][r * a.ldd[b] + c] = a.src[b] ? a.src[b][r * a.lds[b] + c] : 0.f;
  }
}
}  // namespace

extern "C" int hlhgat_copy2d_batched(int n, const float* const* src, const int64_t* lds,
                                     float* const* dst, const int64_t* ldd,
                                     const int64_t* rows, const int64_t* cols, void* stream) {
  HLH_CHECK_ARG(n >= 0 && n <= HLHGAT_MAX_COPY_BLOCKS, "copy2d_batched: n=%d", n);
  CopyArgs a{};
  a.n = n;
  a.start[0] = 0;
  for (int b = 0; b < n; ++b) {
    HLH_CHECK_ARG(rows[b] >= 0 && cols[b] >= 0, "copy2d_batched: block %d: negative size", b);
    HLH_CHECK_ARG(rows[b] * cols[b] == 0 || dst[b], "copy2d_batched: block %d: NULL dst", b);
    HLH_CHECK_ARG(!src[b] || lds[b] >= cols[b], "copy2d_batched: block %d: lds < cols", b);
    HLH_CHECK_ARG(rows[b] <= 1 || ldd[b] >= cols[b], "copy2d_batched: block %d: ldd < cols", b);
    a.src[b] = src[b];
    a.dst[b] = dst[b];
    a.lds[b] = lds[b];
    a.ldd[b] = ldd[b];
    a.cols[b] = cols[b] > 0 ? cols[b] : 1;
    a.start[b + 1] = a.start[b] + rows[b] * cols[b];
  }
  const int64_t total = a.start[n];
  if (total == 0) return HLHGAT_OK;
  int64_t g = ceil_div(total, 256);
  if (g > 2048) g = 2048;
  k_copy2d_batched<<<(unsigned)g, 256, 0, as_stream(stream)>>>(a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// --- Adam over one flat parameter buffer -------------------------------------
// hlhgat.train.TrainStep keeps every parameter in one flat fp32 buffer.  On
// that single tensor torch's fused multi-tensor Adam runs one 65536-element
// chunk per workgroup: ~10 workgroups for the 0.66M ZINC parameters, 100 us
// at the end of every step.  Here every thread owns 4 elements, the update is
// torch's fused Adam (ADAM_MODE::ORIGINAL, L2 weight decay added to the
// gradient; bias corrections from the device step count, as its capturable
// path) evaluated with the same double-precision hyper-parameter arithmetic,
// and the step count is incremented by a one-thread launch afterwards (an
// arrival counter of the update's workgroups on one address cost 10-60 us).
namespace {
struct AdamArgs {
  float* p;
  const float* g;
  float* m;
  float* v;
  int64_t n;
  float* step;
  double lr, beta1, beta2, eps, wd;
  int prepared;  // *step already holds this update's count (hlhgat_adam_prepare)
};

__global__ __launch_bounds__(256) void k_adam_flat(AdamArgs a) {
  // bias corrections once per workgroup (fp64 pow), broadcast through LDS
  __shared__ float sh[2];
  if (threadIdx.x == 0) {
    // torch: state_steps += 1 (fp32), then the update
    const float s = a.prepared ? *a.step : *a.step + 1.0f;
    const double bc1 = 1.0 - pow(a.beta1, (double)s);
    const double bc2 = 1.0 - pow(a.beta2, (double)s);
    sh[0] = (float)bc1;
    sh[1] = (float)sqrt(bc2);
  }
  __syncthreads();
  const float bias_correction1 = sh[0];
  const float bias_correction2_sqrt = sh[1];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n;
       i += (int64_t)gridDim.x * 256) {
    float param = a.p[i];
    float grad = a.g[i];
    float exp_avg = a.m[i];
    float exp_avg_sq = a.v[i];
    if (a.wd != 0.0) grad += param * a.wd;
    exp_avg = a.beta1 * exp_avg + (1 - a.beta1) * grad;
    exp_avg_sq = a.beta2 * exp_avg_sq + (1 - a.beta2) * grad * grad;
    const float step_size = a.lr / bias_correction1;
    const float denom = (sqrtf(exp_avg_sq) / bias_correction2_sqrt) + a.eps;
    param -= step_size * exp_avg / denom;
    a.p[i] = param;
    a.m[i] = exp_avg;
    a.v[i] = exp_avg_sq;
  }
}

__global__ void k_adam_step_inc(float* step) { step[0] = step[0] + 1.0f; }

// zero the gradient buffer (float4 stores) and increment the step count
__global__ __launch_bounds__(256) void k_adam_prepare(float* g, int64_t n, float* step) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t == 0) step[0] = step[0] + 1.0f;
  const int64_t n4 = n / 4;
  float4* g4 = reinterpret_cast<float4*>(g);
  for (int64_t i = t; i < n4; i += (int64_t)gridDim.x * 256) g4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = 4 * n4 + t; i < n; i += (int64_t)gridDim.x * 256) g[i] = 0.f;
}
}  // namespace

extern "C" int hlhgat_adam_prepare(float* grad, int64_t n, float* step, void* stream) {
  HLH_CHECK_ARG(n >= 0 && (n == 0 || grad) && step, "adam_prepare: NULL pointer or n < 0");
  HLH_CHECK_ARG(n == 0 || aligned16(grad), "adam_prepare: grad must be 16-byte aligned");
  int64_t g = ceil_div(n / 4 + 1, (int64_t)256);
  if (g > 1024) g = 1024;
  launch(k_adam_prepare, dim3((unsigned)g), dim3(256), 0, as_stream(stream), nullptr, grad, n,
         step);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_adam_flat_prepared(float* param, const float* grad, float* exp_avg,
                                         float* exp_avg_sq, int64_t n, const float* step,
                                         double lr, double beta1, double beta2, double eps,
                                         double weight_decay, void* stream) {
  HLH_CHECK_ARG(n >= 0 && (n == 0 || (param && grad && exp_avg && exp_avg_sq)) && step,
                "adam_flat_prepared: NULL pointer or n < 0");
  if (n == 0) return HLHGAT_OK;
  int64_t g = ceil_div(n, 256 * 2);
  if (g > 2048) g = 2048;
  AdamArgs a{param, grad, exp_avg, exp_avg_sq, n, const_cast<float*>(step), lr, beta1, beta2,
             eps, weight_decay, 1};
  launch(k_adam_flat, dim3((unsigned)g), dim3(256), 0, as_stream(stream), nullptr, a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_adam_flat(float* param, const float* grad, float* exp_avg,
                                float* exp_avg_sq, int64_t n, float* step,
                                double lr, double beta1, double beta2, double eps,
                                double weight_decay, void* stream) {
  HLH_CHECK_ARG(n >= 0 && (n == 0 || (param && grad && exp_avg && exp_avg_sq)) && step,
                "adam_flat: NULL pointer or n < 0");
  if (n == 0) {
    launch(k_adam_step_inc, dim3(1), dim3(1), 0, as_stream(stream), nullptr, step);
    HLH_CHECK_LAUNCH();
    return HLHGAT_OK;
  }
  int64_t g = ceil_div(n, 256 * 2);
  if (g > 2048) g = 2048;
  AdamArgs a{param, grad, exp_avg, exp_avg_sq, n, step, lr, beta1, beta2, eps, weight_decay, 0};
  launch(k_adam_flat, dim3((unsigned)g), dim3(256), 0, as_stream(stream), nullptr, a);
  HLH_CHECK_LAUNCH();
  launch(k_adam_step_inc, dim3(1), dim3(1), 0, as_stream(stream), nullptr, step);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// --- L1 loss (torch.nn.L1Loss, reduction "mean") ------------------------------
// The regression loss of the ZINC training loop: torch runs it as sub / abs /
// mean and the backward as five more elementwise launches, all on the step's
// critical path between the forward and the backward.  Here one launch each:
//   forward  loss = sum |x - y| / n  (one workgroup, fixed summation order);
//   backward dx = (g / n) * sgn(x - y), the arithmetic of torch's MeanBackward
//            (g / n) followed by AbsBackward (grad * sgn): bitwise torch's dx.
namespace {
__global__ __launch_bounds__(256) void k_l1_loss_fwd(const float* __restrict__ x,
                                                     const float* __restrict__ y, int64_t n,
                                                     float* __restrict__ loss) {
  __shared__ float red[256];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += fabsf(x[i] - y[i]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] / (float)n;
}

__global__ __launch_bounds__(256) void k_l1_loss_bwd(const float* __restrict__ x,
                                                     const float* __restrict__ y, int64_t n,
                                                     const float* __restrict__ gout,
                                                     float* __restrict__ dx) {
  const float q = gout[0] / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const float d = x[i] - y[i];
    const float sg = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);  // torch.sgn: 0 for 0 and NaN
    dx[i] = q * sg;
  }
}
}  // namespace

// --- BCE with logits (torch.nn.BCEWithLogitsLoss, no weights) ---------------
// The multi-label loss of the peptides-func loop and the TSP edge loss
// (main_pepfunc...:181-183, main_TSP...:316-321): ATen composes it of
// log_sigmoid / rsub / mul / sub / mean and ~8 backward launches.  One each:
//   forward  loss = (sum_i (1 - t_i) x_i - log_sigmoid(x_i)) / div
//            (div = n for "mean", 1 for "sum"; one workgroup, fixed order);
//   backward dx = gm (1 - t) + (-gm) (m - s z / (1 + z)), gm = g / div,
//            z = exp(-|x|), (m, s) = (1, 1) for x < 0 else (0, -1): the
//            arithmetic of MulBackward + LogSigmoidBackward summed.
__global__ __launch_bounds__(256) void k_bce_logits_fwd(const float* __restrict__ x,
                                                        const float* __restrict__ y, int64_t n,
                                                        float div, float* __restrict__ loss) {
  __shared__ float red[256];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const float v = x[i];
    const float ls = fminf(v, 0.f) - log1pf(expf(-fabsf(v)));  // log_sigmoid
    s += (1.f - y[i]) * v - ls;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] / div;
}

__global__ __launch_bounds__(256) void k_bce_logits_bwd(const float* __restrict__ x,
                                                        const float* __restrict__ y, int64_t n,
                                                        float div,
                                                        const float* __restrict__ gout,
                                                        float* __restrict__ dx) {
  const float gm = gout[0] / div;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const float v = x[i];
    const bool neg = v < 0.f;
    const float m = neg ? 1.f : 0.f, sg = neg ? 1.f : -1.f;
    const float z = expf(-fabsf(v));
    dx[i] = gm * (1.f - y[i]) + (-gm) * (m - sg * (z / (1.f + z)));
  }
}

extern "C" int hlhgat_bce_logits_fwd(const float* x, const float* y, int64_t n, float div,
                                     float* loss, void* stream) {
  HLH_CHECK_ARG(n > 0 && x && y && loss && div > 0.f,
                "bce_logits_fwd: NULL pointer, n <= 0 or div <= 0");
  launch(k_bce_logits_fwd, dim3(1), dim3(256), 0, as_stream(stream), nullptr, x, y, n, div,
         loss);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_bce_logits_bwd(const float* x, const float* y, int64_t n, float div,
                                     const float* gout, float* dx, void* stream) {
  HLH_CHECK_ARG(n > 0 && x && y && gout && dx && div > 0.f,
                "bce_logits_bwd: NULL pointer, n <= 0 or div <= 0");
  int64_t g = ceil_div(n, 256);
  if (g > 1024) g = 1024;
  launch(k_bce_logits_bwd, dim3((unsigned)g), dim3(256), 0, as_stream(stream), nullptr, x, y,
         n, div, gout, dx);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_l1_loss_fwd(const float* x, const float* y, int64_t n, float* loss,
                                  void* stream) {
  HLH_CHECK_ARG(n > 0 && x && y && loss, "l1_loss_fwd: NULL pointer or n <= 0");
  launch(k_l1_loss_fwd, dim3(1), dim3(256), 0, as_stream(stream), nullptr, x, y, n, loss);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_l1_loss_bwd(const float* x, const float* y, int64_t n, const float* gout,
                                  float* dx, void* stream) {
  HLH_CHECK_ARG(n > 0 && x && y && gout && dx, "l1_loss_bwd: NULL pointer or n <= 0");
  int64_t g = ceil_div(n, 256);
  if (g > 1024) g = 1024;
  launch(k_l1_loss_bwd, dim3((unsigned)g), dim3(256), 0, as_stream(stream), nullptr, x, y, n,
         gout, dx);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

// Introspection of a captured graph (tests/test_rccl_capture.py: the RCCL
// kernels inside a captured training step): kernel nodes, and those whose
// kernel name contains name_part.
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

// --- test hook: hold CUs (tests/test_gpu_parity.py::test_bn_one_launch_beside_cu_hog)
// Workgroups [0, hold) each keep their CU's LDS (dynamic, lds_bytes) for
// `usec` microseconds of the 100 MHz constant clock, sleeping; the rest exit
// at once.  Every workgroup exits on its own time bound.
namespace {
__global__ __launch_bounds__(64) void k_occupy(int hold, unsigned usec) {
  extern __shared__ float occ_lds[];
  if ((int)blockIdx.x >= hold) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t lim = (uint64_t)usec * 100u;
  if (threadIdx.x == 0) occ_lds[0] = 0.f;
  while (__builtin_amdgcn_s_memrealtime() - t0 < lim) __builtin_amdgcn_s_sleep(127);
}
}  // namespace

extern "C" int hlhgat_test_occupy(int workgroups, int hold, int lds_bytes, unsigned usec,
                                  void* stream) {
  HLH_CHECK_ARG(workgroups >= 1 && workgroups <= 65536 && hold >= 0 && lds_bytes >= 0 &&
                    lds_bytes <= 160 * 1024 && usec <= 2000000u,
                "test_occupy: bad arguments");
  HLH_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_occupy),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  launch(k_occupy, dim3((unsigned)workgroups), dim3(64), (uint32_t)lds_bytes, as_stream(stream),
         nullptr, hold, usec);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}
