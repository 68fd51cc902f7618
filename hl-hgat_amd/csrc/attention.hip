// Per-simplex attention score of NodeEdgeInt / MSI with only_att=True
// (lib/Hodge_Cheb_Conv.py:297-305 and :103-111):
//
//   a = sigma( ((1-lam) * <Qc, K> + lam * <Qs, K>) / sqrt(dk) )
//
// There is no softmax in the reference: each row is two dot
// products over dk followed by sigma (Sigmoid or ReLU).  One group of LPR
// lanes owns one row; each lane holds V of the dk features; the dot products
// are reduced across the group with wave shuffles (ds_swizzle / DPP), so the
// three projections are read exactly once and nothing goes through LDS.
#include "common.h"

using namespace hlhgat;

namespace {

struct AttArgs {
  int64_t n;
  int dk;
  const float* Qc;
  int64_t ldqc;
  const float* Qs;
  int64_t ldqs;
  const float* K;
  int64_t ldk;
  float c1, c2, sqrt_dk;
  int sigma;
  const float* a_in;  // bwd: forward output
  const float* da;    // bwd: upstream gradient
  float* a_out;       // fwd output
  float* dQc;
  float* dQs;
  float* dK;
  int64_t ldg;
};

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_att_fwd(AttArgs a) {
  using vt = typename VecT<V>::type;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  const bool live = row < a.n;
  float s1 = 0.f, s2 = 0.f;
  if (live) {
    for (int f = sub * V; f < a.dk; f += LPR * V) {
      vt qc = vload<V>(a.Qc + row * a.ldqc + f);
      vt qs = vload<V>(a.Qs + row * a.ldqs + f);
      vt k = vload<V>(a.K + row * a.ldk + f);
#pragma unroll
      for (int c = 0; c < V; ++c) {
        s1 += vget(qc, c) * vget(k, c);
        s2 += vget(qs, c) * vget(k, c);
      }
    }
  }
  // every lane of the wave takes part in the shuffles
  s1 = group_sum<LPR>(s1);
  s2 = group_sum<LPR>(s2);
  if (live && sub == 0) {
    const float z = (a.c1 * s1 + a.c2 * s2) / a.sqrt_dk;
    float out;
    if (a.sigma == HLHGAT_SIGMA_SIGMOID)
      out = 1.f / (1.f + expf(-z));
    else
      out = z > 0.f ? z : 0.f;
    a.a_out[row] = out;
  }
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_att_bwd(AttArgs a) {
  using vt = typename VecT<V>::type;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (row >= a.n) return;
  const float av = a.a_in[row];
  const float g = a.da[row];
  float dz;
  if (a.sigma == HLHGAT_SIGMA_SIGMOID)
    dz = g * (av * (1.f - av));
  else
    dz = av > 0.f ? g : 0.f;
  const float dzs = dz / a.sqrt_dk;
  const float d1 = a.c1 * dzs;
  const float d2 = a.c2 * dzs;
  for (int f = sub * V; f < a.dk; f += LPR * V) {
    vt qc = vload<V>(a.Qc + row * a.ldqc + f);
    vt qs = vload<V>(a.Qs + row * a.ldqs + f);
    vt k = vload<V>(a.K + row * a.ldk + f);
    vt gqc, gqs, gk;
#pragma unroll
    for (int c = 0; c < V; ++c) {
      vget(gqc, c) = d1 * vget(k, c);
      vget(gqs, c) = d2 * vget(k, c);
      vget(gk, c) = d1 * vget(qc, c) + d2 * vget(qs, c);
    }
    vstore<V>(a.dQc + row * a.ldg + f, gqc);
    vstore<V>(a.dQs + row * a.ldg + f, gqs);
    vstore<V>(a.dK + row * a.ldg + f, gk);
  }
}

// Row scaling by the attention score (the NEAtt product x0 * att,
// main_pepfunc_HL_HGCNN_dense_int3_attpool.py:134-136, lib/Hodge_ST_Model.py:
// 276-280): y[r] = x[r] * a[r]; backward dx[r] = dy[r] * a[r] and
// da[r] = <dy[r], x[r]> in ONE pass over dy and x (ATen: a broadcast multiply,
// a full-size product and a row reduction).  One LPR-lane group per row.
struct ScaleArgs {
  int64_t n;
  int d;
  const float* x;
  int64_t ldx;
  const float* a;
  const float* dy;
  int64_t lddy;
  float* y;  // fwd: y; bwd: dx
  int64_t ldy;
  float* da;
};

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_row_scale_fwd(ScaleArgs p) {
  using vt = typename VecT<V>::type;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (row >= p.n) return;
  const float s = p.a[row];
  for (int f = sub * V; f < p.d; f += LPR * V) {
    vt v = vload<V>(p.x + row * p.ldx + f);
#pragma unroll
    for (int c = 0; c < V; ++c) vget(v, c) = vget(v, c) * s;
    vstore<V>(p.y + row * p.ldy + f, v);
  }
}

template <int V, int LPR>
__global__ __launch_bounds__(256) void k_row_scale_bwd(ScaleArgs p) {
  using vt = typename VecT<V>::type;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  const bool live = row < p.n;
  float acc = 0.f;
  if (live) {
    const float s = p.a[row];
    for (int f = sub * V; f < p.d; f += LPR * V) {
      vt g = vload<V>(p.dy + row * p.lddy + f);
      vt x = vload<V>(p.x + row * p.ldx + f);
      vt o;
#pragma unroll
      for (int c = 0; c < V; ++c) {
        vget(o, c) = vget(g, c) * s;
        acc += vget(g, c) * vget(x, c);
      }
      vstore<V>(p.y + row * p.ldy + f, o);
    }
  }
  acc = group_sum<LPR>(acc);  // every lane of the wave takes part
  if (live && sub == 0) p.da[row] = acc;
}

int pick_v_scale(const ScaleArgs& p) {
  for (int v : {4, 2}) {
    bool ok = p.d % v == 0 && p.ldx % v == 0 && p.ldy % v == 0 &&
              ((uintptr_t)p.x % (4 * v)) == 0 && ((uintptr_t)p.y % (4 * v)) == 0;
    if (p.dy) ok = ok && p.lddy % v == 0 && ((uintptr_t)p.dy % (4 * v)) == 0;
    if (ok) return v;
  }
  return 1;
}

int pick_v(const AttArgs& a, bool bwd) {
  for (int v : {4, 2}) {
    bool ok = a.dk % v == 0 && a.ldqc % v == 0 && a.ldqs % v == 0 && a.ldk % v == 0;
    ok = ok && ((uintptr_t)a.Qc % (4 * v)) == 0 && ((uintptr_t)a.Qs % (4 * v)) == 0 &&
         ((uintptr_t)a.K % (4 * v)) == 0;
    if (bwd)
      ok = ok && a.ldg % v == 0 && ((uintptr_t)a.dQc % (4 * v)) == 0 &&
           ((uintptr_t)a.dQs % (4 * v)) == 0 && ((uintptr_t)a.dK % (4 * v)) == 0;
    if (ok) return v;
  }
  return 1;
}

#define HLH_ATT_DISPATCH(KERNEL, V, L, GRID, S, ARGS)                         \
  switch ((V) * 100 + (L)) {                                                \
    case 101: KERNEL<1, 1><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 102: KERNEL<1, 2><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 104: KERNEL<1, 4><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 108: KERNEL<1, 8><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 116: KERNEL<1, 16><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 132: KERNEL<1, 32><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 164: KERNEL<1, 64><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 201: KERNEL<2, 1><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 202: KERNEL<2, 2><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 204: KERNEL<2, 4><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 208: KERNEL<2, 8><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 216: KERNEL<2, 16><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 232: KERNEL<2, 32><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 264: KERNEL<2, 64><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 401: KERNEL<4, 1><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 402: KERNEL<4, 2><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 404: KERNEL<4, 4><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 408: KERNEL<4, 8><<<GRID, 256, 0, S>>>(ARGS); break;               \
    case 416: KERNEL<4, 16><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 432: KERNEL<4, 32><<<GRID, 256, 0, S>>>(ARGS); break;              \
    case 464: KERNEL<4, 64><<<GRID, 256, 0, S>>>(ARGS); break;              \
    default: break;                                                         \
  }

}  // namespace

using namespace hlhgat;

extern "C" int hlhgat_att_score_fwd(int64_t n, int64_t dk, const float* Qc,
                                    int64_t ldqc, const float* Qs, int64_t ldqs,
                                    const float* Kr, int64_t ldk, float w_cross,
                                    float w_self, float sqrt_dk, int sigma,
                                    float* out,
                                    void* stream) {
  HLH_CHECK_ARG(n >= 0 && dk > 0 && ldqc >= dk && ldqs >= dk && ldk >= dk,
                "att_score_fwd: bad sizes");
  HLH_CHECK_ARG(sigma == HLHGAT_SIGMA_SIGMOID || sigma == HLHGAT_SIGMA_RELU,
                "att_score_fwd: bad sigma %d", sigma);
  HLH_CHECK_ARG(sqrt_dk > 0.f, "att_score_fwd: sqrt_dk must be > 0");
  if (n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(Qc && Qs && Kr && out, "att_score_fwd: NULL pointer");
  AttArgs a{};
  a.n = n;
  a.dk = (int)dk;
  a.Qc = Qc;
  a.ldqc = ldqc;
  a.Qs = Qs;
  a.ldqs = ldqs;
  a.K = Kr;
  a.ldk = ldk;
  a.c1 = w_cross;
  a.c2 = w_self;
  a.sqrt_dk = sqrt_dk;
  a.sigma = sigma;
  a.a_out = out;
  const int v = pick_v(a, false);
  int l = next_pow2((int)ceil_div(dk, v));
  if (l > 64) l = 64;
  const unsigned grid = (unsigned)ceil_div(n, 256 / l);
  hipStream_t s = as_stream(stream);
  HLH_ATT_DISPATCH(k_att_fwd, v, l, grid, s, a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_att_score_bwd(int64_t n, int64_t dk, const float* Qc,
                                    int64_t ldqc, const float* Qs, int64_t ldqs,
                                    const float* Kr, int64_t ldk, float w_cross,
                                    float w_self, float sqrt_dk, int sigma,
                                    const float* aout,
                                    const float* da, float* dQc, float* dQs,
                                    float* dK, int64_t ldg, void* stream) {
  HLH_CHECK_ARG(n >= 0 && dk > 0 && ldqc >= dk && ldqs >= dk && ldk >= dk && ldg >= dk,
                "att_score_bwd: bad sizes");
  HLH_CHECK_ARG(sigma == HLHGAT_SIGMA_SIGMOID || sigma == HLHGAT_SIGMA_RELU,
                "att_score_bwd: bad sigma %d", sigma);
  HLH_CHECK_ARG(sqrt_dk > 0.f, "att_score_bwd: sqrt_dk must be > 0");
  if (n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(Qc && Qs && Kr && aout && da && dQc && dQs && dK,
                "att_score_bwd: NULL pointer");
  AttArgs a{};
  a.n = n;
  a.dk = (int)dk;
  a.Qc = Qc;
  a.ldqc = ldqc;
  a.Qs = Qs;
  a.ldqs = ldqs;
  a.K = Kr;
  a.ldk = ldk;
  a.c1 = w_cross;
  a.c2 = w_self;
  a.sqrt_dk = sqrt_dk;
  a.sigma = sigma;
  a.a_in = aout;
  a.da = da;
  a.dQc = dQc;
  a.dQs = dQs;
  a.dK = dK;
  a.ldg = ldg;
  const int v = pick_v(a, true);
  int l = next_pow2((int)ceil_div(dk, v));
  if (l > 64) l = 64;
  const unsigned grid = (unsigned)ceil_div(n, 256 / l);
  hipStream_t s = as_stream(stream);
  HLH_ATT_DISPATCH(k_att_bwd, v, l, grid, s, a);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_row_scale_fwd(int64_t n, int64_t d, const float* x, int64_t ldx,
                                    const float* a, float* y, int64_t ldy, void* stream) {
  HLH_CHECK_ARG(n >= 0 && d > 0 && ldx >= d && ldy >= d, "row_scale_fwd: bad sizes");
  if (n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(x && a && y, "row_scale_fwd: NULL pointer");
  ScaleArgs p{n, (int)d, x, ldx, a, nullptr, 0, y, ldy, nullptr};
  const int v = pick_v_scale(p);
  int l = next_pow2((int)ceil_div(d, v));
  if (l > 64) l = 64;
  const unsigned grid = (unsigned)ceil_div(n, 256 / l);
  HLH_ATT_DISPATCH(k_row_scale_fwd, v, l, grid, as_stream(stream), p);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}

extern "C" int hlhgat_row_scale_bwd(int64_t n, int64_t d, const float* x, int64_t ldx,
                                    const float* a, const float* dy, int64_t lddy, float* dx,
                                    int64_t lddx, float* da, void* stream) {
  HLH_CHECK_ARG(n >= 0 && d > 0 && ldx >= d && lddy >= d && lddx >= d,
                "row_scale_bwd: bad sizes");
  if (n == 0) return HLHGAT_OK;
  HLH_CHECK_ARG(x && a && dy && dx && da, "row_scale_bwd: NULL pointer");
  ScaleArgs p{n, (int)d, x, ldx, a, dy, lddy, dx, lddx, da};
  const int v = pick_v_scale(p);
  int l = next_pow2((int)ceil_div(d, v));
  if (l > 64) l = 64;
  const unsigned grid = (unsigned)ceil_div(n, 256 / l);
  HLH_ATT_DISPATCH(k_row_scale_bwd, v, l, grid, as_stream(stream), p);
  HLH_CHECK_LAUNCH();
  return HLHGAT_OK;
}
