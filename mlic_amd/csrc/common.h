// mlic_hip — MI355X-native (gfx950 / CDNA4) MLIC++ encode/decode.
// Shared host/device declarations.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace mlic {

// ---------------------------------------------------------------------------------------------
// errors: C++ exceptions inside the library, converted to status codes at the C ABI.
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define MLIC_CHECK(cond, msg)                                                                  \
  do {                                                                                          \
    if (!(cond)) throw ::mlic::Error(std::string("mlic: ") + (msg) + " [" #cond "] at " +       \
                                     __FILE__ + ":" + std::to_string(__LINE__));               \
  } while (0)

#define HIP_OK(expr)                                                                            \
  do {                                                                                          \
    hipError_t _e = (expr);                                                                     \
    if (_e != hipSuccess)                                                                       \
      throw ::mlic::Error(std::string("hip: ") + hipGetErrorString(_e) + " in " #expr " at " + \
                          __FILE__ + ":" + std::to_string(__LINE__));                           \
  } while (0)

// ---------------------------------------------------------------------------------------------
// Activation tensors are NCHW fp32, batch-major; a view is (ptr, C, H, W, batch stride), so a
// channel slice of a bigger tensor is a view with the parent's batch stride.
struct View {
  float* p = nullptr;
  int C = 0, H = 0, W = 0;
  int64_t bs = 0;  // batch stride in floats
  int64_t hw() const { return (int64_t)H * W; }
  View ch(int c0, int nc) const {
    View v = *this;
    v.p = p + (int64_t)c0 * hw();
    v.C = nc;
    return v;
  }
};

// epilogue flags of the conv/GEMM kernel (applied in this order after bias)
enum Epi : int {
  EPI_NONE = 0,
  EPI_GELU = 1,        // exact erf GELU
  EPI_GDN = 2,         // v = aux[c,p] * rsqrt(v)    (compressai GDN, aux = GDN input x)
  EPI_IGDN = 4,        // v = aux[c,p] * sqrt(v)     (inverse GDN)
  EPI_TANH_HALF = 8,   // v = 0.5 * tanh(v)          (LRP head)
  EPI_MASK_ANCHOR = 16,     // v = anchor(p)    ? v : 0   (ckbd_anchor of the conv output)
  EPI_MASK_NONANCHOR = 32,  // v = nonanchor(p) ? v : 0
  EPI_RES = 64,        // v = v + res[c,p]          (residual add, last)
  EPI_SHUFFLE = 128,   // store through PixelShuffle(2): out[c/4, 2h+(c%4)/2, 2w+c%2]
  EPI_SQUARE_IN = 256, // B operand is x*x (GDN's conv2d(x**2, gamma, beta))
};

constexpr int MAXSEG = 6;

struct Seg {  // one input segment of a channel concat: channels [c0, c0 + C) of the concat
  const float* p;
  int C;
  int64_t bs;
};

struct ConvParams {
  Seg seg[MAXSEG];
  int nseg;
  int Cin, H, W;          // input
  int Cout, Ho, Wo;       // conv output grid (before pixel shuffle)
  int K, stride, pad;     // square kernel
  const float* wpk;       // packed weights [K*K][Cin][Cout]
  int wexp;               // split-fp16 paths: the hi/lo weights are the layer's weights * 2^wexp (exact)
  const float* bias;      // [Cout] or null
  float* out;
  int64_t out_bs;         // batch stride of out (floats)
  int64_t out_cs;         // channel stride of out (floats) = Ho*Wo, or (2Ho*2Wo) under shuffle
  int epi;
  const float* aux;       // GDN input (same [Cout][Ho*Wo] layout as the conv output)
  int64_t aux_bs;
  const float* res;       // residual, same layout as the stored output
  int64_t res_bs;
  int B;
  int* rflag;             // fp16 range guard of the split-fp16 paths (range_check), or null
};

// device helpers -----------------------------------------------------------------------------
// fp16 range guard: a split-fp16 operand that does not fit fp16 (|v| >= 65520 rounds to inf; NaN
// included) raises the calling lane's device flag (Lane::rflag, range_report).  The conv kernels test
// their split inputs; the chain kernel tests that its outputs are finite (an overflowing split operand
// becomes +-inf, which its GELU turns into NaN and every later layer carries).  Model::range_hit reads
// and clears the flag: an overflow in the entropy model makes forward() re-run whole in exact fp32 and
// compress() / decompress() refuse the input (the decoder must reproduce the encoder's arithmetic); one
// in g_s alone makes forward() and decompress() re-run g_s alone in exact fp32 (Model::gs_fp32_rerun).
// Every fallback is counted (mlic_range_fallbacks).
// softmax exponent on the hardware exp2 (one v_exp_f32 + one multiply instead of expf's ~12-instruction
// range-reduced sequence): e^x = 2^(x log2 e).  Arguments are x - max <= 0; relative error
// <= 1 ulp + |x| 2^-24 ln 2 (1e-7 at |x| = 1, 1e-6 at |x| = 20, where e^x < 3e-9 of the largest term).
// Encoder and decoder run the same kernels, so bit-reproducibility is unaffected.
__device__ __forceinline__ float softmax_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }

// linear attention: the channel softmax of one pixel's query (context.py:181, 236), in registers; shared by attn_apply and
// the fused pack (linatt_pack_kernel), which must produce the same bits
template <int HD>
__device__ __forceinline__ void query_softmax(const float* qp, int HW, float (&q)[HD]) {
  float mx = -3.0e38f;
#pragma unroll
  for (int c = 0; c < HD; ++c) {
    q[c] = qp[(int64_t)c * HW];
    mx = fmaxf(mx, q[c]);
  }
  float sum = 0.0f;
#pragma unroll
  for (int c = 0; c < HD; ++c) {
    q[c] = softmax_exp(q[c] - mx);
    sum += q[c];
  }
  const float inv = 1.0f / sum;
#pragma unroll
  for (int c = 0; c < HD; ++c) q[c] *= inv;
}

__device__ __forceinline__ bool f16_unsafe(float v) { return (__float_as_uint(v) & 0x7fffffffu) >= 0x477ff000u; }
__device__ __forceinline__ void range_report(int* flag, bool bad) {
  if (bad && flag) atomicOr(flag, 1);
}
// torch.nn.GELU() = x Phi(x) = max(x, 0) - |x| erfc(|x| / sqrt 2) / 2, with erfc(z) = t P(t) exp(-z^2),
// t = 1 / (1 + p z) (Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7; the 1/2 folded into P).
// Branch-free: one v_rcp, one v_exp, 10 FMA-class ops, and no cancellation in the negative tail.
// |error| vs the exact GELU <= 4.4 ulp of max(|x|, 2^-10) over [-12, 12] (numpy model of this exact
// op sequence) -- torch's own fp32 0.5 x (1 + erf(x / sqrt 2)) measures 5.1 on the same grid.
__device__ __forceinline__ float gelu_erf(float x) {
  const float ax = __builtin_fabsf(x);
  const float z = ax * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, z, 1.0f));
  float q = __builtin_fmaf(0.5307027101516724f, t, -0.726576030254364f);
  q = __builtin_fmaf(q, t, 0.710706889629364f);
  q = __builtin_fmaf(q, t, -0.14224836230278015f);
  q = __builtin_fmaf(q, t, 0.1274147927761078f);
  q = q * t;
  const float e = __builtin_amdgcn_exp2f(z * (z * -1.44269504088896341f));  // exp(-z^2)
  return __builtin_fmaxf(x, 0.0f) - ax * (q * e);
}
// gelu_erf of two values at once: the same operation sequence element for element (bit-identical),
// with the multiply / FMA steps as packed-fp32 VALU (v_pk_mul_f32 / v_pk_fma_f32: one instruction
// for both) -- for epilogues that hold pixel pairs
typedef float mlic_float2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ mlic_float2 gelu_erf2(mlic_float2 x) {
  const mlic_float2 ax = {__builtin_fabsf(x.x), __builtin_fabsf(x.y)};
  const mlic_float2 z = ax * 0.70710678118654752440f;
  const mlic_float2 d = __builtin_elementwise_fma(mlic_float2{0.3275911f, 0.3275911f}, z, mlic_float2{1.0f, 1.0f});
  const mlic_float2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  mlic_float2 q = __builtin_elementwise_fma(mlic_float2{0.5307027101516724f, 0.5307027101516724f}, t,
                                            mlic_float2{-0.726576030254364f, -0.726576030254364f});
  q = __builtin_elementwise_fma(q, t, mlic_float2{0.710706889629364f, 0.710706889629364f});
  q = __builtin_elementwise_fma(q, t, mlic_float2{-0.14224836230278015f, -0.14224836230278015f});
  q = __builtin_elementwise_fma(q, t, mlic_float2{0.1274147927761078f, 0.1274147927761078f});
  q = q * t;
  const mlic_float2 zz = z * (z * -1.44269504088896341f);
  const mlic_float2 e = {__builtin_amdgcn_exp2f(zz.x), __builtin_amdgcn_exp2f(zz.y)};
  const mlic_float2 m = {__builtin_fmaxf(x.x, 0.0f), __builtin_fmaxf(x.y, 0.0f)};
  return m - ax * (q * e);
}
// torch's own formula 0.5 x (1 + erf(x / sqrt 2)) on the library erff: the x3v2 tiles' epilogue, whose
// fully unrolled element loops the branch-free form pushes into scratch (576 B per lane)
__device__ __forceinline__ float gelu_erff(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }
// every other conv / depthwise epilogue's GELU (x4, pw_resident, dwpw, the exact-fp32 MFMA convs, the
// depthwise kernels): the chain kernel's branch-free gelu_erf (round 4: the g_s subpel convs' GELU
// epilogue 0.7 -> 0.3 ms of 7.7 per 8 images; library erff spends ~25 VALU per value on its branches)
__device__ __forceinline__ float gelu_epi(float x) {
#ifndef MLIC_GELU_EPI_ERFF  // A/B build: -DMLIC_GELU_EPI_ERFF = the library form everywhere
  return gelu_erf(x);
#else
  return gelu_erff(x);
#endif
}

// GDN / IGDN output: x * rsqrt(v) / x * sqrt(v) on the hardware v_rsq / v_sqrt (1 ulp; v >= beta > 0)
__device__ __forceinline__ float gdn_apply(float x, float v, bool inverse) {
  return inverse ? x * __builtin_amdgcn_sqrtf(v) : x * __builtin_amdgcn_rsqf(v);
}

__device__ __forceinline__ bool is_anchor(int h, int w) { return ((h + w) & 1) == 1; }

// the shared conv epilogue: bias, activation/normalisation, masks, residual, (shuffled) store of
// output channel co at conv-grid pixel p of image b (flag order as the Epi enum)
__device__ __forceinline__ void conv_store(const ConvParams& P, int b, int co, int p, float v) {
  const int epi = P.epi;
  const int HWo = P.Ho * P.Wo;
  v = ldexpf(v, -P.wexp);
  if (P.bias) v += P.bias[co];
  if (epi & EPI_GELU) v = gelu_epi(v);
  if (epi & (EPI_GDN | EPI_IGDN)) {
    const float x = P.aux[(int64_t)b * P.aux_bs + (int64_t)co * HWo + p];
    v = gdn_apply(x, v, (epi & EPI_GDN) == 0);
  }
  if (epi & EPI_TANH_HALF) v = 0.5f * tanhf(v);
  int oh = 0, ow = 0;
  if (epi & (EPI_MASK_ANCHOR | EPI_MASK_NONANCHOR | EPI_SHUFFLE)) {
    oh = p / P.Wo;
    ow = p - oh * P.Wo;
  }
  if (epi & EPI_MASK_ANCHOR) v = is_anchor(oh, ow) ? v : 0.0f;
  if (epi & EPI_MASK_NONANCHOR) v = is_anchor(oh, ow) ? 0.0f : v;
  int64_t off;
  if (epi & EPI_SHUFFLE) {
    const int oc = co >> 2;
    const int y2 = 2 * oh + ((co >> 1) & 1), x2 = 2 * ow + (co & 1);
    off = (int64_t)oc * P.out_cs + (int64_t)y2 * (2 * P.Wo) + x2;
  } else {
    off = (int64_t)co * P.out_cs + p;
  }
  if (epi & EPI_RES) v = P.res[(int64_t)b * P.res_bs + off] + v;
  P.out[(int64_t)b * P.out_bs + off] = v;
}

// vectorised forms of conv_store for kernels that stage their output tile (conv_x4): four outputs
// per lane as one 16-byte store.  conv_store4: channel co at pixels p .. p+3 of one row (no pixel
// shuffle).  conv_store_shuf4: under PixelShuffle(2), channels co0 (= 4 oc + 2 dy) and co0 + 1 at
// pixels p, p+1 fill x2 = 2 ow .. 2 ow + 3 of output row 2 oh + dy; v = (co0@p, co0+1@p, co0@p+1,
// co0+1@p+1).  Callers check 16-byte alignment of every operand (conv_vec_ok) and full validity.
__host__ __device__ __forceinline__ bool conv_vec_ok(const ConvParams& P) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(P.out) | reinterpret_cast<uintptr_t>(P.aux) |
                      reinterpret_cast<uintptr_t>(P.res);
  return (a & 15) == 0 && ((P.out_bs | P.out_cs | P.aux_bs | P.res_bs) & 3) == 0 && (P.Wo & 3) == 0;
}

__device__ __forceinline__ void conv_store4(const ConvParams& P, int b, int co, int p, float4 v) {
  const int epi = P.epi;
  float a[4] = {v.x, v.y, v.z, v.w};
  const float bi = P.bias ? P.bias[co] : 0.0f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] = ldexpf(a[e], -P.wexp) + bi;
    if (epi & EPI_GELU) a[e] = gelu_epi(a[e]);
  }
  if (epi & (EPI_GDN | EPI_IGDN)) {
    const float4 x = *reinterpret_cast<const float4*>(P.aux + (int64_t)b * P.aux_bs + (int64_t)co * P.Ho * P.Wo + p);
    const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] = gdn_apply(xs[e], a[e], (epi & EPI_GDN) == 0);
  }
  if (epi & EPI_TANH_HALF) {
#pragma unroll
    for (int e = 0; e < 4; ++e) a[e] = 0.5f * tanhf(a[e]);
  }
  if (epi & (EPI_MASK_ANCHOR | EPI_MASK_NONANCHOR)) {
    const int oh = p / P.Wo, ow = p - oh * P.Wo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool anc = is_anchor(oh, ow + e);
      if ((epi & EPI_MASK_ANCHOR) && !anc) a[e] = 0.0f;
      if ((epi & EPI_MASK_NONANCHOR) && anc) a[e] = 0.0f;
    }
  }
  const int64_t off = (int64_t)co * P.out_cs + p;
  if (epi & EPI_RES) {
    const float4 r = *reinterpret_cast<const float4*>(P.res + (int64_t)b * P.res_bs + off);
    a[0] = r.x + a[0]; a[1] = r.y + a[1]; a[2] = r.z + a[2]; a[3] = r.w + a[3];
  }
  *reinterpret_cast<float4*>(P.out + (int64_t)b * P.out_bs + off) = make_float4(a[0], a[1], a[2], a[3]);
}

// GDN / masks never combine with the pixel shuffle in this model (checked by the caller)
__device__ __forceinline__ void conv_store_shuf4(const ConvParams& P, int b, int co0, int p, float4 v) {
  const int epi = P.epi;
  float a[4] = {v.x, v.y, v.z, v.w};
  const float b0 = P.bias ? P.bias[co0] : 0.0f, b1 = P.bias ? P.bias[co0 + 1] : 0.0f;
  a[0] = ldexpf(a[0], -P.wexp) + b0; a[1] = ldexpf(a[1], -P.wexp) + b1;
  a[2] = ldexpf(a[2], -P.wexp) + b0; a[3] = ldexpf(a[3], -P.wexp) + b1;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (epi & EPI_GELU) a[e] = gelu_epi(a[e]);
    if (epi & EPI_TANH_HALF) a[e] = 0.5f * tanhf(a[e]);
  }
  const int oh = p / P.Wo, ow = p - oh * P.Wo;
  const int64_t off = (int64_t)(co0 >> 2) * P.out_cs + (int64_t)(2 * oh + ((co0 >> 1) & 1)) * (2 * P.Wo) + 2 * ow;
  if (epi & EPI_RES) {
    const float4 r = *reinterpret_cast<const float4*>(P.res + (int64_t)b * P.res_bs + off);
    a[0] = r.x + a[0]; a[1] = r.y + a[1]; a[2] = r.z + a[2]; a[3] = r.w + a[3];
  }
  *reinterpret_cast<float4*>(P.out + (int64_t)b * P.out_bs + off) = make_float4(a[0], a[1], a[2], a[3]);
}

// CU count of the CURRENT device (grid sizing of the persistent-style kernels), cached per device id:
// lane threads of several models may launch on different devices concurrently, so the cache is an
// array of atomics keyed by hipGetDevice(), not one function static (a racing first store writes the
// same value)
inline int device_cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  MLIC_CHECK(dev >= 0 && dev < 64, "device id");
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    HIP_OK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

}  // namespace mlic
