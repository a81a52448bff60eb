// mlic_hip — MI355X-native (gfx950 / CDNA4) MLIC++ encode/decode.
// Shared host/device declarations.
#pragma once
#include <hip/hip_runtime.h>

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
};

// device helpers -----------------------------------------------------------------------------
__device__ __forceinline__ float gelu_erf(float x) {
  // torch.nn.GELU(): 0.5 * x * (1 + erf(x / sqrt(2)))
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

__device__ __forceinline__ bool is_anchor(int h, int w) { return ((h + w) & 1) == 1; }

// the shared conv epilogue: bias, activation/normalisation, masks, residual, (shuffled) store of
// output channel co at conv-grid pixel p of image b (flag order as the Epi enum)
__device__ __forceinline__ void conv_store(const ConvParams& P, int b, int co, int p, float v) {
  const int epi = P.epi;
  const int HWo = P.Ho * P.Wo;
  if (P.bias) v += P.bias[co];
  if (epi & EPI_GELU) v = gelu_erf(v);
  if (epi & (EPI_GDN | EPI_IGDN)) {
    const float x = P.aux[(int64_t)b * P.aux_bs + (int64_t)co * HWo + p];
    v = (epi & EPI_GDN) ? x * (1.0f / sqrtf(v)) : x * sqrtf(v);
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

}  // namespace mlic
