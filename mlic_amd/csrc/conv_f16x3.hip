// Implicit-GEMM convolution on the fp16 MFMA pipe with a 3-term split ("f16x3"), gfx950.
//
// Each fp32 operand is split as  v = hi + lo + r  with hi = fp16(v), lo = fp16(v - hi), and  a.b  is
// computed as  lo_a.hi_b + hi_a.lo_b + hi_a.hi_b  by three fp16 MFMAs with fp32 accumulation (fp16
// products are exact in fp32), at 3/16 of the fp32-MFMA cost per FLOP.  Error of the split:
//  * |r| <= 2^-22 |v| while lo is a normal fp16, i.e. |v| >= 2^-3 (lo ~ 2^-11 v >= 2^-14); below that
//    lo is subnormal and |r| <= 2^-25 absolute.  Weights are therefore prescaled per layer by an exact
//    power of two (split_weights, max|w| -> [2^14, 2^15)) and the scale is undone on the fp32
//    accumulator, so every weight within 2^17 of its layer's largest splits to 2^-22.  Activations are
//    split unscaled: 2^-22 relative for |v| >= 2^-3, 2^-25 absolute below (below fp32's own 2^-24
//    rounding of the dot product once the typical activation is >= 0.5).
//  * |v| >= 65520 overflows fp16 (GDN squares its input: |x| >= 256): the split sites count such
//    values in a device flag (range_flag) and the executor re-runs the call on the exact fp32 MFMA
//    path (Model::guarded).
// Measured on the oracle at 256x384 MLICPP_L: delta-bpp 0, delta-PSNR 0, x_hat 4e-6.
//
// The v1 tile family (conv_f16x3_kernel, `set_precision(1)`) is an A/B baseline and lives in
// ab/conv_f16x3_v1.hip, outside the product library (make AB=1).
// GEMM view as conv_mfma.hip: out[co, p] = sum_k W[co, k] X[k, p], k = (tap, ci); tiles BM x BN x
// BK(=32); LDS images are k-contiguous ([row][k], 80-byte pitch => conflict-free ds_read_b128 for
// the MFMA fragments: lane l reads row l&31, halves 8*(l>>5) .. +7); weights are pre-split and
// padded to [Cout][K*K][Cin_pad32] (hi, lo), activations are split while being staged.
#include "common.h"
#include "kernels.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>

namespace mlic {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int XB_K = 32;         // k per tile
constexpr int XB_PITCH = 40;     // halves per LDS row (32 + 8 pad) = 80 bytes

// $MLIC_V2_WIDE=0 disables the 8-wave 256x256 tile (A/B switch)
static bool v2_wide() {
  static const bool on = [] {
    const char* e = std::getenv("MLIC_V2_WIDE");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

// ---------------------------------------------------------------------------------------------
// v2: B (activations) staged in its natural [k][n] orientation — float4 loads along pixels for
// 1x1 convs, 4-pixel strips otherwise, conflict-free ds_write_b64 of the hi/lo halves — and the
// MFMA B fragments fetched with gfx950's transposing ds_read_b64_tr_b16 (guide T10): per 16-lane
// group it returns a 4(k) x 16(n) block column-major, i.e. 4 consecutive k of one column per lane.
// B rows are padded to BN + 32 halves so the 4 rows of one tr read fall on disjoint 16-bank spans.
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ half8 tr_read8(const _Float16* p0, const _Float16* p1) {
  const short4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)p0);
  const short4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4v*)p1);
  const short8v c = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(half8, c);
}

template <int BM, int BN, int WAVES_M = 2, int WAVES_N = 2>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void conv_x3v2_kernel(ConvParams P, const _Float16* __restrict__ wh,
                                                                            const _Float16* __restrict__ wl, int cin_pad) {
  constexpr int XT = 64 * WAVES_M * WAVES_N;  // threads
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int A_CHUNKS = BM * XB_K / 8 / XT;
  constexpr int QN = BN / 4;                 // pixel quads per k row
  constexpr int RPT = XB_K * QN / XT;  // k rows staged per thread
  static_assert(A_CHUNKS >= 1 && RPT >= 1 && RPT <= 16, "tile");
  constexpr int APITCH = XB_PITCH;           // halves
  constexpr int BPITCH = BN + 32;            // halves
  constexpr int A_SZ = BM * APITCH, B_SZ = XB_K * BPITCH;
  constexpr int BUF = 2 * A_SZ + 2 * B_SZ;
  __shared__ __attribute__((aligned(16))) _Float16 sm[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int nct = gridDim.x, npt = gridDim.y, nblk = nct * npt;
  const int bid = blockIdx.y * nct + blockIdx.x;
  int logical = bid;
  if (nblk >= 16) {
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int ct = logical % nct, pt = logical / nct;
  const int b = blockIdx.z;
  const int co0 = ct * BM, p0 = pt * BN;
  const int HWo = P.Ho * P.Wo;
  const int64_t HWi = (int64_t)P.H * P.W;
  const int KK = P.K * P.K;

  const int pq = tid % QN, kr0 = (tid / QN) * RPT;
  const int n0 = 4 * pq;
  int ohs[4], ows[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p = min(p0 + n0 + q, HWo - 1);
    ohs[q] = p / P.Wo;
    ows[q] = p - ohs[q] * P.Wo;
  }
  const bool fast1x1 = P.K == 1 && P.stride == 1 && P.pad == 0 && (HWo & 3) == 0;
  const bool quad_ok = p0 + n0 + 3 < HWo;

  const int nck = cin_pad / XB_K;
  const int ntile = KK * nck;
  const bool square = (P.epi & EPI_SQUARE_IN) != 0;

  uint4 ra_h[A_CHUNKS], ra_l[A_CHUNKS];
  float rb[RPT][4];
  bool bad = false;

  auto load_tile = [&](int t) {
    const int tap = t / nck;
    const int c0 = (t - tap * nck) * XB_K;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int id = tid + i * XT;
      const int row = id >> 2, qq = id & 3;
      const int co = co0 + row;
      if (co < P.Cout) {
        const int64_t off = ((int64_t)co * KK + tap) * cin_pad + c0 + 8 * qq;
        ra_h[i] = *reinterpret_cast<const uint4*>(wh + off);
        ra_l[i] = *reinterpret_cast<const uint4*>(wl + off);
      } else {
        ra_h[i] = make_uint4(0, 0, 0, 0);
        ra_l[i] = make_uint4(0, 0, 0, 0);
      }
    }
    // rows kr0 .. kr0 + RPT of this tile lie inside one 16-channel group => one segment
    const int cg = c0 + kr0;
    int s = 0, segc0 = 0;
    while (s + 1 < P.nseg && cg >= segc0 + P.seg[s].C) { segc0 += P.seg[s].C; ++s; }
    const Seg sg = P.seg[s];
    const int cl = cg - segc0;
    const float* plane = sg.p + (int64_t)b * sg.bs + (int64_t)cl * HWi;
    if (fast1x1 && quad_ok) {
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const bool ok = (cg + r) < P.Cin && (cl + r) < sg.C;
        float4 v = ok ? *reinterpret_cast<const float4*>(plane + (int64_t)r * HWi + p0 + n0) : make_float4(0.f, 0.f, 0.f, 0.f);
        rb[r][0] = v.x; rb[r][1] = v.y; rb[r][2] = v.z; rb[r][3] = v.w;
      }
    } else {
      const int ky = tap / P.K, kx = tap - ky * P.K;
      int off[4];
      bool inb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int ih = ohs[q] * P.stride + ky - P.pad, iw = ows[q] * P.stride + kx - P.pad;
        inb[q] = (p0 + n0 + q) < HWo && ih >= 0 && ih < P.H && iw >= 0 && iw < P.W;
        off[q] = ih * P.W + iw;
      }
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const bool ok = (cg + r) < P.Cin && (cl + r) < sg.C;
#pragma unroll
        for (int q = 0; q < 4; ++q) rb[r][q] = (ok && inb[q]) ? plane[(int64_t)r * HWi + off[q]] : 0.0f;
      }
    }
    if (square) {
#pragma unroll
      for (int r = 0; r < RPT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) rb[r][q] *= rb[r][q];
    }
  };

  auto store_tile = [&](int buf) {
    _Float16* base = sm + buf * BUF;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int id = tid + i * XT;
      const int row = id >> 2, qq = id & 3;
      *reinterpret_cast<uint4*>(base + row * APITCH + 8 * qq) = ra_h[i];
      *reinterpret_cast<uint4*>(base + A_SZ + row * APITCH + 8 * qq) = ra_l[i];
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      typedef _Float16 half4 __attribute__((ext_vector_type(4)));
      half4 h, l;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bad |= f16_unsafe(rb[r][q]);
        const _Float16 hv = (_Float16)rb[r][q];
        h[q] = hv;
        l[q] = (_Float16)(rb[r][q] - (float)hv);
      }
      *reinterpret_cast<half4*>(base + 2 * A_SZ + (kr0 + r) * BPITCH + n0) = h;
      *reinterpret_cast<half4*>(base + 2 * A_SZ + B_SZ + (kr0 + r) * BPITCH + n0) = l;
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int l32 = lane & 31;
  const int kh = (lane >> 5) * 8;
  // tr-read addressing: 16-lane group g, lane 4q+p supplies row q, columns 4p..4p+3
  const int g = lane >> 4, li = lane & 15;
  const int trow = kh + (li >> 2);
  const int tcol = (g & 1) * 16 + 4 * (li & 3);
  for (int t = 0; t < ntile; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(t + 1);
    const _Float16* base = sm + cur * BUF;
    const _Float16* Bh = base + 2 * A_SZ;
    const _Float16* Bl = base + 2 * A_SZ + B_SZ;
#pragma unroll
    for (int ks = 0; ks < XB_K; ks += 16) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + l32;
        ah[i] = *reinterpret_cast<const half8*>(base + row * APITCH + ks + kh);
        al[i] = *reinterpret_cast<const half8*>(base + A_SZ + row * APITCH + ks + kh);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 32 + tcol;
        const int o0 = (ks + trow) * BPITCH + col;
        bh[j] = tr_read8(Bh + o0, Bh + o0 + 4 * BPITCH);
        bl[j] = tr_read8(Bl + o0, Bl + o0 + 4 * BPITCH);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    if (t + 1 < ntile) store_tile(cur ^ 1);
    __syncthreads();
  }
  range_report(P.rflag, bad);

  const int epi = P.epi;
  const int khalf = lane >> 5;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int p = p0 + wn * WN + j * 32 + l32;
      if (p >= HWo) continue;
      const int oh = p / P.Wo, ow = p - (p / P.Wo) * P.Wo;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        if (co >= P.Cout) continue;
        float v = acc[i][j][r];
        v = ldexpf(v, -P.wexp);
        if (P.bias) v += P.bias[co];
        if (epi & EPI_GELU) v = gelu_erff(v);
        if (epi & (EPI_GDN | EPI_IGDN)) {
          const float x = P.aux[(int64_t)b * P.aux_bs + (int64_t)co * HWo + p];
          v = (epi & EPI_GDN) ? x * (1.0f / sqrtf(v)) : x * sqrtf(v);
        }
        if (epi & EPI_TANH_HALF) v = 0.5f * tanhf(v);
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
    }
  }
}

template <int BM, int BN, int WAVES_M = 2, int WAVES_N = 2>
static void launch_v2(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  const int HWo = P.Ho * P.Wo;
  dim3 grid((P.Cout + BM - 1) / BM, (HWo + BN - 1) / BN, P.B);
  hipLaunchKernelGGL((conv_x3v2_kernel<BM, BN, WAVES_M, WAVES_N>), grid, dim3(64 * WAVES_M * WAVES_N), 0, st, P, wh,
                     wl, cin_pad);
  HIP_OK(hipGetLastError());
}

// 0 <64,128>, 1 <128,256>, 2 <128,128>, 3 <256,256> (8 waves of 64 x 128: twice the MFMAs per
// LDS fragment read of the 64 x 64 wave tiles, which are LDS-bandwidth-bound in split-fp16;
// measured 244 vs 184 TF/s on the g_s subpel conv).  The wide tile is used where its 256-row
// Cout tiles are at least 3/4 occupied (Cout 192..256, 384..512, 576..768, ...).
int conv_x3v2_variant(const ConvParams& P) {
  const int64_t HWo = (int64_t)P.Ho * P.Wo;
  if (P.Cout <= 64) return 0;
  const int ct = (P.Cout + 255) / 256;
  if (v2_wide() && P.Cout >= 192 && 4 * P.Cout >= 3 * 256 * ct && HWo >= 1024) return 3;  // per image (conv_select)
  if (P.Cout <= 192 && HWo >= 128 * 512) return 1;
  return 2;
}

// rows [r0, r0 + n) of a conv as a conv of its own (weights, bias, output, aux and residual shifted)
static ConvParams cout_slice(const ConvParams& P, int r0, int n) {
  ConvParams Q = P;
  const int64_t HWo = (int64_t)P.Ho * P.Wo;
  const int64_t oc = (P.epi & EPI_SHUFFLE) ? (int64_t)(r0 >> 2) * P.out_cs : (int64_t)r0 * P.out_cs;
  Q.Cout = n;
  Q.out = P.out + oc;
  if (P.bias) Q.bias = P.bias + r0;
  if (P.aux) Q.aux = P.aux + (int64_t)r0 * HWo;
  if (P.res) Q.res = P.res + oc;
  return Q;
}

void conv_x3v2_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  MLIC_CHECK(cin_pad % XB_K == 0 && cin_pad >= P.Cin, "f16x3: padded Cin");
  for (int s = 0; s + 1 < P.nseg; ++s) MLIC_CHECK(P.seg[s].C % 16 == 0, "f16x3: segments must be 16-aligned");
  const int v = conv_x3v2_variant(P);
  const int64_t HWo = (int64_t)P.Ho * P.Wo;
  // Cout = 256k + r with r <= 128 (e.g. the entropy-parameters 640 -> 320 layer): the 256-row tiles
  // take 256k rows and a narrow tile the remainder, instead of 128-row tiles for everything
  const int r0 = 256 * (P.Cout / 256), rem = P.Cout - r0;
  if (v == 2 && v2_wide() && r0 > 0 && rem > 0 && rem <= 128 && HWo >= 1024 && (r0 & 3) == 0) {
    const int64_t wofs = (int64_t)r0 * P.K * P.K * cin_pad;
    launch_v2<256, 256, 4, 2>(cout_slice(P, 0, r0), wh, wl, cin_pad, st);
    const ConvParams Q = cout_slice(P, r0, rem);
    if (rem <= 64) launch_v2<64, 128>(Q, wh + wofs, wl + wofs, cin_pad, st);
    else launch_v2<128, 128>(Q, wh + wofs, wl + wofs, cin_pad, st);
    return;
  }
  switch (v) {
    case 0: launch_v2<64, 128>(P, wh, wl, cin_pad, st); break;
    case 1: launch_v2<128, 256>(P, wh, wl, cin_pad, st); break;
    case 3: launch_v2<256, 256, 4, 2>(P, wh, wl, cin_pad, st); break;
    default: launch_v2<128, 128>(P, wh, wl, cin_pad, st); break;
  }
}

// Exact power-of-two prescale of a layer's split weights: the layer is multiplied by 2^e with
// max|w| * 2^e in [2^14, 2^15), so hi = fp16(v) and lo = fp16(v - hi) are both normal for every
// weight within 2^17 of the layer's largest (|r| <= 2^-22 |v|; an unscaled 0.05 weight would leave lo
// subnormal, ~2^-20) and nothing overflows.  The epilogues undo it on the fp32 accumulator with one
// exact ldexp (ConvParams::wexp).  A layer of zeros keeps e = 0.
__global__ void weight_absmax_kernel(const float* __restrict__ w, int64_t n, unsigned* __restrict__ out) {
  __shared__ float red[256];
  float m = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) m = fmaxf(m, fabsf(w[i]));
  red[threadIdx.x] = m;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + k]);
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(red[0]));  // non-negative floats order as uints
}

int weight_prescale_exp(const float* w, int64_t n, hipStream_t st) {
  unsigned* d = nullptr;
  HIP_OK(hipMalloc(&d, sizeof(unsigned)));
  HIP_OK(hipMemsetAsync(d, 0, sizeof(unsigned), st));
  const int nb = (int)std::min<int64_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(weight_absmax_kernel, dim3(std::max(1, nb)), dim3(256), 0, st, w, n, d);
  unsigned u = 0;
  HIP_OK(hipMemcpyAsync(&u, d, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  HIP_OK(hipFree(d));
  float m;
  std::memcpy(&m, &u, sizeof m);
  if (!(m > 0.0f) || !std::isfinite(m)) return 0;
  int ex;
  std::frexp(m, &ex);  // m = f * 2^ex, f in [0.5, 1)  ->  m * 2^(15 - ex) in [2^14, 2^15)
  return std::min(std::max(15 - ex, -60), 60);
}

// weights [Cout][Cin][K][K] fp32 -> hi/lo fp16 [Cout][K*K][cin_pad] (zero padded) of w * 2^wexp
__global__ void split_weights_kernel(const float* __restrict__ w, _Float16* __restrict__ wh, _Float16* __restrict__ wl,
                                     int Cout, int Cin, int KK, int cin_pad, int wexp) {
  const int64_t n = (int64_t)Cout * KK * cin_pad;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int ci = (int)(i % cin_pad);
  const int tap = (int)((i / cin_pad) % KK);
  const int co = (int)(i / ((int64_t)cin_pad * KK));
  const float v = ci < Cin ? ldexpf(w[((int64_t)co * Cin + ci) * KK + tap], wexp) : 0.0f;
  const _Float16 h = (_Float16)v;
  wh[i] = h;
  wl[i] = (_Float16)(v - (float)h);
}

int split_weights(const float* w, _Float16* wh, _Float16* wl, int Cout, int Cin, int KK, int cin_pad, bool prescale,
                  hipStream_t st) {
  const int wexp = prescale ? weight_prescale_exp(w, (int64_t)Cout * Cin * KK, st) : 0;
  const int64_t n = (int64_t)Cout * KK * cin_pad;
  hipLaunchKernelGGL(split_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, wh, wl, Cout, Cin,
                     KK, cin_pad, wexp);
  HIP_OK(hipGetLastError());
  return wexp;
}

}  // namespace mlic
