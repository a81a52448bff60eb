// A/B-only kernel family (built with `make AB=1`, not part of the product libmlic_hip.so): the v1
// split-fp16 implicit-GEMM tiles ("f16x3", mlic_set_precision(1)), the round-1 baseline every later
// split-fp16 family (x3v2, x4, pw_resident, dwpw, chain) was measured against.  Arithmetic and
// layout notes: ../conv_f16x3.hip.
#include "../common.h"
#include "../kernels.h"

#include <algorithm>

namespace mlic {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int XB_K = 32;         // k per tile
constexpr int XB_PITCH = 40;     // halves per LDS row (32 + 8 pad) = 80 bytes
constexpr int XB_THREADS = 256;

template <int BM, int BN, int WAVES_M = 2>
__global__ __launch_bounds__(XB_THREADS) void conv_f16x3_kernel(ConvParams P, const _Float16* __restrict__ wh,
                                                                 const _Float16* __restrict__ wl, int cin_pad) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int A_CHUNKS = (BM * XB_K / 8 + XB_THREADS - 1) / XB_THREADS;  // 16-byte chunks per thread
  constexpr int B_ROWS = XB_K * BN / XB_THREADS;         // fp32 values staged per thread
  constexpr int G = B_ROWS < 16 ? B_ROWS : 16;          // channels per segment-uniform group
  static_assert(A_CHUNKS >= 1 && (B_ROWS == 8 || B_ROWS == 16 || B_ROWS == 32), "tile");
  // one LDS array (guide trap 4(a)): [buf][ A_hi | A_lo | B_hi | B_lo ]
  constexpr int A_SZ = BM * XB_PITCH, B_SZ = BN * XB_PITCH;
  constexpr int BUF = 2 * A_SZ + 2 * B_SZ;
  __shared__ __attribute__((aligned(16))) _Float16 sm[2 * BUF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;

  const int nct = gridDim.x, npt = gridDim.y, nblk = nct * npt;
  const int bid = blockIdx.y * nct + blockIdx.x;
  int logical = bid;
  if (nblk >= 16) {  // XCD-aware remap (bijective), as conv_mfma.hip
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int ct = logical % nct, pt = logical / nct;
  const int b = blockIdx.z;
  const int co0 = ct * BM, p0 = pt * BN;
  const int HWo = P.Ho * P.Wo;
  const int64_t HWi = (int64_t)P.H * P.W;
  const int KK = P.K * P.K;

  // B staging: pixel column nB, k rows [kB0, kB0 + B_ROWS)
  const int nB = tid % BN;
  const int kB0 = (tid / BN) * B_ROWS;
  const int pB = p0 + nB;
  const bool pvalid = pB < HWo;
  const int ohB = pvalid ? pB / P.Wo : 0;
  const int owB = pvalid ? pB - ohB * P.Wo : 0;

  const int nck = cin_pad / XB_K;
  const int ntile = KK * nck;
  const bool square = (P.epi & EPI_SQUARE_IN) != 0;

  uint4 ra_h[A_CHUNKS], ra_l[A_CHUNKS];
  float rb[B_ROWS];
  bool bad = false;

  auto load_tile = [&](int t) {
    const int tap = t / nck;
    const int c0 = (t - tap * nck) * XB_K;
    // A: chunk id = tid + i*256 -> row = id / 4, q = id % 4 (8 halves each)
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int id = tid + i * XB_THREADS;
      const int row = id >> 2, q = id & 3;
      const int co = co0 + row;
      if (row < BM && co < P.Cout) {
        const int64_t off = ((int64_t)co * KK + tap) * cin_pad + c0 + 8 * q;
        ra_h[i] = *reinterpret_cast<const uint4*>(wh + off);
        ra_l[i] = *reinterpret_cast<const uint4*>(wl + off);
      } else {
        ra_h[i] = make_uint4(0, 0, 0, 0);
        ra_l[i] = make_uint4(0, 0, 0, 0);
      }
    }
    // B: channels c0 + kB0 .. + B_ROWS at this tap (a 16-channel group never straddles segments)
    const int ky = tap / P.K, kx = tap - ky * P.K;
    const int ih = ohB * P.stride + ky - P.pad;
    const int iw = owB * P.stride + kx - P.pad;
    const bool inb = pvalid && ih >= 0 && ih < P.H && iw >= 0 && iw < P.W;
#pragma unroll
    for (int g = 0; g < B_ROWS; g += G) {
      const int cg = c0 + kB0 + g;
      int s = 0, segc0 = 0;
      while (s + 1 < P.nseg && cg >= segc0 + P.seg[s].C) { segc0 += P.seg[s].C; ++s; }
      const Seg sg = P.seg[s];
      const int cl = cg - segc0;
      const float* src = sg.p + (int64_t)b * sg.bs + (int64_t)cl * HWi + (int64_t)ih * P.W + iw;
#pragma unroll
      for (int r = 0; r < G; ++r) {
        const bool ok = inb && (cg + r) < P.Cin && (cl + r) < sg.C;
        const float v = ok ? src[(int64_t)r * HWi] : 0.0f;
        rb[g + r] = square ? v * v : v;
      }
    }
  };

  auto store_tile = [&](int buf) {
    _Float16* base = sm + buf * BUF;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int id = tid + i * XB_THREADS;
      const int row = id >> 2, q = id & 3;
      if (row >= BM) continue;
      *reinterpret_cast<uint4*>(base + row * XB_PITCH + 8 * q) = ra_h[i];
      *reinterpret_cast<uint4*>(base + A_SZ + row * XB_PITCH + 8 * q) = ra_l[i];
    }
    _Float16* bh = base + 2 * A_SZ + nB * XB_PITCH + kB0;
    _Float16* bl = base + 2 * A_SZ + B_SZ + nB * XB_PITCH + kB0;
#pragma unroll
    for (int g = 0; g < B_ROWS; g += 8) {
      half8 h, l;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = rb[g + j];
        bad |= f16_unsafe(v);
        const _Float16 hv = (_Float16)v;
        h[j] = hv;
        l[j] = (_Float16)(v - (float)hv);
      }
      *reinterpret_cast<half8*>(bh + g) = h;
      *reinterpret_cast<half8*>(bl + g) = l;
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
  for (int t = 0; t < ntile; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(t + 1);
    const _Float16* base = sm + cur * BUF;
#pragma unroll
    for (int ks = 0; ks < XB_K; ks += 16) {
      half8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + l32;
        ah[i] = *reinterpret_cast<const half8*>(base + row * XB_PITCH + ks + kh);
        al[i] = *reinterpret_cast<const half8*>(base + A_SZ + row * XB_PITCH + ks + kh);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 32 + l32;
        bh[j] = *reinterpret_cast<const half8*>(base + 2 * A_SZ + col * XB_PITCH + ks + kh);
        bl[j] = *reinterpret_cast<const half8*>(base + 2 * A_SZ + B_SZ + col * XB_PITCH + ks + kh);
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
  // epilogue (C/D map of the 32x32 MFMAs: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5))
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
        if (epi & EPI_GELU) v = gelu_epi(v);
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

int conv_f16x3_variant(const ConvParams& P) {
  const int64_t HWo = (int64_t)P.Ho * P.Wo;
  if (P.Cout <= 64) return 1;  // <64,128> (the <32,256> 1x4-wave tile measured slower on 192->12)
  return HWo >= 128 * 512 ? 3 : 2;
}

template <int BM, int BN, int WAVES_M = 2>
static void launch_x3(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  const int HWo = P.Ho * P.Wo;
  dim3 grid((P.Cout + BM - 1) / BM, (HWo + BN - 1) / BN, P.B);
  hipLaunchKernelGGL((conv_f16x3_kernel<BM, BN, WAVES_M>), grid, dim3(XB_THREADS), 0, st, P, wh, wl, cin_pad);
  HIP_OK(hipGetLastError());
}

void conv_f16x3_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad,
                        hipStream_t st) {
  MLIC_CHECK(cin_pad % XB_K == 0 && cin_pad >= P.Cin, "f16x3: padded Cin");
  for (int s = 0; s + 1 < P.nseg; ++s) MLIC_CHECK(P.seg[s].C % 16 == 0, "f16x3: segments must be 16-aligned");
  switch (conv_f16x3_variant(P)) {
    case 0: launch_x3<32, 256, 1>(P, wh, wl, cin_pad, st); break;
    case 1: launch_x3<64, 128>(P, wh, wl, cin_pad, st); break;
    case 2: launch_x3<128, 64>(P, wh, wl, cin_pad, st); break;
    default: launch_x3<128, 128>(P, wh, wl, cin_pad, st); break;
  }
}


}  // namespace mlic
