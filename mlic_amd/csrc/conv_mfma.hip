// Implicit-GEMM convolution on the fp32 MFMA pipe (v_mfma_f32_32x32x2_f32), gfx950.
//
// out[b, co, p] = epi( sum_k A[co, k] * B_b[k, p] + bias[co] )
//   k = tap * Cin + ci  (tap = ky*K + kx),  A = packed weights wpk[tap][ci][co]
//   B_b[k, p] = x_b[ci, oh*s + ky - pad, ow*s + kx - pad]  (zero outside), x = channel concat of
//   up to MAXSEG input segments (no torch.cat is ever materialised).
// Covers every dense conv of the reference: DepthWiseConv's 1x1 half, subpel_conv3x3's 3x3
// (PixelShuffle fused in the store), the 5x5 reprojections, stride-2 1x1 skips, GDN/IGDN
// (conv2d(x**2, gamma, beta) with the x * rsqrt / sqrt in the epilogue), Linear layers and the
// LocalContext 5x5 window fusion (as a 1x1 conv over the 800-row window tensor).
//
// Tile: BM x BN outputs per 256-thread workgroup (2x2 waves, each wave (BM/2)x(BN/2) made of
// 32x32 MFMA sub-tiles), BK = 16 deep, LDS double-buffered, register-staged prefetch of the
// next K tile while the MFMAs run on the current one.  Exact f32 (MFMA f32 = k-ordered fma
// chain), so parity with the CPU reference is limited only by summation order.
#include "common.h"

namespace mlic {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int CONV_BK = 16;
constexpr int CONV_THREADS = 256;

template <int BM, int BN>
__global__ __launch_bounds__(CONV_THREADS) void conv_mfma_kernel(ConvParams P) {
  constexpr int BK = CONV_BK;
  constexpr int WM = BM / 2, WN = BN / 2;   // wave tile
  constexpr int TM = WM / 32, TN = WN / 32; // 32x32 sub-tiles per wave
  constexpr int RA = BK * BM / CONV_THREADS;  // A elements staged per thread
  constexpr int RB = BK * BN / CONV_THREADS;  // B elements staged per thread
  static_assert(TM >= 1 && TN >= 1 && RA >= 1 && RB >= 1, "tile");

  __shared__ float As[2][BK][BM];
  __shared__ float Bs[2][BK][BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware remap (guide T1): blocks b and b+8 share an XCD under round-robin dispatch; give
  // each XCD a contiguous run of logical tiles so the Cout tiles of one pixel tile (which share
  // the B operand) run on one L2.  Bijective for any grid size.  Speed only, never correctness.
  const int nct = gridDim.x;            // Cout tiles (fastest)
  const int npt = gridDim.y;            // pixel tiles
  const int nblk = nct * npt;
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

  // B loader: column nB (pixel), rows rB0 .. rB0 + RB
  const int nB = tid % BN;
  const int rB0 = (tid / BN) * RB;
  const int pB = p0 + nB;
  const bool pvalid = pB < HWo;
  const int ohB = pvalid ? pB / P.Wo : 0;
  const int owB = pvalid ? pB - ohB * P.Wo : 0;
  // A loader: column mA (cout), rows rA0 .. rA0 + RA
  const int mA = tid % BM;
  const int rA0 = (tid / BM) * RA;
  const int coA = co0 + mA;
  const bool covalid = coA < P.Cout;

  const int nck = (P.Cin + BK - 1) / BK;
  const int ntile = P.K * P.K * nck;
  const bool square = (P.epi & EPI_SQUARE_IN) != 0;

  float ra[RA], rb[RB];

  auto load_tile = [&](int t) {
    const int tap = t / nck;
    const int c0 = (t - tap * nck) * BK;
    const int ky = tap / P.K, kx = tap - ky * P.K;
    // A: wpk[(tap*Cin + c)*Cout + co]
    const float* wrow = P.wpk + ((int64_t)tap * P.Cin + c0 + rA0) * P.Cout + coA;
#pragma unroll
    for (int r = 0; r < RA; ++r) {
      const bool ok = covalid && (c0 + rA0 + r) < P.Cin;
      ra[r] = ok ? wrow[(int64_t)r * P.Cout] : 0.0f;
    }
    // B: locate the segment holding channel c0 (segments are 16-aligned, so a tile never straddles)
    int s = 0, segc0 = 0;
    while (s + 1 < P.nseg && c0 >= segc0 + P.seg[s].C) { segc0 += P.seg[s].C; ++s; }
    const Seg sg = P.seg[s];
    const int ih = ohB * P.stride + ky - P.pad;
    const int iw = owB * P.stride + kx - P.pad;
    const bool inb = pvalid && ih >= 0 && ih < P.H && iw >= 0 && iw < P.W;
    const int cl = c0 - segc0 + rB0;  // local channel of row rB0
    const float* src = sg.p + (int64_t)b * sg.bs + (int64_t)cl * HWi + (int64_t)ih * P.W + iw;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const bool ok = inb && (cl + r) < sg.C;
      float v = ok ? src[(int64_t)r * HWi] : 0.0f;
      rb[r] = square ? v * v : v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int r = 0; r < RA; ++r) As[buf][rA0 + r][mA] = ra[r];
#pragma unroll
    for (int r = 0; r < RB; ++r) Bs[buf][rB0 + r][nB] = rb[r];
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
  const int khalf = lane >> 5;
  for (int t = 0; t < ntile; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(t + 1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[cur][kk + khalf][wm * WM + i * 32 + l32];
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = Bs[cur][kk + khalf][wn * WN + j * 32 + l32];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < ntile) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int epi = P.epi;
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

template <int BM, int BN>
static void launch_conv(const ConvParams& P, hipStream_t st) {
  const int HWo = P.Ho * P.Wo;
  dim3 grid((P.Cout + BM - 1) / BM, (HWo + BN - 1) / BN, P.B);
  hipLaunchKernelGGL((conv_mfma_kernel<BM, BN>), grid, dim3(CONV_THREADS), 0, st, P);
  HIP_OK(hipGetLastError());
}

int conv_variant(const ConvParams& P) {
  const int64_t HWo = (int64_t)P.Ho * P.Wo;
  if (P.Cout <= 64) return HWo >= 128 * 256 ? 1 : 0;
  return HWo >= 128 * 512 ? 3 : 2;
}

void conv_forward(const ConvParams& P, hipStream_t st) {
  MLIC_CHECK(P.nseg >= 1 && P.nseg <= MAXSEG, "segment count");
  int tot = 0;
  for (int s = 0; s < P.nseg; ++s) {
    MLIC_CHECK(P.seg[s].p != nullptr, "null input segment");
    if (P.nseg > 1) MLIC_CHECK(P.seg[s].C % CONV_BK == 0 || s == P.nseg - 1, "segments must be 16-channel aligned");
    tot += P.seg[s].C;
  }
  MLIC_CHECK(tot == P.Cin, "segment channels != Cin");
  MLIC_CHECK(P.Ho == (P.H + 2 * P.pad - P.K) / P.stride + 1 && P.Wo == (P.W + 2 * P.pad - P.K) / P.stride + 1,
             "conv output size");
  MLIC_CHECK(!(P.epi & (EPI_GDN | EPI_IGDN)) || P.aux, "GDN needs aux");
  MLIC_CHECK(!(P.epi & EPI_RES) || P.res, "residual pointer");
  MLIC_CHECK(!(P.epi & EPI_SHUFFLE) || P.Cout % 4 == 0, "pixel shuffle needs Cout % 4 == 0");
  switch (conv_variant(P)) {
    case 0: launch_conv<64, 64>(P, st); break;
    case 1: launch_conv<64, 128>(P, st); break;
    case 2: launch_conv<128, 64>(P, st); break;
    default: launch_conv<128, 128>(P, st); break;
  }
}

}  // namespace mlic
