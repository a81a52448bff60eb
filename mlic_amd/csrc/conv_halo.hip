// Halo-tiled 3x3 stride-1 convolution on the split-fp16 MFMA pipe (gfx950).
//
// The dense 3x3 convs of g_s / h_s (subpel N -> 4N with PixelShuffle, mlicpp synthesis) are the
// largest GEMMs of the step.  As an implicit GEMM with a BK=32 K-step per tap (conv_x3v2) every
// K-step re-reads both operands from L2 — 32 KB per 128x128x32 block step, ~25 TB/s of L2 traffic
// at full MFMA rate, which is where that kernel saturates.  Here a block owns a 128(Cout) x
// 8x32(pixels) output tile and walks the input in 32-channel chunks:
//   * the chunk's (8+2) x (32+2) input patch is staged ONCE in LDS, split into hi/lo fp16 and
//     stored channel-contiguous ([position][channel], 80-byte pitch), so each of the 9 taps reads
//     its B fragments (8 consecutive channels of one shifted position per lane) with ds_read_b128
//     straight from the shared patch;
//   * the weights are staged per (chunk, tap) as a 128 x 32 hi/lo tile (double-buffered);
//   * the next chunk's patch is loaded during the current chunk's first taps.
// Per 128x256x32 step: 16 KB of weights + 1/9 of a 54 KB patch from L2 (≈ 3x less than x3v2 per
// FLOP).  8 waves, each a 64(Cout) x 64(pixels) sub-tile: 2 x 2 v_mfma_f32_32x32x16_f16 tiles x
// 3 split terms per 16-deep k-step.  Epilogue = the shared conv_store (bias, GELU, GDN, masks,
// PixelShuffle, residual).
#include "common.h"
#include "kernels.h"

namespace mlic {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

namespace {
constexpr int HT = 512;                    // threads (8 waves)
constexpr int HBM = 128;                   // Cout per block
constexpr int TH = 8, TW = 32;             // output tile (rows x cols) = 256 pixels
constexpr int PH = TH + 2, PW = TW + 2;    // input patch
constexpr int NPOS = PH * PW;              // 340 positions
constexpr int CK = 32;                     // channels per chunk
constexpr int PITCH = 40;                  // halves per LDS row (32 + 8): conflict-free b128 reads
constexpr int A_SZ = HBM * PITCH;          // one hi or lo weight tile
constexpr int B_SZ = NPOS * PITCH;         // one hi or lo patch
constexpr int A_BUF = 2 * A_SZ, B_BUF = 2 * B_SZ;
constexpr int LDS_HALVES = 2 * A_BUF + 2 * B_BUF;
constexpr int PITEMS = NPOS * (CK / 8);    // patch staging items: 8 channels at one position
constexpr int PSTEPS = (PITEMS + HT - 1) / HT;  // taps of a chunk that carry patch loads (3)
static_assert(PSTEPS <= 9, "patch staging must fit in one chunk's taps");
static_assert(LDS_HALVES * 2 <= 160 * 1024, "LDS budget");
}  // namespace

__global__ __launch_bounds__(HT) void conv3x3_halo_kernel(ConvParams P, const _Float16* __restrict__ wh,
                                                          const _Float16* __restrict__ wl, int cin_pad) {
  __shared__ __attribute__((aligned(16))) _Float16 sm[LDS_HALVES];
  _Float16* As = sm;                  // [2][hi|lo][HBM][PITCH]
  _Float16* Bs = sm + 2 * A_BUF;      // [2][hi|lo][NPOS][PITCH]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // 2 x 4 waves: 64 Cout x (2 rows x 32 cols)

  // block -> (Cout tile, spatial tile), XCD-aware bijective remap as conv_x3v2
  const int ntx = (P.Wo + TW - 1) / TW, nty = (P.Ho + TH - 1) / TH;
  const int nct = gridDim.x, npt = ntx * nty, nblk = nct * npt;
  const int bid = blockIdx.y * nct + blockIdx.x;
  int logical = bid;
  if (nblk >= 16) {
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int ct = logical % nct, pt = logical / nct;
  const int co0 = ct * HBM;
  const int oy0 = (pt / ntx) * TH, ox0 = (pt % ntx) * TW;
  const int b = blockIdx.z;
  const int H = P.H, W = P.W;
  const int64_t HW = (int64_t)H * W;
  const float* x = P.seg[0].p + (int64_t)b * P.seg[0].bs;
  const int nchunk = cin_pad / CK;
  const int nsteps = nchunk * 9;

  // ---- staging helpers
  uint4 ra_h, ra_l;  // one 16-byte chunk of the hi and lo weight tile per thread (128 x 32 / 512 / 8 = 1)
  auto load_a = [&](int s) {
    const int c = s / 9, tap = s - 9 * (s / 9);
    const int row = tid >> 2, q = tid & 3;
    const int co = co0 + row;
    if (co < P.Cout) {
      const int64_t off = ((int64_t)co * 9 + tap) * cin_pad + c * CK + 8 * q;
      ra_h = *reinterpret_cast<const uint4*>(wh + off);
      ra_l = *reinterpret_cast<const uint4*>(wl + off);
    } else {
      ra_h = make_uint4(0, 0, 0, 0);
      ra_l = make_uint4(0, 0, 0, 0);
    }
  };
  auto store_a = [&](int buf) {
    const int row = tid >> 2, q = tid & 3;
    _Float16* base = As + buf * A_BUF;
    *reinterpret_cast<uint4*>(base + row * PITCH + 8 * q) = ra_h;
    *reinterpret_cast<uint4*>(base + A_SZ + row * PITCH + 8 * q) = ra_l;
  };
  float rp[8];  // 8 channels of one patch position
  auto load_p = [&](int c, int part) {
    const int item = part * HT + tid;
    if (item >= PITEMS) return;
    const int pos = item % NPOS, g = item / NPOS;  // position fastest: coalesced along patch rows
    const int py = pos / PW, px = pos - py * PW;
    const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
    const bool inb = iy >= 0 && iy < H && ix >= 0 && ix < W;
    const int ch0 = c * CK + 8 * g;
    const float* src = x + (int64_t)ch0 * HW + (int64_t)iy * W + ix;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = inb && (ch0 + j) < P.Cin;
      float v = ok ? src[(int64_t)j * HW] : 0.0f;
      if (P.epi & EPI_SQUARE_IN) v *= v;
      rp[j] = v;
    }
  };
  auto store_p = [&](int buf, int part) {
    const int item = part * HT + tid;
    if (item >= PITEMS) return;
    const int pos = item % NPOS, g = item / NPOS;
    half8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const _Float16 hv = (_Float16)rp[j];
      h[j] = hv;
      l[j] = (_Float16)(rp[j] - (float)hv);
    }
    _Float16* base = Bs + buf * B_BUF + pos * PITCH + 8 * g;
    *reinterpret_cast<half8*>(base) = h;
    *reinterpret_cast<half8*>(base + B_SZ) = l;
  };

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // ---- prologue: chunk 0's patch and step 0's weights
  for (int part = 0; part < PSTEPS; ++part) {
    load_p(0, part);
    store_p(0, part);
  }
  load_a(0);
  store_a(0);
  __syncthreads();

  const int l32 = lane & 31, kh = (lane >> 5) * 8;
  for (int s = 0; s < nsteps; ++s) {
    const int c = s / 9, tap = s - 9 * c;
    const int ky = tap / 3, kx = tap - 3 * ky;
    const bool more = s + 1 < nsteps;
    const bool pstage = (c + 1 < nchunk) && tap < PSTEPS;
    if (more) load_a(s + 1);
    if (pstage) load_p(c + 1, tap);

    const _Float16* A = As + (s & 1) * A_BUF;
    const _Float16* Bp = Bs + (c & 1) * B_BUF;
#pragma unroll
    for (int ks = 0; ks < CK; ks += 16) {
      half8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = wm * 64 + i * 32 + l32;
        ah[i] = *reinterpret_cast<const half8*>(A + row * PITCH + ks + kh);
        al[i] = *reinterpret_cast<const half8*>(A + A_SZ + row * PITCH + ks + kh);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int pos = (2 * wn + j + ky) * PW + l32 + kx;
        bh[j] = *reinterpret_cast<const half8*>(Bp + pos * PITCH + ks + kh);
        bl[j] = *reinterpret_cast<const half8*>(Bp + B_SZ + pos * PITCH + ks + kh);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    // the weight buffer (s+1)&1 was last read in step s-1 and the patch buffer (c+1)&1 in chunk
    // c-1, both before the previous barrier
    if (more) store_a((s + 1) & 1);
    if (pstage) store_p((c + 1) & 1, tap);
    __syncthreads();
  }

  // ---- epilogue (C/D map: col = lane&31 = pixel column, row = Cout)
  const int khalf = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int oy = oy0 + 2 * wn + j, ox = ox0 + l32;
    if (oy >= P.Ho || ox >= P.Wo) continue;
    const int p = oy * P.Wo + ox;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = co0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf;
        if (co < P.Cout) conv_store(P, b, co, p, acc[i][j][r]);
      }
  }
}

bool conv_halo_ok(const ConvParams& P, int cin_pad) {
  return P.K == 3 && P.stride == 1 && P.pad == 1 && P.nseg == 1 && P.Ho == P.H && P.Wo == P.W &&
         cin_pad % CK == 0 && cin_pad >= P.Cin && P.Cin >= 64 && P.Cout >= 64;
}

void conv_halo_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  MLIC_CHECK(conv_halo_ok(P, cin_pad), "conv_halo: unsupported shape");
  const int ntx = (P.Wo + TW - 1) / TW, nty = (P.Ho + TH - 1) / TH;
  dim3 grid((P.Cout + HBM - 1) / HBM, ntx * nty, P.B);
  hipLaunchKernelGGL(conv3x3_halo_kernel, grid, dim3(HT), 0, st, P, wh, wl, cin_pad);
  HIP_OK(hipGetLastError());
}

}  // namespace mlic
