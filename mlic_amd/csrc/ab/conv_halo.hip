// Halo-tiled KxK stride-1 convolution / 1x1 GEMM on the split-fp16 MFMA pipe (gfx950).
//
// The dense 3x3 convs of g_s / h_s (subpel N -> 4N with PixelShuffle, mlicpp synthesis) are the
// largest GEMMs of the step.  As an implicit GEMM with a BK=32 K-step per tap (conv_x3v2) every
// K-step re-reads both operands from L2 — 32 KB per 128x128x32 block step, ~25 TB/s of L2 traffic
// at full MFMA rate, which is where that kernel saturates.  Here a block owns a 128(Cout) x
// TH x 32(pixels) output tile and walks the input in 32-channel chunks:
//   * the chunk's (TH+K-1) x (32+K-1) input patch is staged ONCE in LDS, split into hi/lo fp16 and
//     stored channel-contiguous ([position][channel], 80-byte pitch), so each of the K*K taps
//     reads its B fragments (8 consecutive channels of one shifted position per lane) with
//     ds_read_b128 straight from the shared patch;
//   * the weights are staged per (chunk, tap) as a 128 x 32 hi/lo tile (double-buffered);
//   * the next chunk's patch is loaded while the current chunk's first taps run.
// K = 3, TH = 8 (g_s / h_s 3x3): per 128x256x32 step 16 KB of weights + 1/9 of a 54 KB patch from
// L2 (~3x less than x3v2 per FLOP).  K = 1, TH = 8: the latent-resolution 1x1 GEMMs (entropy
// parameters, LRP, context MLPs) with the same 8-wave 128x256 tile.  K = 5, TH = 4: the inter-slice
// context reprojection.  8 waves, each a 64(Cout) x (TH/4 rows x 32) sub-tile of
// v_mfma_f32_32x32x16_f16 x 3 split terms.  Multi-segment (channel-concat) inputs are read in
// place (segments are 16-channel aligned).  Epilogue = the shared conv_store.
#include "../common.h"
#include "../kernels.h"

#include <cstdlib>

namespace mlic {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

namespace {
constexpr int HT = 512;       // threads (8 waves)
constexpr int TW = 32;        // output tile width
constexpr int CK = 32;        // channels per chunk
constexpr int PITCH = 40;     // halves per LDS row (32 + 8): conflict-free b128 reads

// BM = Cout per block.  BM = 128: 2 x 4 waves of 64 Cout x (TH/4 rows x 32 px), double-buffered
// patch.  (A BM = 256 form — 64 x 128 wave tiles, single patch buffer refilled from registers —
// needs > 256 VGPRs at 2 waves/SIMD and spills; measured 2.7x slower, so only 128 is built.)
template <int K, int TH, int BM>
struct Halo {
  static constexpr int KK = K * K;
  static constexpr int WAVES_M = BM / 64, WAVES_N = 8 / WAVES_M;
  static constexpr int TN = TH / WAVES_N;                    // pixel rows per wave
  static constexpr bool PATCH_DB = BM == 128;
  static constexpr int A_SZ = BM * PITCH, A_BUF = 2 * A_SZ;
  static constexpr int PH = TH + K - 1, PW = TW + K - 1, NPOS = PH * PW;
  static constexpr int B_SZ = NPOS * PITCH, B_BUF = 2 * B_SZ;
  static constexpr int LDS_HALVES = 2 * A_BUF + (PATCH_DB ? 2 : 1) * B_BUF;
  static constexpr int PITEMS = NPOS * (CK / 8);            // staging items: 8 channels at one position
  static constexpr int PARTS = (PITEMS + HT - 1) / HT;       // items per thread per chunk
  static constexpr int PPT = PATCH_DB ? (PARTS + KK - 1) / KK : PARTS;  // parts held per load tap
  static constexpr int ACH = BM * CK / 8 / HT;               // 16-byte weight chunks per thread
  static_assert(LDS_HALVES * 2 <= 160 * 1024, "LDS budget");
  static_assert(TH % WAVES_N == 0 && ACH >= 1, "tile");
  static_assert(PATCH_DB || KK > 1, "single patch buffer needs a later tap to write it");
};
}  // namespace

template <int K, int TH, int BM>
__global__ __launch_bounds__(HT) void conv_halo_kernel(ConvParams P, const _Float16* __restrict__ wh,
                                                       const _Float16* __restrict__ wl, int cin_pad) {
  using G = Halo<K, TH, BM>;
  constexpr int KK = G::KK, PW = G::PW, NPOS = G::NPOS, B_SZ = G::B_SZ, B_BUF = G::B_BUF, TN = G::TN;
  constexpr int A_SZ = G::A_SZ, A_BUF = G::A_BUF, HBM = BM;
  __shared__ __attribute__((aligned(16))) _Float16 sm[G::LDS_HALVES];
  _Float16* As = sm;                  // [2][hi|lo][BM][PITCH]
  _Float16* Bs = sm + 2 * A_BUF;      // [1 or 2][hi|lo][NPOS][PITCH]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / G::WAVES_N, wn = wave % G::WAVES_N;

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
  const int H = P.H, W = P.W, pad = P.pad;
  const int64_t HW = (int64_t)H * W;
  const int nchunk = cin_pad / CK;
  const int nsteps = nchunk * KK;
  const bool square = (P.epi & EPI_SQUARE_IN) != 0;

  // ---- staging helpers
  uint4 ra_h[G::ACH], ra_l[G::ACH];  // 16-byte chunks of the hi and lo weight tile
  auto load_a = [&](int s) {
    const int c = s / KK, tap = s - KK * (s / KK);
#pragma unroll
    for (int u = 0; u < G::ACH; ++u) {
      const int id = tid + u * HT;
      const int row = id >> 2, q = id & 3;
      const int co = co0 + row;
      if (co < P.Cout) {
        const int64_t off = ((int64_t)co * KK + tap) * cin_pad + c * CK + 8 * q;
        ra_h[u] = *reinterpret_cast<const uint4*>(wh + off);
        ra_l[u] = *reinterpret_cast<const uint4*>(wl + off);
      } else {
        ra_h[u] = make_uint4(0, 0, 0, 0);
        ra_l[u] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_a = [&](int buf) {
    _Float16* base = As + buf * A_BUF;
#pragma unroll
    for (int u = 0; u < G::ACH; ++u) {
      const int id = tid + u * HT;
      const int row = id >> 2, q = id & 3;
      *reinterpret_cast<uint4*>(base + row * PITCH + 8 * q) = ra_h[u];
      *reinterpret_cast<uint4*>(base + A_SZ + row * PITCH + 8 * q) = ra_l[u];
    }
  };
  float rp[G::PPT][8];  // 8 channels of one patch position, per part held in registers
  auto load_p = [&](int c, int part, float (&dst)[8]) {
    const int item = part * HT + tid;
    if (item >= G::PITEMS) return;
    const int pos = item % NPOS, g = item / NPOS;  // position fastest: coalesced along patch rows
    const int py = pos / PW, px = pos - py * PW;
    const int iy = oy0 - pad + py, ix = ox0 - pad + px;
    const bool inb = iy >= 0 && iy < H && ix >= 0 && ix < W;
    const int ch0 = c * CK + 8 * g;
    int s = 0, c0 = 0;  // 8-channel groups never straddle a segment (16-aligned segments)
    while (s + 1 < P.nseg && ch0 >= c0 + P.seg[s].C) { c0 += P.seg[s].C; ++s; }
    const Seg sg = P.seg[s];
    const float* src = sg.p + (int64_t)b * sg.bs + (int64_t)(ch0 - c0) * HW + (int64_t)iy * W + ix;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = inb && (ch0 + j) < P.Cin && (ch0 - c0 + j) < sg.C;
      float v = ok ? src[(int64_t)j * HW] : 0.0f;
      dst[j] = square ? v * v : v;
    }
  };
  bool bad = false;  // fp16 range guard (common.h)
  auto store_p = [&](int buf, int part, const float (&v8)[8]) {
    const int item = part * HT + tid;
    if (item >= G::PITEMS) return;
    const int pos = item % NPOS, g = item / NPOS;
    half8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bad |= f16_unsafe(v8[j]);
      const _Float16 hv = (_Float16)v8[j];
      h[j] = hv;
      l[j] = (_Float16)(v8[j] - (float)hv);
    }
    _Float16* base = Bs + buf * B_BUF + pos * PITCH + 8 * g;
    *reinterpret_cast<half8*>(base) = h;
    *reinterpret_cast<half8*>(base + B_SZ) = l;
  };

  floatx16 acc[2][TN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  // ---- prologue: chunk 0's patch and step 0's weights
  for (int part = 0; part < G::PARTS; ++part) {
    load_p(0, part, rp[0]);
    store_p(0, part, rp[0]);
  }
  load_a(0);
  store_a(0);
  __syncthreads();

  const int l32 = lane & 31, kh = (lane >> 5) * 8;
  // chunk loop with the taps unrolled: tap, ky, kx and every staging decision are compile-time,
  // and every barrier is unconditional (a data-dependent barrier made hipcc keep the
  // accumulators in scratch)
  for (int c = 0; c < nchunk; ++c) {
    const bool next_chunk = c + 1 < nchunk;
    const _Float16* Bp = Bs + (G::PATCH_DB ? (c & 1) * B_BUF : 0);
#pragma unroll
    for (int tap = 0; tap < KK; ++tap) {
      const int s = c * KK + tap;
      const int ky = tap / K, kx = tap - K * (tap / K);
      const bool more = s + 1 < nsteps;
      if (more) load_a(s + 1);
      if constexpr (G::PATCH_DB) {
        if (tap * G::PPT < G::PARTS && next_chunk) {
#pragma unroll
          for (int u = 0; u < G::PPT; ++u)
            if (tap * G::PPT + u < G::PARTS) load_p(c + 1, tap * G::PPT + u, rp[u]);
        }
      } else if (tap == 0 && next_chunk) {  // held in registers until the chunk's last tap
#pragma unroll
        for (int u = 0; u < G::PARTS; ++u) load_p(c + 1, u, rp[u]);
      }

      const _Float16* A = As + (s & 1) * A_BUF;
#pragma unroll
      for (int ks = 0; ks < CK; ks += 16) {
        half8 ah[2], al[2], bh[TN], bl[TN];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int row = wm * 64 + i * 32 + l32;
          ah[i] = *reinterpret_cast<const half8*>(A + row * PITCH + ks + kh);
          al[i] = *reinterpret_cast<const half8*>(A + A_SZ + row * PITCH + ks + kh);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int pos = (TN * wn + j + ky) * PW + l32 + kx;
          bh[j] = *reinterpret_cast<const half8*>(Bp + pos * PITCH + ks + kh);
          bl[j] = *reinterpret_cast<const half8*>(Bp + B_SZ + pos * PITCH + ks + kh);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
      // the weight buffer (s+1)&1 was last read in step s-1 and the patch buffer (c+1)&1 in chunk
      // c-1, both before the previous barrier
      if (more) store_a((s + 1) & 1);
      if constexpr (G::PATCH_DB) {
        if (tap * G::PPT < G::PARTS && next_chunk) {
#pragma unroll
          for (int u = 0; u < G::PPT; ++u)
            if (tap * G::PPT + u < G::PARTS) store_p((c + 1) & 1, tap * G::PPT + u, rp[u]);
        }
      } else if (tap == KK - 1) {
        __syncthreads();  // every wave is done with this chunk's patch (uniform: tap is static)
        if (next_chunk) {
#pragma unroll
          for (int u = 0; u < G::PARTS; ++u) store_p(0, u, rp[u]);
        }
      }
      __syncthreads();
    }
  }

  range_report(P.rflag, bad);
  // ---- epilogue (C/D map: col = lane&31 = pixel column, row = Cout)
  const int khalf = lane >> 5;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int oy = oy0 + TN * wn + j, ox = ox0 + l32;
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
  if (!(P.K == 1 || P.K == 3 || P.K == 5) || P.stride != 1 || P.pad != P.K / 2) return false;
  if (P.Ho != P.H || P.Wo != P.W || cin_pad % CK != 0 || cin_pad < P.Cin || P.Cin < 32 || P.Cout < 32) return false;
  for (int s = 0; s + 1 < P.nseg; ++s)
    if (P.seg[s].C % 16 != 0) return false;
  return true;
}

template <int K, int TH, int BM>
static void launch_halo(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  const int ntx = (P.Wo + TW - 1) / TW, nty = (P.Ho + TH - 1) / TH;
  dim3 grid((P.Cout + BM - 1) / BM, ntx * nty, P.B);
  hipLaunchKernelGGL((conv_halo_kernel<K, TH, BM>), grid, dim3(HT), 0, st, P, wh, wl, cin_pad);
  HIP_OK(hipGetLastError());
}

void conv_halo_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  MLIC_CHECK(conv_halo_ok(P, cin_pad), "conv_halo: unsupported shape");
  switch (P.K) {
    case 1: launch_halo<1, 8, 128>(P, wh, wl, cin_pad, st); break;
    case 3: launch_halo<3, 8, 128>(P, wh, wl, cin_pad, st); break;
    default: launch_halo<5, 4, 128>(P, wh, wl, cin_pad, st); break;
  }
}

}  // namespace mlic
