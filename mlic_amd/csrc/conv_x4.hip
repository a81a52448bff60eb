// Split-fp16 implicit-GEMM convolution with both operands staged by LDS-DMA (gfx950), "x4".
//
// Same arithmetic as conv_f16x3.hip (v = hi + lo + r, a.b = lo_a.hi_b + hi_a.lo_b + hi_a.hi_b on the
// fp16 MFMA pipe with fp32 accumulation), re-organised so the K loop is a pure DMA -> LDS -> MFMA
// pipeline with no register staging:
//   * activations are first packed by x4_pack_act_kernel into a zero-bordered, channel-chunked
//     split layout  act[b][chunk][Hp][Wp][64 halves]  (hi of 32 channels | lo of the same 32),
//     Hp = H + 2 pad, Wp = W + 2 pad.  One 128-byte line = one pixel's 32-channel chunk, so the B
//     tile of a (tap, chunk) K-step is 256 whole lines gathered straight into LDS with
//     global_load_lds_dwordx4 (the border is real zeros: no bounds checks in the loop);
//   * weights are packed once into the exact LDS image of each K-step, [ct][step][BM][64 halves];
//   * LDS rows are 128 bytes; 16-byte granule G of row n sits at G ^ ((n >> 1) & 7), applied on the
//     global SOURCE address of the DMA (the LDS destination of a glds is lane-linear) and on the
//     read, which makes every ds_read_b128 fragment read of v_mfma_f32_16x16x32_f16 conflict-free;
//   * a 2-deep A ring and a 3-deep B ring: while step s computes, the weights of step s+1 and the
//     activations of steps s+1 and s+2 are in flight (counted vmcnt, raw s_barrier: a
//     __syncthreads() would drain every DMA); one barrier per step.
// Block tile: BM (Cout) x 256 pixels (8 rows x 32 columns), 8 waves, wave tile 64 x (256 / waves_n).
// K-step = one 32-channel chunk at one tap (chunk-major, tap-minor, so consecutive steps re-read
// the same input lines shifted by a pixel: L2 hits).
#include "common.h"
#include "kernels.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include <vector>

namespace mlic {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

namespace {
constexpr int X4T = 512;               // threads (8 waves)
constexpr int TR = 8, TC = 32;         // pixel tile: 8 rows x 32 columns
constexpr int BN = TR * TC;            // 256 pixels
constexpr int ROWB = 128;              // LDS row: 32 hi + 32 lo halves
constexpr int ROWH = 64;               // halves per row

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* src, void* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// The same DMA as an asm statement: hipcc cannot see that it writes LDS, so it does not wait for it
// before the k-loop's own ds_reads of the other buffers (it would, conservatively, for the builtin).
// Ordering is the caller's: counted vmcnt + barrier before any read of the destination buffer.
__device__ __forceinline__ void glds16_asm(const void* src, const void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)lds));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(l) : "m0");
}

__device__ __forceinline__ half8 lds_frag(const char* base, int row, int granule) {
  return *reinterpret_cast<const half8*>(base + row * ROWB + ((granule ^ swz(row)) << 4));
}
}  // namespace

// RS: register-staged operands (global_load_dwordx4 one step ahead, ds_write_b128 into a 2-slot
// LDS ring) instead of LDS-DMA: a DMA piece costs ~100-185 issue cycles next to the ds_read/MFMA
// stream (MI355X_MICROARCH.md), a dwordx4 load + ds_write_b128 pair a fraction of that.  (Measured:
// A fragments loaded fragment-shaped straight into registers, skipping LDS, ran 2-15 % slower on
// every bench shape -- twice the VMEM instructions for the same bytes.)
// HI: the reduced-precision form (g_s only): rows hold the fp16 value of 64 channels
// (granules 0-3: channels 0-31 of the chunk, 4-7: channels 32-63) and a K-step is 2 MFMAs per
// fragment pair covering 64 channels: fp16 x fp16 products, fp32 accumulation
// DIR (K = 1, split form): no packed copy -- the B rows are built from the fp32 NCHW input segments
// in registers (lane = pixel, 16 channels per thread, split hi / lo with the pack kernel's RNE
// conversions) and written into the same swizzled LDS image; the fp16 range check rides along
// HALO (K = 3, 5, stride 1; register-staged): the B operand of a 32-channel chunk is staged ONCE per
// chunk as the tile's (8 + K - 1) x (32 + K - 1) halo of packed lines (K = 3: 340 lines, 43.5 KB), and
// every tap reads its fragments from that image at the tap's (ky, kx) shift -- instead of 256 lines
// per tap (K^2 x the L2 -> LDS bytes and VMEM instructions for B).  The next chunk's halo is loaded one
// piece per thread per step, spread over the current chunk's taps, into the other halo slot.
// diagnostics builds only (-DMLIC_X4_ABL_RS=mask, never the product): 1 = no staging in the K loop
// (the prologue's LDS images are re-read every step), 2 = no MFMAs (fragment reads kept alive), 4 = no
// per-step barrier -- wrong results, timing decomposition of the register-staged loop
#ifndef MLIC_X4_ABL_RS
#define MLIC_X4_ABL_RS 0
#endif
#ifndef MLIC_X4_SPREAD  // A/B build: 1 = the staging loads/stores spread over the step's pixel groups, one slice
#define MLIC_X4_SPREAD 0  // after each (measured slower: g_s subpel conv 7.79 vs 7.17 ms, main line 99.7 vs
#endif                    // 103.4 img/s, profiles/r06/ab/x4_spread_staging_ab.log)
#ifndef MLIC_X4_STAGGER  // A/B build: 1 = staging point staggered between the two waves of a SIMD (measured
#define MLIC_X4_STAGGER 0  // slower: g_s subpel conv 7.40 vs 7.08-7.13 ms, profiles/r06/ab/x4_stagger_halo_ab.log)
#endif
template <int K, int BM, bool RS, bool HI, bool DIR = false, bool HALO = false>
__global__ __launch_bounds__(X4T) void conv_x4_kernel(ConvParams P, const _Float16* __restrict__ act,
                                                      const _Float16* __restrict__ wx, int nchunk, int H, int W,
                                                      int abl, int nsplit) {
  constexpr int KK = K * K;
  // BM 256 / 128 / 64: 64 Cout rows per wave (4 fragments); BM 192 (Cout 129..192, e.g. the
  // small-decoder model's dense 192 -> 192 convs, which waste a quarter of a 256-row tile): 4 x 2
  // waves of 48 rows (3 fragments) x 128 pixels; BM 96 (Cout 65..96: the context reprojections'
  // 96 outputs): 2 x 4 waves of 48 rows x 64 pixels; BM 224 (Cout 193..224: the LRP's and the
  // context's 224-channel 1x1s): 2 x 4 waves of 112 rows (7 fragments) x 64 pixels
  constexpr int WAVES_M = BM == 192 ? 4 : (BM == 96 || BM == 224) ? 2 : BM / 64, WAVES_N = 8 / WAVES_M;
  constexpr int WN = BN / WAVES_N;        // pixels per wave
  constexpr int TM = BM / (16 * WAVES_M), TN = WN / 16;  // 16x16 fragments per wave
  constexpr int WR = 16 * TM;             // Cout rows per wave
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB;
  constexpr int NAB = RS ? 2 : 3;  // A ring slots
  constexpr int HR = TR + K - 1, HC = TC + K - 1, HLINES = HR * HC;  // HALO: the chunk's halo image
  constexpr int BSLOT = HALO ? HLINES * ROWB : B_BYTES;
  constexpr int B_OFF = NAB * A_BYTES, LDS = NAB * A_BYTES + 2 * BSLOT;
  constexpr int NA = A_BYTES / 1024 / 8;  // 1 KB glds instructions per wave for A
  constexpr int NB = B_BYTES / 1024 / 8;  // ... for B
  static_assert(NA >= 1 && NB == 4 && LDS <= 160 * 1024, "x4 tile");
  static_assert(!HALO || (RS && !DIR && K > 1), "x4 halo: register-staged K x K only");
  __shared__ __attribute__((aligned(1024))) char sm[LDS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int pad = K / 2;  // H, W: the tiling grid (= P.Ho, P.Wo, or H*W folded into rows of 32 for K = 1)
  const int npix = P.Ho * P.Wo;
  // the packed input plane (zero border pad) and the stride: output (oy, ox), tap (ky, kx) reads the
  // packed line (S oy + ky, S ox + kx)
  const int S = K == 1 ? 1 : P.stride;
  const int Hp = (K == 1 ? H : P.H) + 2 * pad, Wp = (K == 1 ? W : P.W) + 2 * pad;
  const int ntx = (W + TC - 1) / TC;
  const int nct = gridDim.x, npt = gridDim.y, nblk = nct * npt;
  const int bid = blockIdx.y * nct + blockIdx.x;
  int logical = bid;
  if (nblk >= 16) {  // XCD-aware bijective remap (the blocks of one XCD take consecutive tiles)
    const int xcd = bid & 7, q = nblk >> 3, r = nblk & 7;
    logical = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  // tile order: Cout tiles fastest.  For GEMMs of many Cout tiles (the hoisted 640 -> 6400
  // EntropyParameters hyper GEMM: 25 tiles of a 16 MB weight image) in groups of XG Cout tiles, the
  // pixel tiles then advancing: the blocks an XCD runs back to back share XG weight slabs (2.6 MB,
  // L2-resident) instead of cycling through the whole weight image per pixel tile
  constexpr int XG = 4;
  int ct, pt;
  if (K == 1 && nct >= 2 * XG) {
    const int band = XG * npt, g = logical / band, first = g * XG, r = logical - g * band;
    const int gs = min(XG, nct - first);
    ct = first + r % gs;
    pt = r / gs;
  } else {
    ct = logical % nct;
    pt = logical / nct;
  }
  const int oy0 = (pt / ntx) * TR, ox0 = (pt % ntx) * TC;
  // split-K (nsplit > 1): blockIdx.z = image + B * split; the block runs steps [s0, s1) and stores
  // its raw partial sums into plane `split` of the partial buffer (P carries that layout, no epilogue)
  const int b = blockIdx.z % P.B, split = blockIdx.z / P.B;
  const int nsteps = nchunk * KK;
  // (HALO: the K ranges start and end on chunk boundaries, so every chunk a block runs is whole)
  const int s0 = HALO ? split * nchunk / nsplit * KK : split * nsteps / nsplit;
  const int s1 = HALO ? (split + 1) * nchunk / nsplit * KK : (split + 1) * nsteps / nsplit;
  if (nsplit > 1) P.out += (int64_t)split * P.B * P.out_bs;

  // per-lane DMA sources.  B: instruction i of this wave moves pixels n = (wave*NB + i)*8 + lane/8,
  // physical granule lane%8 <- logical granule (lane%8) ^ swz(n).  Pixels past the image edge read a
  // clamped (valid) line; their outputs are discarded.
  const int64_t plane = (int64_t)Hp * Wp * ROWH;  // halves per (image, chunk)
  const _Float16* bsrc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = (wave * NB + i) * 8 + (lane >> 3);
    const int oy = min(oy0 + n / TC, H - 1), ox = min(ox0 + n % TC, W - 1);
    const int G = (lane & 7) ^ swz(n);
    bsrc[i] = act + (int64_t)b * nchunk * plane + ((int64_t)oy * S * Wp + ox * S) * ROWH + G * 8;
  }
  const _Float16* asrc = wx + ((int64_t)ct * nsteps * BM) * ROWH + (wave * NA) * 512 + lane * 8;

  // DMA instruction g of one step: g < NB moves the wave's B lines of step sb into B buffer sb & 1,
  // g >= NB its A rows of step sa into A buffer abuf (B before A: the vmcnt accounting relies on it)
  auto glds_one = [&](int g, int sb, int sa, int abuf) {
    if (g < NB) {
      const int cc = sb / KK, tap = sb - cc * KK;
      const int ky = tap / K, kx = tap - ky * K;
      const int64_t d = cc * plane + ((int64_t)ky * Wp + kx) * ROWH;
      glds16_asm(bsrc[g] + d, sm + B_OFF + (sb & 1) * B_BYTES + (wave * NB + g) * 1024);
    } else {
      const int i = g - NB;
      glds16_asm(asrc + (int64_t)sa * BM * ROWH + i * 512, sm + abuf * A_BYTES + (wave * NA + i) * 1024);
    }
  };
  constexpr int NG = NA + NB;

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int G = lane >> 4, l16 = lane & 15;
  if constexpr (RS) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    // A pieces (1 KB = 8 rows of the step's image) dealt round-robin over the 8 waves: piece
    // wave + 8 i (BM 96 has 12: waves 0-3 take two)
    constexpr int NPA = A_BYTES / 1024, NAR = (NPA + 7) / 8;
    constexpr bool SPREAD = MLIC_X4_SPREAD && !DIR && !HALO && !HI;
    const _Float16* asrc_rs = wx + ((int64_t)ct * nsteps * BM) * ROWH + wave * 512 + lane * 8;
    u32x4 rb[(DIR || HALO) ? 1 : NB], ra[NAR];
    // HALO: pieces (16 bytes = one granule of one halo line) per thread per chunk; piece q of thread
    // tid is q * X4T + tid: line (q * X4T + tid) >> 3, logical granule & 7
    constexpr int NPH = (HLINES * 8 + X4T - 1) / X4T;
    static_assert(!HALO || NPH + 1 <= KK, "x4 halo: the next chunk's pieces must land within the chunk");
    u32x4 hb;
    const _Float16* himg = act + (int64_t)b * nchunk * plane;
    auto hsrc = [&](int q) __attribute__((always_inline)) {  // packed line of halo piece q (clamped)
      const int id = q * X4T + tid, line = min(id >> 3, HLINES - 1);
      const int hr = line / HC, hc = line - hr * HC;
      const int y = min(oy0 + hr, Hp - 1), x = min(ox0 + hc, Wp - 1);
      return ((int64_t)y * Wp + x) * ROWH + (id & 7) * 8;
    };
    auto hdst = [&](int q, int slot) __attribute__((always_inline)) {
      const int id = q * X4T + tid, line = id >> 3;
      return sm + B_OFF + slot * BSLOT + line * ROWB + (((id & 7) ^ swz(line)) << 4);
    };
    auto hvalid = [&](int q) __attribute__((always_inline)) { return q * X4T + tid < HLINES * 8; };
    // DIR: tile pixel dn = 64 (wave & 3) + lane (flat pixel dp, clamped into the image: the ragged
    // tail's outputs are discarded), channels dch .. dch + 15 of the step's 32-channel chunk
    float rv[DIR ? 16 : 1];
    const int dn = (wave & 3) * 64 + lane, dch = (wave >> 2) * 16;
    const int dp = min(oy0 * TC + dn, npix - 1);
    uint32_t dmax = 0;  // max |bits| of every input value this thread split (the fp16 range check)
    auto gload = [&](int st) __attribute__((always_inline)) {  // step st's pieces of this wave -> registers
      const int cc = st / KK, tap = st - cc * KK;
      const int ky = tap / K, kx = tap - ky * K;
      if constexpr (DIR) {
        // 16-aligned 16-channel groups never straddle a segment (conv_x4_ok)
        const int ch0 = cc * 32 + dch;
        // (compile-time segment indices: a runtime index into P would copy it to scratch)
        const float* sp = P.seg[0].p;
        int64_t sbs = P.seg[0].bs;
        int c0 = 0, cend = 0;
#pragma unroll
        for (int k = 1; k < MAXSEG; ++k) {
          cend += P.seg[k - 1].C;
          // (opaque copies: a select between two loads of P would become a load from a selected
          // address into P, which also sends P to scratch)
          uint64_t pk = (uint64_t)P.seg[k].p, bk = (uint64_t)P.seg[k].bs;
          asm("" : "+s"(pk), "+s"(bk));
          if (k < P.nseg && ch0 >= cend) {
            sp = (const float*)pk;
            sbs = (int64_t)bk;
            c0 = cend;
          }
        }
        typedef const __attribute__((address_space(1))) float gfloat;
        gfloat* src = (gfloat*)(sp + (int64_t)b * sbs + (int64_t)(ch0 - c0) * npix) + dp;
        const int nval = P.Cin - ch0;
        if (nval >= 16) {
#pragma unroll
          for (int j = 0; j < 16; ++j) rv[j] = src[(int64_t)j * npix];
        } else {
#pragma unroll
          for (int j = 0; j < 16; ++j) rv[j] = j < nval ? src[(int64_t)j * npix] : 0.0f;
        }
      } else if constexpr (!HALO) {
        const int64_t d = cc * plane + ((int64_t)ky * Wp + kx) * ROWH;
#pragma unroll
        for (int i = 0; i < NB; ++i) rb[i] = *reinterpret_cast<const u32x4*>(bsrc[i] + d);
      }
#pragma unroll
      for (int i = 0; i < NAR; ++i)
        if (NPA % 8 == 0 || wave + 8 * i < NPA)
          ra[i] = *reinterpret_cast<const u32x4*>(asrc_rs + (int64_t)st * BM * ROWH + i * 8 * 512);
    };
    auto lstore = [&](int st) __attribute__((always_inline)) {  // registers -> the LDS slot of step st (the DMA's lane-linear image)
      if constexpr (DIR) {
        typedef float float2v __attribute__((ext_vector_type(2)));
        typedef _Float16 half2v __attribute__((ext_vector_type(2)));
        char* row = sm + B_OFF + (st & 1) * B_BYTES + dn * ROWB;
        const int sw = swz(dn), g0 = dch / 8;  // logical granules g0, g0 + 1 (hi), g0 + 4, g0 + 5 (lo)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          half8 h, l;
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            const float2v v = {rv[8 * q + j], rv[8 * q + j + 1]};
            const half2v hv = __builtin_convertvector(v, half2v);
            const half2v lv = __builtin_convertvector(v - __builtin_convertvector(hv, float2v), half2v);
            h[j] = hv[0];
            h[j + 1] = hv[1];
            l[j] = lv[0];
            l[j + 1] = lv[1];
            dmax = max(dmax, max(__float_as_uint(v[0]) & 0x7fffffffu, __float_as_uint(v[1]) & 0x7fffffffu));
          }
          *reinterpret_cast<half8*>(row + (((g0 + q) ^ sw) << 4)) = h;
          *reinterpret_cast<half8*>(row + (((g0 + q + 4) ^ sw) << 4)) = l;
        }
      } else if constexpr (!HALO) {
#pragma unroll
        for (int i = 0; i < NB; ++i)
          *reinterpret_cast<u32x4*>(sm + B_OFF + (st & 1) * B_BYTES + (wave * NB + i) * 1024 + lane * 16) = rb[i];
      }
#pragma unroll
      for (int i = 0; i < NAR; ++i)
        if (NPA % 8 == 0 || wave + 8 * i < NPA)
          *reinterpret_cast<u32x4*>(sm + (st & 1) * A_BYTES + (wave + 8 * i) * 1024 + lane * 16) = ra[i];
    };
    // SPREAD (plain register-staged form): the step's staging cut into its pieces (NB B pieces + NAR A
    // pieces of 1 KB per wave), piece p stored and re-loaded after pixel group p * TN / NPC -- instead of
    // all of them after group 0, where the 8 waves' 64 loads of a step met in the CU's address unit at
    // one point (at 64 B/clk, ~1 k cycles during which every wave's in-order issue, MFMAs included,
    // waited behind its loads: timing decomposition, profiles/r06/ab/x4_ablation.log)
    constexpr int NPC = NB + NAR;
    auto gload_piece = [&](int st, int p) __attribute__((always_inline)) {
      if (p < NB) {
        const int cc = st / KK, tap = st - cc * KK;
        const int ky = tap / K, kx = tap - ky * K;
        const int64_t d = cc * plane + ((int64_t)ky * Wp + kx) * ROWH;
        rb[p] = *reinterpret_cast<const u32x4*>(bsrc[p] + d);
      } else {
        const int i = p - NB;
        if (NPA % 8 == 0 || wave + 8 * i < NPA)
          ra[i] = *reinterpret_cast<const u32x4*>(asrc_rs + (int64_t)st * BM * ROWH + i * 8 * 512);
      }
    };
    auto lstore_piece = [&](int st, int p) __attribute__((always_inline)) {
      if (p < NB) {
        *reinterpret_cast<u32x4*>(sm + B_OFF + (st & 1) * B_BYTES + (wave * NB + p) * 1024 + lane * 16) = rb[p];
      } else {
        const int i = p - NB;
        if (NPA % 8 == 0 || wave + 8 * i < NPA)
          *reinterpret_cast<u32x4*>(sm + (st & 1) * A_BYTES + (wave + 8 * i) * 1024 + lane * 16) = ra[i];
      }
    };
    // step s's MFMAs on LDS slot s & 1 (fragment reads one pixel group ahead)
    // hook: the step's staging work (next slot's LDS stores, the loads two steps ahead), issued after
    // the first pixel group's MFMAs, so that the step opens with its fragment reads and the LDS
    // latency they expose overlaps the staging's register waits instead of following them
    auto mfma_step = [&](int s, auto jh_c, auto&& hook) {
      constexpr int JH = decltype(jh_c)::value;  // the pixel group after whose MFMAs the staging runs
      const char* As = sm + (s & 1) * A_BYTES;
      const char* Bs;
      int tapoff = 0;  // HALO: the tap's (ky, kx) shift in the halo image, in lines
      if constexpr (HALO) {
        const int cc = s / KK, tap = s - cc * KK, ky = tap / K;
        Bs = sm + B_OFF + (cc & 1) * BSLOT;
        tapoff = ky * HC + (tap - ky * K);
      } else {
        Bs = sm + B_OFF + (s & 1) * B_BYTES;
      }
      // B row of tile pixel n: the pixel's own line, or its halo line at the tap's shift
      auto brow = [&](int n) __attribute__((always_inline)) {
        return HALO ? (n / TC) * HC + (n % TC) + tapoff : n;
      };
      half8 ah[TM], al[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WR + i * 16 + l16;
        ah[i] = lds_frag(As, row, G);
        al[i] = lds_frag(As, row, G + 4);
      }
      half8 bh[2], bl[2];
      bh[0] = lds_frag(Bs, brow(wn * WN + l16), G);
      bl[0] = lds_frag(Bs, brow(wn * WN + l16), G + 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (j + 1 < TN) {
          const int n = brow(wn * WN + (j + 1) * 16 + l16);
          bh[(j + 1) & 1] = lds_frag(Bs, n, G);
          bl[(j + 1) & 1] = lds_frag(Bs, n, G + 4);
        }
        if constexpr ((MLIC_X4_ABL_RS & 2) != 0) {
          asm volatile("" :: "v"(bh[j & 1]), "v"(bl[j & 1]));
          if (j == 0)
#pragma unroll
            for (int i = 0; i < TM; ++i) asm volatile("" :: "v"(ah[i]), "v"(al[i]));
        } else if constexpr (HI) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j & 1], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bl[j & 1], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j & 1], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j & 1], acc[i][j], 0, 0, 0);
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j & 1], acc[i][j], 0, 0, 0);
        }
        if constexpr (SPREAD) {
          // this group's pieces (a compile-time range: j is unrolled)
          if ((j + 1) * NPC / TN > j * NPC / TN) {
            __builtin_amdgcn_sched_barrier(0);
            hook(j);
            __builtin_amdgcn_sched_barrier(0);
          }
        } else if (j == JH) {
          __builtin_amdgcn_sched_barrier(0);
          hook(j);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    };
    if (HALO && s0 < s1) {  // the first chunk's halo image, whole
      const int c0 = s0 / KK;
#pragma unroll
      for (int q = 0; q < NPH; ++q)
        if (hvalid(q)) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(himg + c0 * plane + hsrc(q));
          *reinterpret_cast<u32x4*>(hdst(q, c0 & 1)) = v;
        }
    }
    if (s0 < s1) {
      gload(s0);
      lstore(s0);
    }
    if (s0 + 1 < s1) gload(s0 + 1);
    // the K loop with the staging after pixel group JH.  STAGGER: the two waves of each SIMD (waves w and
    // w + 4 of the workgroup share one) stage at different points of the step -- w < 4 after group 0,
    // w >= 4 after group TN / 2 -- so that while one wave writes its LDS slot and waits for its loads, the
    // other keeps the SIMD's matrix pipe busy (both at the same point left the pipe idle through the
    // staging of both: timing decomposition, profiles/r06/ab/x4_ablation.log)
    auto kloop = [&](auto jh_c) __attribute__((always_inline)) {
    for (int s = s0; s < s1; ++s) {
      // this wave's stores of step s done; barrier: every wave's too, and step s-1's reads of the
      // other slot are finished
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr ((MLIC_X4_ABL_RS & 4) == 0) __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      auto staging = [&](int j) __attribute__((always_inline)) {
        if constexpr ((MLIC_X4_ABL_RS & 1) != 0) return;
        if constexpr (SPREAD) {
#pragma unroll
          for (int p = 0; p < NPC; ++p)
            if (p >= j * NPC / TN && p < (j + 1) * NPC / TN) {
              if (s + 1 < s1) lstore_piece(s + 1, p);
              if (s + 2 < s1) gload_piece(s + 2, p);
            }
          return;
        }
        if (s + 1 < s1) lstore(s + 1);
        if constexpr (HALO) {
          // the next chunk's halo: piece j - 1 stored and piece j loaded at local step j (the slot
          // (cc + 1) & 1 was last read in chunk cc - 1, before this chunk's first barrier; its last
          // piece lands at step NPH <= KK - 1, before chunk cc + 1's first barrier)
          const int cc = s / KK, j = s - cc * KK;
          if ((cc + 1) * KK < s1) {
            if (j >= 1 && j <= NPH && hvalid(j - 1)) *reinterpret_cast<u32x4*>(hdst(j - 1, (cc + 1) & 1)) = hb;
            if (j < NPH && hvalid(j)) hb = *reinterpret_cast<const u32x4*>(himg + (cc + 1) * plane + hsrc(j));
          }
        }
        if (s + 2 < s1) gload(s + 2);
      };
#ifdef MLIC_X4_STAGING_FIRST  // A/B build: the round-3 order (staging, then the step's reads and MFMAs)
      staging(0);
      mfma_step(s, jh_c, [](int) {});
#else
      mfma_step(s, jh_c, staging);
#endif
    }
    };
    // (K x K convs only: the 1 x 1 direct form's two loop copies spill at the register cap)
    if constexpr (MLIC_X4_STAGGER && K > 1) {
      if (__builtin_amdgcn_readfirstlane(wave) & 4) kloop(std::integral_constant<int, TN / 2>{});
      else kloop(std::integral_constant<int, 0>{});
    } else {
      kloop(std::integral_constant<int, 0>{});
    }
    if constexpr (DIR) range_report(P.rflag, f16_unsafe(__uint_as_float(dmax)));
  } else {
  static_assert(!HI, "the reduced-precision form runs on the register-staged path");
  // issue order: A0 B0 A1 | step 0: B1 A2 | step 1: B2 A3 | ...  Every step issues its NG DMA
  // instructions (past the end they re-fetch the last step into buffers no longer read), spread over
  // its pixel groups so the matrix pipe keeps running while the TA works through them.  At the top of
  // step s the newest NA requests are A(s+1); everything older (B(s), A(s)) must have landed.
#pragma unroll
  for (int g = NB; g < NG; ++g) glds_one(g, 0, 0, 0);
#pragma unroll
  for (int g = 0; g < NB; ++g) glds_one(g, 0, 0, 0);
#pragma unroll
  for (int g = NB; g < NG; ++g) glds_one(g, 0, min(1, nsteps - 1), 1);
  int acur = 0;  // s % 3
  for (int s = 0; s < ((abl & 8) ? 0 : nsteps); ++s) {
    static_assert(NA == 1 || NA == 2 || NA == 4, "vmcnt immediate");
    if constexpr (NA == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (NA == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    __builtin_amdgcn_s_barrier();     // every wave's DMA of step s has landed; step s-1's reads are done
    asm volatile("" ::: "memory");    // no LDS read moves above the barrier
    const int sb = min(s + 1, nsteps - 1), sa = min(s + 2, nsteps - 1);
    const int anext = acur == 0 ? 2 : acur - 1;  // (s + 2) % 3
    const char* As = sm + acur * A_BYTES;
    const char* Bs = sm + B_OFF + (s & 1) * B_BYTES;
    acur = acur == 2 ? 0 : acur + 1;
    half8 ah[TM], al[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WR + i * 16 + l16;
      ah[i] = lds_frag(As, row, G);
      al[i] = lds_frag(As, row, G + 4);
    }
    // B fragments one pixel group ahead: the reads of group j+1 are in flight while group j's 12
    // MFMAs issue (both waves of a SIMD reach these waits together, so an exposed LDS latency
    // idles the matrix pipe)
    half8 bh[2], bl[2];
    bh[0] = lds_frag(Bs, wn * WN + l16, G);
    bl[0] = lds_frag(Bs, wn * WN + l16, G + 4);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (!(abl & 1)) {
#pragma unroll
        for (int g = j * NG / TN; g < (j + 1) * NG / TN; ++g) glds_one(g, sb, sa, anext);
      }
      __builtin_amdgcn_sched_barrier(0);  // one DMA slice per pixel group, between its MFMA groups
      if (j + 1 < TN) {
        const int n = wn * WN + (j + 1) * 16 + l16;
        bh[(j + 1) & 1] = lds_frag(Bs, n, G);
        bl[(j + 1) & 1] = lds_frag(Bs, n, G + 4);
      }
      if (abl & 2) {
        asm volatile("" :: "v"(bh[j & 1]), "v"(bl[j & 1]));
        continue;
      }
      // term-major: consecutive MFMAs never chain on one accumulator
#pragma unroll
      for (int i = 0; i < TM; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh[j & 1], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl[j & 1], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh[j & 1], acc[i][j], 0, 0, 0);
    }

  }
  }  // RS

  // epilogue through a wave-private LDS strip (the stage buffers are free once every wave is past
  // its last read): C/D map of 16x16x32 is (row 4*(lane>>4) + e, col lane&15) with row = Cout and
  // col = pixel; per 16-row group the wave transposes to rows of WN pixels and stores each Cout row
  // as 128-byte runs.  Every acc index stays compile-time (a runtime-indexed acc goes to scratch).
  constexpr int EP = WN + 4;  // row pitch (floats): the 4 row groups of a write land on distinct banks
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (abl & 4) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" :: "v"(acc[i][j]));
    return;
  }
  float* ep = reinterpret_cast<float*>(sm) + wave * 16 * EP;
  const int co_w = ct * BM + wm * WR;
  const bool shuf = (P.epi & EPI_SHUFFLE) != 0;
  const bool vec = conv_vec_ok(P) && !(shuf && (P.epi & (EPI_GDN | EPI_IGDN | EPI_MASK_ANCHOR | EPI_MASK_NONANCHOR)));
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) ep[(4 * G + e) * EP + j * 16 + l16] = acc[i][j][e];
    // 16 rows x WN pixels -> 16-byte stores: 4 pixels of one Cout row, or under the pixel shuffle
    // 2 pixels x the 2 channels that interleave along one output row
#pragma unroll 1
    for (int k = 0; k < WN / 16; ++k) {
      const int idx = k * 64 + lane;
      int r0, n;
      float4 v;
      if (!shuf) {
        r0 = idx / (WN / 4);
        n = 4 * (idx % (WN / 4));
        v = *reinterpret_cast<const float4*>(ep + r0 * EP + n);
      } else {
        const int combo = idx / (WN / 2);  // (oc, dy) within the 16 rows
        r0 = 4 * (combo >> 1) + 2 * (combo & 1);
        n = 2 * (idx % (WN / 2));
        const float2 c0 = *reinterpret_cast<const float2*>(ep + r0 * EP + n);
        const float2 c1 = *reinterpret_cast<const float2*>(ep + (r0 + 1) * EP + n);
        v = make_float4(c0.x, c1.x, c0.y, c1.y);
      }
      const int nn = wn * WN + n;
      const int oy = oy0 + nn / TC, ox = ox0 + nn % TC;
      const int co = co_w + i * 16 + r0;
      const int p = oy * W + ox;
      if (oy >= H || ox >= W || p >= npix) continue;
      if (!shuf) {
        if (vec && co < P.Cout && ox + 3 < W && p + 3 < npix) {
          conv_store4(P, b, co, p, v);
        } else if (co < P.Cout) {
          const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (ox + e < W && p + e < npix) conv_store(P, b, co, p + e, vs[e]);
        }
      } else {
        if (vec && co + 1 < P.Cout && ox + 1 < W) {
          conv_store_shuf4(P, b, co, p, v);
        } else {
          if (co < P.Cout) conv_store(P, b, co, p, v.x);
          if (co + 1 < P.Cout) conv_store(P, b, co + 1, p, v.y);
          if (ox + 1 < W) {
            if (co < P.Cout) conv_store(P, b, co, p + 1, v.z);
            if (co + 1 < P.Cout) conv_store(P, b, co + 1, p + 1, v.w);
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// activation packing: NCHW fp32 (multi-segment concat) -> act[b][chunk][Hp][Wp][hi 32 | lo 32]
struct X4Pack {
  Seg seg[MAXSEG];
  int nseg, Cin, H, W, pad, nchunk, square, npix;  // npix: real pixels (K = 1 folds H*W into rows of 32)
  int hi;  // reduced-precision layout: [hi of channels 0-31 | hi of channels 32-63] per 64-channel chunk
  _Float16* dst;
  int* rflag;
};

// grid (ceil(Hp*Wp / 64), nchunk, B), 256 threads: lane = position (64 consecutive), wave = 8-channel group
__global__ __launch_bounds__(256) void x4_pack_act_kernel(X4Pack Q) {
  const int Hp = Q.H + 2 * Q.pad, Wp = Q.W + 2 * Q.pad;
  const int pos = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int cc = blockIdx.y, b = blockIdx.z;
  const int y = pos / Wp - Q.pad, x = pos % Wp - Q.pad;
  const bool inb = pos < Hp * Wp && y >= 0 && y < Q.H && x >= 0 && x < Q.W && y * Q.W + x < Q.npix;
  const int64_t HW = Q.npix;  // channel plane stride of the (unfolded) input
  bool bad = false;
  // 8 consecutive channels from ch0 (8-channel groups never straddle a segment: segments are
  // 16-aligned); out-of-range channels and border positions are zeros
  auto load8 = [&](int ch0, float (&v)[8]) {
    int s = 0, c0 = 0;
    while (s + 1 < Q.nseg && ch0 >= c0 + Q.seg[s].C) { c0 += Q.seg[s].C; ++s; }
    const Seg sg = Q.seg[s];
    const float* src = sg.p + (int64_t)b * sg.bs + (int64_t)(ch0 - c0) * HW + (int64_t)y * Q.W + x;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = inb && ch0 + j < Q.Cin && ch0 - c0 + j < sg.C;
      v[j] = ok ? src[(int64_t)j * HW] : 0.0f;
      if (Q.square) v[j] *= v[j];
      bad |= f16_unsafe(v[j]);
    }
  };
  half8 h, l;
  float v[8];
  if (Q.hi) {
    load8(cc * 64 + 8 * g, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (_Float16)v[j];
    load8(cc * 64 + 32 + 8 * g, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) l[j] = (_Float16)v[j];
  } else {
    load8(cc * 32 + 8 * g, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const _Float16 hv = (_Float16)v[j];
      h[j] = hv;
      l[j] = (_Float16)(v[j] - (float)hv);
    }
  }
  // the block's 64 lines are 8 KB contiguous in the destination: assemble them in LDS (rows padded
  // to 144 B: conflict-free 16-byte writes) and store them lane-consecutively, whole lines per
  // instruction (a direct store would scatter 16-byte pieces over 64 lines per instruction)
  constexpr int SP = ROWH + 8;
  __shared__ __attribute__((aligned(16))) _Float16 stg[64 * SP];
  const int lane = threadIdx.x & 63;
  *reinterpret_cast<half8*>(stg + lane * SP + 8 * g) = h;
  *reinterpret_cast<half8*>(stg + lane * SP + 32 + 8 * g) = l;
  __syncthreads();
  const int nlines = min(64, Hp * Wp - (int)blockIdx.x * 64);
  _Float16* d = Q.dst + (((int64_t)b * Q.nchunk + cc) * Hp * Wp + (int64_t)blockIdx.x * 64) * ROWH;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = k * 256 + threadIdx.x;  // 16-byte piece: line q / 8, granule q % 8
    if (q / 8 < nlines)
      *reinterpret_cast<half8*>(d + q * 8) = *reinterpret_cast<const half8*>(stg + (q / 8) * SP + (q % 8) * 8);
  }
  range_report(Q.rflag, bad);
}

// ---------------------------------------------------------------------------------------------
// the linear attention's output (context.py:181-187, 236-239: att = ctx^T . softmax_c(q) per pixel)
// computed straight into the packed split layout of the reprojection conv that consumes it: one pass
// over Q instead of attn_apply's fp32 att write + x4_pack_act's read.  Same op sequence as attn_apply
// (query_softmax, then one fma chain over c per output channel) and the pack's split, so the packed
// halves equal x4_pack_act(attn_apply(...)) bit for bit.  grid (ceil(Hp*Wp / 64), nchunk, B), 256
// threads: lane = position, wave g = channels 8g .. 8g + 7 of the chunk (one head for hd = 32; the
// chunk's two heads for hd = 16).  qmask: queries at non-anchor positions only (anchors output 0).
struct LinAttPack {
  const float* Q;
  int64_t q_bs;
  const float* ctx;  // [B][heads][hd][hd]
  int heads, H, W, pad, nchunk, qmask;
  _Float16* dst;
  int* rflag;
};

template <int HD>
__global__ __launch_bounds__(256) void linatt_pack_kernel(LinAttPack A) {
  constexpr int HPC = 32 / HD;  // heads per 32-channel chunk
  __shared__ __attribute__((aligned(16))) float cs[HPC * HD * HD];
  const int Hp = A.H + 2 * A.pad, Wp = A.W + 2 * A.pad, HW = A.H * A.W;
  const int cc = blockIdx.y, b = blockIdx.z;
  const float* cb = A.ctx + ((int64_t)b * A.heads + cc * HPC) * HD * HD;
  for (int i = threadIdx.x; i < HPC * HD * HD; i += 256) cs[i] = cb[i];
  __syncthreads();
  const int pos = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int y = pos / Wp - A.pad, x = pos % Wp - A.pad;
  const bool inb = pos < Hp * Wp && y >= 0 && y < A.H && x >= 0 && x < A.W;
  const int hl = (8 * g) / HD, d0 = (8 * g) % HD;  // head within the chunk, first output channel
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = 0.0f;
  if (inb && !(A.qmask && is_anchor(y, x))) {
    float q[HD];
    query_softmax<HD>(A.Q + (int64_t)b * A.q_bs + (int64_t)(cc * HPC + hl) * HD * HW + (int64_t)y * A.W + x, HW, q);
    const float* w = cs + hl * HD * HD + d0;
#pragma unroll
    for (int c = 0; c < HD; ++c) {
      const float4 w0 = *reinterpret_cast<const float4*>(w + c * HD), w1 = *reinterpret_cast<const float4*>(w + c * HD + 4);
      a[0] = fmaf(w0.x, q[c], a[0]);
      a[1] = fmaf(w0.y, q[c], a[1]);
      a[2] = fmaf(w0.z, q[c], a[2]);
      a[3] = fmaf(w0.w, q[c], a[3]);
      a[4] = fmaf(w1.x, q[c], a[4]);
      a[5] = fmaf(w1.y, q[c], a[5]);
      a[6] = fmaf(w1.z, q[c], a[6]);
      a[7] = fmaf(w1.w, q[c], a[7]);
    }
  }
  bool bad = false;
  half8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 hv = (_Float16)a[j];
    h[j] = hv;
    l[j] = (_Float16)(a[j] - (float)hv);
    bad |= f16_unsafe(a[j]);
  }
  // x4_pack_act_kernel's store: the block's 64 lines assembled in LDS, whole lines per instruction
  constexpr int SP = ROWH + 8;
  __shared__ __attribute__((aligned(16))) _Float16 stg[64 * SP];
  const int lane = threadIdx.x & 63;
  *reinterpret_cast<half8*>(stg + lane * SP + 8 * g) = h;
  *reinterpret_cast<half8*>(stg + lane * SP + 32 + 8 * g) = l;
  __syncthreads();
  const int nlines = min(64, Hp * Wp - (int)blockIdx.x * 64);
  _Float16* d = A.dst + (((int64_t)b * A.nchunk + cc) * Hp * Wp + (int64_t)blockIdx.x * 64) * ROWH;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = k * 256 + threadIdx.x;
    if (q / 8 < nlines)
      *reinterpret_cast<half8*>(d + q * 8) = *reinterpret_cast<const half8*>(stg + (q / 8) * SP + (q % 8) * 8);
  }
  range_report(A.rflag, bad);
}

void linatt_pack(const float* Q, int64_t q_bs, const float* ctx, int heads, int hd, int qmask, const ConvParams& P,
                 _Float16* dst, hipStream_t st) {
  MLIC_CHECK((hd == 16 || hd == 32) && P.Cin == heads * hd && P.Cin % 32 == 0 && P.K > 1 && P.stride == 1,
             "linatt_pack: shape");
  LinAttPack A{};
  A.Q = Q;
  A.q_bs = q_bs;
  A.ctx = ctx;
  A.heads = heads;
  A.H = P.H;
  A.W = P.W;
  A.pad = P.K / 2;
  A.nchunk = P.Cin / 32;
  A.qmask = qmask;
  A.dst = dst;
  A.rflag = P.rflag;
  const int npos = (A.H + 2 * A.pad) * (A.W + 2 * A.pad);
  const dim3 grid((npos + 63) / 64, A.nchunk, P.B);
  if (hd == 16) hipLaunchKernelGGL(linatt_pack_kernel<16>, grid, dim3(256), 0, st, A);
  else hipLaunchKernelGGL(linatt_pack_kernel<32>, grid, dim3(256), 0, st, A);
  HIP_OK(hipGetLastError());
}

// weights: hi/lo [Cout][KK][cin_pad] -> [ct][step = chunk*KK + tap][BM rows][64 halves], swizzled;
// hi: the reduced-precision image, chunks of 64 channels of hi only (channels >= cin_pad are zeros)
__global__ void x4_pack_weights_kernel(const _Float16* __restrict__ wh, const _Float16* __restrict__ wl,
                                       _Float16* __restrict__ dst, int Cout, int KK, int cin_pad, int BM,
                                       int64_t n, int hi) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = (int)(i % ROWH);           // physical half within the row
  const int row = (int)((i / ROWH) % BM);
  const int64_t ts = i / ((int64_t)ROWH * BM);  // ct * nsteps + step
  const int nchunk = hi ? (cin_pad + 63) / 64 : cin_pad / 32, nsteps = nchunk * KK;
  const int step = (int)(ts % nsteps), ct = (int)(ts / nsteps);
  const int cc = step / KK, tap = step - cc * KK;
  const int Gp = e >> 3, G = Gp ^ ((row >> 1) & 7);  // logical granule stored at physical Gp
  const int k = (G & 3) * 8 + (e & 7);               // channel within the 32-channel half
  const int co = ct * BM + row;
  _Float16 v = (_Float16)0.0f;
  if (co < Cout) {
    const int ch = hi ? cc * 64 + (G >> 2) * 32 + k : cc * 32 + k;
    const int64_t off = ((int64_t)co * KK + tap) * cin_pad + ch;
    if (hi) v = ch < cin_pad ? wh[off] : (_Float16)0.0f;
    else v = G < 4 ? wh[off] : wl[off];
  }
  dst[i] = v;
}

// ---------------------------------------------------------------------------------------------
// 256-row Cout tiles unless 128-row tiles pad at least 1/8 of Cout less (e.g. 320, 640 -> 128)
int x4_bm(int Cout) {
  // A/B: $MLIC_X4_BM_FOR="Cout:BM,Cout:BM" forces the tile height of the listed Cout values
  static const std::vector<std::pair<int, int>> force = [] {
    std::vector<std::pair<int, int>> v;
    const char* e = std::getenv("MLIC_X4_BM_FOR");
    for (const char* q = e; q && *q;) {
      int c = 0, m = 0, n = 0;
      if (std::sscanf(q, "%d:%d%n", &c, &m, &n) != 2) break;
      if (m == 64 || m == 96 || m == 128 || m == 192 || m == 224 || m == 256) v.emplace_back(c, m);
      q += n;
      if (*q == ',') ++q;
    }
    return v;
  }();
  for (const auto& f : force)
    if (f.first == Cout) return f.second;
  if (Cout <= 64) return 64;
  // MLICPP_L's h_s 320 -> 1280 subpel conv runs at 1/64 of the image (17 x 30 at 1080p: 24 pixel tiles
  // per 8 images): 256-row tiles leave half the CUs idle (120 workgroups), 128-row tiles fill them --
  // 252 -> 157 us (8 x 17 x 30, profiles/r06/ab/x4_tile_height_ab.log); 480 -> 1920 (1/32) is equal either way
  if (Cout == 1280) return 128;
  static const bool t96 = [] {  // A/B: MLIC_X4_BM96=0 keeps 128-row tiles for Cout 65..96
    const char* e = std::getenv("MLIC_X4_BM96");
    return !(e && e[0] == '0');
  }();
  if (t96 && Cout > 64 && Cout <= 96) return 96;
  if (Cout > 128 && Cout <= 192) return 192;
  static const bool t224 = [] {  // A/B: MLIC_X4_BM224=0 keeps 256-row tiles for Cout 193..224
    const char* e = std::getenv("MLIC_X4_BM224");
    return !(e && e[0] == '0');
  }();
  if (t224 && Cout > 192 && Cout <= 224) return 224;
  const int w256 = (Cout + 255) / 256 * 256 - Cout, w128 = (Cout + 127) / 128 * 128 - Cout;
  return (Cout >= 192 && 8 * (w256 - w128) <= Cout) ? 256 : 128;
}

int x4_nchunk(int cin_pad, bool hi) { return hi ? (cin_pad + 63) / 64 : cin_pad / 32; }

int64_t x4_weight_halves(int Cout, int KK, int cin_pad, bool hi) {
  const int bm = x4_bm(Cout);
  return (int64_t)((Cout + bm - 1) / bm) * bm * KK * x4_nchunk(cin_pad, hi) * ROWH;
}

void x4_pack_weights(const _Float16* wh, const _Float16* wl, int Cout, int KK, int cin_pad, _Float16* dst,
                     hipStream_t st, bool hi) {
  const int64_t n = x4_weight_halves(Cout, KK, cin_pad, hi);
  hipLaunchKernelGGL(x4_pack_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wh, wl, dst, Cout,
                     KK, cin_pad, x4_bm(Cout), n, hi ? 1 : 0);
  HIP_OK(hipGetLastError());
}
// K = 1: no spatial coupling, so the flat pixel index is folded into rows of TC = 32: every
// 8 x 32 tile is 256 consecutive pixels and only the image's last tile is ragged
static void x4_grid(const ConvParams& P, int& H, int& W) {  // the packed input's grid
  H = P.K == 1 ? (P.H * P.W + TC - 1) / TC : P.H;
  W = P.K == 1 ? TC : P.W;
}
static void x4_tgrid(const ConvParams& P, int& H, int& W) {  // the output tiling grid
  H = P.K == 1 ? (P.H * P.W + TC - 1) / TC : P.Ho;
  W = P.K == 1 ? TC : P.Wo;
}

int64_t x4_act_halves(const ConvParams& P, int cin_pad, bool hi) {
  const int pad = P.K / 2;
  int H, W;
  x4_grid(P, H, W);
  return (int64_t)P.B * x4_nchunk(cin_pad, hi) * (H + 2 * pad) * (W + 2 * pad) * ROWH;
}

bool conv_x4_ok(const ConvParams& P, int cin_pad) {
  // stride 1 (K = 1, 3, 5), or stride 2 for K = 3 (the small-decoder model's dense strided convs)
  if (!(P.K == 1 || P.K == 3 || P.K == 5) || P.pad != P.K / 2) return false;
  if (!(P.stride == 1 || (P.stride == 2 && P.K == 3))) return false;
  if (P.Ho != (P.H - 1) / P.stride + 1 || P.Wo != (P.W - 1) / P.stride + 1) return false;
  if (cin_pad % 32 != 0 || cin_pad < P.Cin || P.Cout < 32) return false;
  for (int s = 0; s + 1 < P.nseg; ++s)
    if (P.seg[s].C % 16 != 0) return false;
  return true;
}

void x4_pack_act(const ConvParams& P, int cin_pad, _Float16* dst, hipStream_t st, bool hi) {
  X4Pack Q{};
  for (int s = 0; s < P.nseg; ++s) Q.seg[s] = P.seg[s];
  Q.nseg = P.nseg;
  Q.Cin = P.Cin;
  x4_grid(P, Q.H, Q.W);
  Q.npix = P.H * P.W;
  Q.pad = P.K / 2;
  Q.nchunk = x4_nchunk(cin_pad, hi);
  Q.hi = hi ? 1 : 0;
  Q.square = (P.epi & EPI_SQUARE_IN) ? 1 : 0;
  Q.dst = dst;
  Q.rflag = P.rflag;
  const int npos = (Q.H + 2 * Q.pad) * (Q.W + 2 * Q.pad);
  hipLaunchKernelGGL(x4_pack_act_kernel, dim3((npos + 63) / 64, Q.nchunk, P.B), dim3(256), 0, st, Q);
  HIP_OK(hipGetLastError());
}

// split-K combine: out = epilogue(sum over the nsplit partial planes, in split order)
__global__ __launch_bounds__(256) void x4_split_reduce_kernel(ConvParams P, const float* __restrict__ part,
                                                              int nsplit) {
  const int HWo = P.Ho * P.Wo;
  const int64_t n = (int64_t)P.B * P.Cout * HWo;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int p = (int)(i % HWo);
  const int64_t r = i / HWo;
  const int co = (int)(r % P.Cout), b = (int)(r / P.Cout);
  float v = part[i];
  for (int k = 1; k < nsplit; ++k) v += part[(int64_t)k * n + i];
  conv_store(P, b, co, p, v);
}

// $MLIC_X4_RS=0: the LDS-DMA operand path (A/B switch); default the register-staged one
static bool x4_rs() {
  static const bool on = [] {
    const char* e = std::getenv("MLIC_X4_RS");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

// the halo-staged B operand (conv_x4_kernel HALO) for a packed K x K stride-1 conv whose LDS images fit;
// $MLIC_X4_HALO=0: B staged per tap (A/B switch)
static int g_x4_halo = -1;  // mlic_set_kernel_option("x4_halo"): -1 = $MLIC_X4_HALO / default (5 x 5 only)
void x4_set_halo(int on) { g_x4_halo = on; }
// 0 = off, 1 = 5 x 5 only (the default), 2 = 3 x 3 too ($MLIC_X4_HALO=2; the option's 1 means 3 x 3 too)
static int x4_halo_setting() {
  static const int env = [] {
    const char* e = std::getenv("MLIC_X4_HALO");
    return e ? std::atoi(e) : 1;
  }();
  if (g_x4_halo >= 0) return g_x4_halo == 0 ? 0 : 2;
  return env;
}
static bool x4_halo_on() { return x4_halo_setting() != 0; }
template <int K, int BM>
constexpr bool x4_halo_fits() {
  constexpr int a = 2 * BM * ROWB, h = 2 * (TR + K - 1) * (TC + K - 1) * ROWB;
  return K > 1 && a + h <= 160 * 1024;
}
// Measured (tools/gpu/r4_halo.sh, 8 images, profiles/r04/ab/): 5x5 reprojection 320 -> 320 at 68 x 120
// 1396 -> 1303 us; 3x3 g_s subpel conv 192 -> 768 at 272 x 480 7146 -> 7215 us and at 136 x 240 2133 ->
// 2115 us (the per-tap fragment addresses become runtime: the swizzle of a tap-shifted line is
// recomputed per read, which eats the saved B loads).  Default: 5x5 only; "x4_halo" = 1 forces it for
// 3x3 too (A/B), 0 turns it off.
static bool x4_halo(const ConvParams& P, bool hi) {
  if (!x4_halo_on() || P.K == 1 || P.stride != 1) return false;
  if (P.K == 3 && x4_halo_setting() != 2) return false;
  const int bm = x4_bm(P.Cout);
  return 2 * bm * ROWB + 2 * (TR + P.K - 1) * (TC + P.K - 1) * ROWB <= 160 * 1024;
}

// $MLIC_X4_DIRECT=0: 1x1 layers read the packed copy too (A/B switch)
bool x4_direct_ok(const ConvParams& P, bool hi) {
  static const bool on = [] {
    const char* e = std::getenv("MLIC_X4_DIRECT");
    return !(e && std::atoi(e) == 0);
  }();
  return on && P.K == 1 && !hi && !(P.epi & EPI_SQUARE_IN) && x4_rs();
}

template <int K, int BM>
static void launch_x4(const ConvParams& P, const _Float16* act, const _Float16* wx, int nchunk, hipStream_t st,
                      int nsplit, bool hi) {
  int H, W;
  x4_tgrid(P, H, W);
  const int ntx = (W + TC - 1) / TC, nty = (H + TR - 1) / TR;
  dim3 grid((P.Cout + BM - 1) / BM, ntx * nty, P.B * nsplit);
  static const int abl = [] {
    const char* e = std::getenv("MLIC_X4_ABL");  // diagnostics: 1 = no DMA in the loop, 2 = no MFMA
    return e ? std::atoi(e) : 0;
  }();
  if (K == 1 && !act)
    hipLaunchKernelGGL((conv_x4_kernel<K, BM, true, false, K == 1>), grid, dim3(X4T), 0, st, P, act, wx, nchunk, H, W,
                       abl, nsplit);
  else if (hi && x4_halo(P, hi)) {
    if constexpr (x4_halo_fits<K, BM>())
      hipLaunchKernelGGL((conv_x4_kernel<K, BM, true, true, false, true>), grid, dim3(X4T), 0, st, P, act, wx, nchunk,
                         H, W, abl, nsplit);
  } else if (hi)
    hipLaunchKernelGGL((conv_x4_kernel<K, BM, true, true>), grid, dim3(X4T), 0, st, P, act, wx, nchunk, H, W, abl,
                       nsplit);
  else if (x4_rs() && x4_halo(P, hi)) {
    if constexpr (x4_halo_fits<K, BM>())
      hipLaunchKernelGGL((conv_x4_kernel<K, BM, true, false, false, true>), grid, dim3(X4T), 0, st, P, act, wx, nchunk,
                         H, W, abl, nsplit);
  } else if (x4_rs())
    hipLaunchKernelGGL((conv_x4_kernel<K, BM, true, false>), grid, dim3(X4T), 0, st, P, act, wx, nchunk, H, W, abl,
                       nsplit);
  else if constexpr (BM != 192 && BM != 96 && BM != 224)  // (the DMA path's counted waits: 1, 2 or 4 A pieces per wave)
    hipLaunchKernelGGL((conv_x4_kernel<K, BM, false, false>), grid, dim3(X4T), 0, st, P, act, wx, nchunk, H, W, abl, 1);
  else
    hipLaunchKernelGGL((conv_x4_kernel<K, BM, true, false>), grid, dim3(X4T), 0, st, P, act, wx, nchunk, H, W, abl,
                       nsplit);
  HIP_OK(hipGetLastError());
}

// split-K factor: a launch of few tiles per image (the latent-resolution 5x5 reprojections: 36 tiles
// of one Cout tile, 1.1 waves of blocks over the CUs at 8 images) with a long K loop is cut into
// nsplit K ranges whose partial sums a combine kernel adds in a fixed order.  A function of the
// per-image shape only: the result bits must not depend on the batch (encoder = decoder).
// Round 4: OFF by default.  Alone on the GPU a split launch is faster, but the timed configuration
// keeps 8 lanes of kernels in flight, which fill the CUs those few-tile launches leave idle, and the
// split adds a partial-sum pass and a combine launch: main config 91.1 / 91.6 img/s without against
// 90.2 / 90.3 with (alternating, one box); Kodak-size and MLICPP_M_SMALL_DEC within noise.
// $MLIC_X4_SPLITK=1 or mlic_set_kernel_option("x4_splitk", 1) turns it on (tests, A/B).
static int g_x4_splitk = -1;
void x4_set_splitk(int v) { g_x4_splitk = v; }
int x4_splitk(const ConvParams& P, int cin_pad, bool hi) {
  static const bool env_on = [] {
    const char* e = std::getenv("MLIC_X4_SPLITK");
    return e && std::atoi(e) != 0;
  }();
  const bool on = g_x4_splitk >= 0 ? g_x4_splitk != 0 : env_on;
  if (!on || !x4_rs() || P.K == 1) return 1;
  int H, W;
  x4_tgrid(P, H, W);
  const int tiles = ((P.Cout + x4_bm(P.Cout) - 1) / x4_bm(P.Cout)) * ((W + TC - 1) / TC) * ((H + TR - 1) / TR);
  const int nsteps = x4_nchunk(cin_pad, hi) * P.K * P.K;
  if (tiles > 48 || nsteps < 48) return 1;
  const int s = std::min(4, nsteps / 24);
  // the halo form splits on chunk boundaries: no more splits than chunks
  return x4_halo(P, hi) ? std::max(1, std::min(s, x4_nchunk(cin_pad, hi))) : s;
}

int64_t x4_part_bytes(const ConvParams& P, int cin_pad, bool hi) {
  const int s = x4_splitk(P, cin_pad, hi);
  return s > 1 ? (int64_t)s * P.B * P.Cout * P.Ho * P.Wo * 4 : 0;
}

void conv_x4_forward(const ConvParams& P, const _Float16* act, const _Float16* wx, int cin_pad, hipStream_t st,
                     float* part, bool hi) {
  // act == nullptr: the direct form (x4_direct_ok), which reads the ConvParams input segments;
  // otherwise they are not read: the packed copy (x4_pack_act) is
  MLIC_CHECK(conv_x4_ok(P, cin_pad) && wx && (act || x4_direct_ok(P, hi)), "conv_x4: unsupported shape");
  ConvParams Q = P;
  if (act) Q.epi &= ~EPI_SQUARE_IN;
  const int nchunk = x4_nchunk(cin_pad, hi);
  const int bm = x4_bm(P.Cout);
  const int nsplit = part ? x4_splitk(P, cin_pad, hi) : 1;
  ConvParams R = Q;  // the launch's view: the raw partial planes when split
  if (nsplit > 1) {
    R.epi = EPI_NONE;
    R.bias = nullptr;
    R.wexp = 0;
    R.aux = nullptr;
    R.res = nullptr;
    R.out = part;
    R.out_cs = (int64_t)P.Ho * P.Wo;
    R.out_bs = (int64_t)P.Cout * R.out_cs;
  }
#define MLIC_X4_BM(K)                                                  \
  (bm == 256 ? launch_x4<K, 256>(R, act, wx, nchunk, st, nsplit, hi)       \
   : bm == 192 ? launch_x4<K, 192>(R, act, wx, nchunk, st, nsplit, hi)     \
   : bm == 96 ? launch_x4<K, 96>(R, act, wx, nchunk, st, nsplit, hi)       \
   : bm == 224 ? launch_x4<K, 224>(R, act, wx, nchunk, st, nsplit, hi)     \
   : bm == 128 ? launch_x4<K, 128>(R, act, wx, nchunk, st, nsplit, hi)     \
               : launch_x4<K, 64>(R, act, wx, nchunk, st, nsplit, hi))
  switch (P.K) {
    case 1: MLIC_X4_BM(1); break;
    case 3: MLIC_X4_BM(3); break;
    default: MLIC_X4_BM(5); break;
  }
#undef MLIC_X4_BM
  if (nsplit > 1) {
    const int64_t n = (int64_t)P.B * P.Cout * P.Ho * P.Wo;
    hipLaunchKernelGGL(x4_split_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, Q,
                       (const float*)part, nsplit);
    HIP_OK(hipGetLastError());
  }
}

}  // namespace mlic
