// Fused depthwise-separable conv, row-pipelined producer / consumer form ("dwpw2"): the fork's
// DepthWiseConv (modules/layers/conv.py:22-32, 46-63: depthwise 3x3 stride 1 pad 1 + bias, pointwise
// 1x1 + bias, then the block's GELU / residual; res_blk.py:62-154) in one kernel, for the
// full-resolution g_a / g_s layers (Cin = Cout = N, N a multiple of 32).  Same arithmetic as
// conv_dwpw.hip's dwpw_kernel, bit for bit: the depthwise in dw3x3's FMA order, the hi / lo split, the
// three split-fp16 MFMA terms per k-step in pw_resident's order (transposed operands give the same
// bits), pw_resident's epilogue.
//
// Why a second form: dwpw_kernel keeps the split weights in LDS and ALL N output rows of 64 pixels in
// the accumulators of one wave per SIMD, so a wave serialises its loads, its MFMA + depthwise stream and
// its stores (ablation, 8 x 192 x 544 x 960 GELU: loads alone 0.72 ms, + stores 2.12, + MFMA 1.56,
// everything 2.40; profiles/r05/ab/dwpw_ablation.log).  Here the weights live in REGISTERS and the
// depthwise output in LDS; a CU runs N / 16 waves (three per SIMD at N = 192) with two jobs:
//   * consumers (waves 0 .. N/32 - 1): wave w owns output channels 32w .. 32w + 31; its split weights
//     are the B operand of v_mfma_f32_32x32x16_f16 for every k-step (96 VGPRs at N = 192), the A
//     operand is the depthwise output of one 32-pixel row block read from LDS.  D = X^T W^T: a lane
//     holds 4 consecutive PIXELS of one channel, so each step ends with 4 dwordx4 stores per wave.
//   * producers (waves N/32 .. N/16 - 1): producer p owns input channels 32p .. 32p + 31 of every step.
//     It stages its channels of one input row per step into LDS by LDS-DMA (global_load_lds_dwordx4,
//     a zero page as the source where the row leaves the image), keeps the two previous rows of its
//     channels in registers (the vertical window), and writes the split depthwise output of the next
//     row block into the A image.
// Work unit: a strip of R rows x 32 columns; a step = one output row of the strip.  Iteration s:
// consumers MFMA row ys + s from A[s & 1] and store it; producers DMA input row ys + s + 3 into raw
// slot s & 1 and compute output row ys + s + 1 (window rows ys + s, ys + s + 1 and the new row ys + s + 2
// from slot (s + 1) & 1) into A[(s + 1) & 1]; then s_waitcnt lgkmcnt(0) + s_barrier.  Every input row
// crosses the memory system once per strip (+ 2 rows of vertical halo per R, + 8 columns of
// horizontal halo per 32), and every step both reads and writes, so the per-CU memory stream is even.
// (A first form stepped over 32-channel chunks of 6 x 32-pixel tiles: its producers spent ~11 k cycles
// per step on DMA issue and LDS re-reads and its consumers stored a whole tile in one burst: 2.85 ms.)
// LDS: two raw slots [N][40 floats] (columns x0 - 4 .. x0 + 35: the DMA wants 16-byte aligned
// sources), two A images [k-step][hi / lo][32 pixels x 32 bytes] (the 16-byte halves of pixel row n
// swapped when (n >> 3) & 1: conflict-free ds_read_b128), taps, bias: 120.6 KB at N = 192.
// Needs W % 4 == 0 (16-byte pieces, dwordx4 stores), Cin = Cout = N in {96, 128, 160, 192}.
#include "../common.h"
#include "../kernels.h"

#include <cstdlib>

namespace mlic {

namespace {
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));
typedef float float4v __attribute__((ext_vector_type(4)));

constexpr int D2_TC = 32;                   // strip width: one MFMA row block
constexpr int D2_RP = 10;                   // 16-byte pieces per raw row: x0 - 4 .. x0 + 35
constexpr int D2_RF = 4 * D2_RP;            // floats per raw row of one channel
constexpr int D2_TAP = 12;                  // floats per channel: 9 taps, bias, 2 pad
constexpr int D2_NDMA = 32 * D2_RP / 64;    // DMA wave-instructions per producer per row (32 channels)
constexpr int DPP_SHL1 = 0x130, DPP_SHR1 = 0x138;  // wave_shl:1 / wave_shr:1
static_assert(32 * D2_RP % 64 == 0, "dwpw2: DMA pieces");

#ifndef MLIC_D2_FG  // channels per scheduling group of the producers' depthwise (2, 4, 8, 16)
#define MLIC_D2_FG 4
#endif
constexpr int D2_FG = MLIC_D2_FG;
#ifndef MLIC_D2_DMA  // A/B build: 1 = raw rows staged by LDS-DMA instead of registers
#define MLIC_D2_DMA 0
#endif
#ifndef MLIC_D2_RESPOS  // residual loads: 2 = unmasked (zero page), 0 = exec-masked (wrong results in some
#define MLIC_D2_RESPOS 2  // rows on gfx950: tools/gpu/d2diag_run.sh), 1 = masked + scheduling fences (same)
#endif

// the DMA source of a piece outside the image: every DMA wave-instruction is issued by all 64 lanes
// (a lane-masked skip of a whole instruction would break the producers' counted vmcnt)
__device__ float d2_zeros[4];

// global -> LDS DMA of one 16-byte piece per lane to lds_base + 16 * lane (wave-uniform base); the same
// asm form as conv_x4.hip: hipcc does not count it, the caller waits with vmcnt
__device__ __forceinline__ void d2_glds16(const float* src, uint32_t lds_base) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(lds_base) : "m0");
}

__device__ __forceinline__ void d2_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A image byte offset of pixel row n, channel half g (0: channels 0-7, 1: 8-15) in a 32 x 32-byte block
__device__ __forceinline__ uint32_t d2_aoff(int n, int g) { return (uint32_t)(n * 32 + ((g ^ ((n >> 3) & 1)) << 4)); }

template <int CTRL>
__device__ __forceinline__ float d2_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
}  // namespace

// diagnostics build (-DMLIC_D2_TRACE, tools/gpu/dwpw2_probe.hip): per-phase s_memtime cycles summed over
// the waves of each role into d2_trace[role * 8 + phase] (role 0 consumers, 1 producers)
#ifdef MLIC_D2_TRACE
__device__ unsigned long long* d2_trace;
#define D2_T0() uint64_t _t = __builtin_amdgcn_s_memtime(); uint64_t _ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define D2_TS(k)                                      \
  do {                                                \
    const uint64_t _n = __builtin_amdgcn_s_memtime(); \
    _ph[k] += _n - _t;                                \
    _t = _n;                                          \
  } while (0)
#define D2_TFLUSH(role)                                                                  \
  do {                                                                                   \
    if (lane == 0)                                                                       \
      for (int _k = 0; _k < 8; ++_k) atomicAdd(d2_trace + (role) * 8 + _k, _ph[_k]); \
  } while (0)
#else
#define D2_T0() (void)0
#define D2_TS(k) (void)0
#define D2_TFLUSH(role) (void)0
#endif

// MODE: 0 = bias only, 1 = GELU (dwpw_kernel's modes); RES: residual add last
template <int N, int MODE, bool RES>
__global__ __launch_bounds__(N / 16 * 64) void dwpw2_kernel(ConvParams P, int R, const _Float16* __restrict__ wh,
                                                           const _Float16* __restrict__ wl, int cin_pad,
                                                           const float* __restrict__ dww,
                                                           const float* __restrict__ dwb) {
  constexpr int NC = N / 32;  // consumer waves (32 output channels each) = producer waves (32 inputs)
  constexpr int KS = N / 16;  // k-steps of 16 channels
  constexpr int SLOT = N * D2_RF * 4;
  constexpr int AB = KS * 2 * 1024;
  constexpr int RAW0 = 0, AIMG0 = 2 * SLOT, TAPS0 = AIMG0 + 2 * AB, BIAS0 = TAPS0 + N * D2_TAP * 4;
  constexpr int LDS = BIAS0 + N * 4;
  static_assert(LDS <= 160 * 1024, "dwpw2: LDS");
  __shared__ __attribute__((aligned(16))) char sm[LDS];
  float* staps = reinterpret_cast<float*>(sm + TAPS0);
  float* sbias = reinterpret_cast<float*>(sm + BIAS0);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < N * D2_TAP; i += blockDim.x) {
    const int c = i / D2_TAP, k = i - c * D2_TAP;
    staps[i] = k < 9 ? dww[c * 9 + k] : (k == 9 && dwb ? dwb[c] : 0.0f);
  }
  for (int r = tid; r < N; r += blockDim.x) sbias[r] = P.bias ? P.bias[r] : 0.0f;

  const int H = P.H, W = P.W, HW = H * W;
  const int nseg = (W + D2_TC - 1) / D2_TC;
  const int nys = (H + R - 1) / R;
  const int spi = nseg * nys;  // strips per image, ordered (row band, segment)
  const int nstrips = spi * P.B;
  const int xcd = (int)blockIdx.x & 7, nslot = (int)gridDim.x >> 3;
  const int t_end = (int)((int64_t)(xcd + 1) * nstrips / 8);
  const int strip0 = (int)((int64_t)xcd * nstrips / 8) + ((int)blockIdx.x >> 3);
  const int nstrip = strip0 < t_end ? (t_end - strip0 + nslot - 1) / nslot : 0;
  if (nstrip == 0) return;  // the whole workgroup, before any barrier
  auto strip_of = [&](int k, int& b, int& ys, int& x0) {
    const int t = strip0 + k * nslot;
    b = t / spi;
    const int r = t - b * spi;
    const int yb = r / nseg;
    ys = yb * R;
    x0 = (r - yb * nseg) * D2_TC;
  };

  if (wave >= NC) {
    // ------------------------------------------------------------------------------ producers
    const int pw = wave - NC;  // input channels 32 pw .. 32 pw + 31
    const int c = lane & 31, q = lane >> 5;
    const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)sm);
    const float* zp = d2_zeros;
    asm volatile("" : "+v"(zp));  // keep the zero page's address in registers (no re-load per DMA)
    // this lane's piece of DMA instruction i: channel 32 pw + j, piece k; its offset from the row base
    int doff[D2_NDMA], dpc[D2_NDMA];
#pragma unroll
    for (int i = 0; i < D2_NDMA; ++i) {
      const int qq = 64 * i + lane;
      const int j = qq / D2_RP, k = qq - j * D2_RP;
      doff[i] = j * HW + 4 * k;
      dpc[i] = k;
    }
    const float* ximg = nullptr;
    int ys = 0, x0 = 0, colmask = 0;
    // DMA input row Y (channels 32 pw ..) into raw slot `slot`
    // register staging (default; MLIC_D2_DMA=1 builds the LDS-DMA form): the row's 16-byte pieces are
    // loaded into registers one row ahead and written into their slot with ds_write_b128 when the slot
    // is free.  Measured: the LDS-DMA form spent most of its producers' time issuing the DMAs
    // (global_load_lds_dwordx4 + M0 writes; tools/gpu/dwpw2_probe.hip), register staging a fraction.
    float4v stg0[D2_NDMA];  // the row in flight
    auto load_row = [&](int Y, float4v (&stg)[D2_NDMA]) {
      const bool rok = Y >= 0 && Y < H;
      const float* rb = ximg + (int64_t)(32 * pw) * HW + (int64_t)(rok ? Y : 0) * W + (x0 - 4);
#pragma unroll
      for (int i = 0; i < D2_NDMA; ++i) {
        const bool ok = rok && ((colmask >> dpc[i]) & 1);
        stg[i] = *reinterpret_cast<const float4v*>(ok ? rb + doff[i] : zp);
      }
    };
    auto store_row = [&](int slot, const float4v (&stg)[D2_NDMA]) {
      char* dst = sm + RAW0 + slot * SLOT + 32 * pw * D2_RF * 4 + 16 * lane;
#pragma unroll
      for (int i = 0; i < D2_NDMA; ++i) *reinterpret_cast<float4v*>(dst + 64 * 16 * i) = stg[i];
    };
    auto dma_row = [&](int Y, int slot) {
      const bool rok = Y >= 0 && Y < H;
      const float* rb = ximg + (int64_t)(32 * pw) * HW + (int64_t)(rok ? Y : 0) * W + (x0 - 4);
      const uint32_t dst = lds0 + (uint32_t)(RAW0 + slot * SLOT + 32 * pw * D2_RF * 4);
#pragma unroll
      for (int i = 0; i < D2_NDMA; ++i) {
        const bool ok = rok && ((colmask >> dpc[i]) & 1);
        d2_glds16(ok ? rb + doff[i] : zp, dst + (uint32_t)(64 * 16 * i));
      }
    };
    // running depthwise sums of the lane's 16 channels (32 pw + 16 q + i) at column x0 + c: every input
    // row adds its three tap rows to the three output rows it touches, so each output row accumulates
    // its input rows in order dy = 0, 1, 2 and, within a row, dx = 0, 1, 2 -- exactly
    // dw3x3_s1_vec_kernel's fma order (acc = 0, taps row-major, + bias last); only the newest input row
    // is read (from its raw slot), the two rows before it live on as the partial sums
    float pa[16], pb[16];  // output rows Y (two tap rows in) and Y + 1 (one tap row in)
    uint32_t tapo = (uint32_t)((32 * pw + 16 * q) * D2_TAP);  // floats
    // feed input row `slot` with tap rows (dy for pa, dy - 1 for pb, dy - 2 for the new partial): the
    // stage flags say which of the three outputs it touches; complete = pa is finished (into A `buf`)
    auto feed = [&](int slot, bool to_pa, bool to_pb, int buf) {
      uint32_t rawo = (uint32_t)(RAW0 / 4 + slot * (SLOT / 4) + (32 * pw + 16 * q) * D2_RF + c + 3);  // floats
      half8 bh[2], bl[2];
#pragma unroll
      for (int i = 0; i < 16; i += D2_FG) {
        // a scheduling fence per channel group (and the tap / row offsets redefined): otherwise the
        // compiler hoists every tap and row read of the 16 channels and spills
        asm volatile("" : "+v"(tapo), "+v"(rawo));
        __builtin_amdgcn_sched_barrier(0);
        const float* r = reinterpret_cast<const float*>(sm) + rawo;
        float o[D2_FG];
#pragma unroll
        for (int e = 0; e < D2_FG; ++e) {
          const float* rc = r + (i - i / D2_FG * D2_FG + e) * D2_RF;
          const float L = rc[0], C = rc[1], Rr = rc[2];
          const float* tp = staps + tapo + (i + e) * D2_TAP;
          const float4 w0 = *reinterpret_cast<const float4*>(tp);
          const float4 w1 = *reinterpret_cast<const float4*>(tp + 4);
          const float2 w2 = *reinterpret_cast<const float2*>(tp + 8);
          // dy = 2 into the finishing row, dy = 1 into the next, dy = 0 starts the one after
          float a = pa[i + e], bsum = pb[i + e], nw = 0.0f;
          // (uniform branches: a strip's first two rows skip the sums that are not started yet; they also
          // keep the compiler from scheduling the 16 channels as one block, which spills)
          if (to_pa) {
            a = fmaf(w1.z, L, a);
            a = fmaf(w1.w, C, a);
            a = fmaf(w2.x, Rr, a);
          }
          if (to_pb) {
            bsum = fmaf(w0.w, L, bsum);
            bsum = fmaf(w1.x, C, bsum);
            bsum = fmaf(w1.y, Rr, bsum);
          }
          nw = fmaf(w0.x, L, nw);
          nw = fmaf(w0.y, C, nw);
          nw = fmaf(w0.z, Rr, nw);
          o[e] = a + w2.y;  // + bias: the finished output row
          pa[i + e] = bsum;
          pb[i + e] = nw;
        }
#pragma unroll
        for (int e = 0; e < D2_FG; e += 2) {
          const float2v vv = {o[e], o[e + 1]};
          const half2v hv = __builtin_convertvector(vv, half2v);
          const half2v lv = __builtin_convertvector(vv - __builtin_convertvector(hv, float2v), half2v);
          const int k = i + e;
          bh[k >> 3][k & 7] = hv[0];
          bh[k >> 3][(k & 7) + 1] = hv[1];
          bl[k >> 3][k & 7] = lv[0];
          bl[k >> 3][(k & 7) + 1] = lv[1];
        }
        rawo += D2_FG * D2_RF;
      }
      if (buf >= 0) {  // (uniform)
        char* a = sm + AIMG0 + buf * AB + (2 * pw + q) * 2048;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          *reinterpret_cast<half8*>(a + d2_aoff(c, g)) = bh[g];
          *reinterpret_cast<half8*>(a + 1024 + d2_aoff(c, g)) = bl[g];
        }
      }
    };
    d2_barrier();  // taps / bias written by every wave
    D2_T0();
    for (int k = 0; k < nstrip; ++k) {
      int b;
      strip_of(k, b, ys, x0);
      ximg = P.seg[0].p + (int64_t)b * P.seg[0].bs;
      colmask = 0;
#pragma unroll
      for (int j = 0; j < D2_RP; ++j) {
        const int x = x0 - 4 + 4 * j;
        colmask |= (x >= 0 && x + 4 <= W) ? (1 << j) : 0;
      }
      // input rows ys - 1 + u, u = 0 .. R + 1, fed in order (row u from raw slot u & 1): row u >= 2 finishes
      // output row ys + u - 2 into A[u & 1]; one barrier after every u >= 2 (the consumers' prologue
      // barrier, then one per output row), plus the one after the last row's consumption
#if MLIC_D2_DMA
      dma_row(ys - 1, 0);
      dma_row(ys, 1);
      for (int u = 0; u < R + 3; ++u) {
        if (u <= R + 1) {
          if (u + 1 <= R + 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D2_NDMA) : "memory");  // row u landed
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          D2_TS(1);
          feed(u & 1, u >= 2, u >= 1, u >= 2 ? (u & 1) : -1);
          D2_TS(2);
          if (u + 2 <= R + 1) dma_row(ys + u + 1, u & 1);  // the slot's reads are consumed
          D2_TS(0);
        }
        if (u >= 2) {
          d2_barrier();
          D2_TS(3);
        }
      }
#else
      // row u (= ys - 1 + u) is loaded into registers at step u - 2, written into slot u & 1 at step
      // u - 1 (the slot's previous row was fed at u - 2), fed at step u.  (Two rows in flight -- a second
      // register set -- made the compiler spill the producer at the three-waves-per-SIMD register cap.)
      load_row(ys - 1, stg0);
      store_row(0, stg0);
      load_row(ys, stg0);
      for (int u = 0; u < R + 3; ++u) {
        if (u <= R + 1) {
          if (u + 1 <= R + 1) store_row((u + 1) & 1, stg0);  // row u + 1
          if (u + 2 <= R + 1) load_row(ys + u + 1, stg0);    // row u + 2
          D2_TS(1);
          feed(u & 1, u >= 2, u >= 1, u >= 2 ? (u & 1) : -1);
          D2_TS(2);
        }
        if (u >= 2) {
          d2_barrier();
          D2_TS(3);
        }
      }
#endif
    }
    D2_TFLUSH(1);
    return;
  }

  // -------------------------------------------------------------------------------- consumers
  const int cw = wave;
  const int n = lane & 31, h = lane >> 5;
  // weights: A operand of k-step k = W[32 cw .. +32][16 k .. +16]: lane holds row n (output channel
  // 32 cw + n), channels 16 k + 8 h .. + 8 of hi and of lo; the B operand is the depthwise image (lane:
  // pixel n, channels 8 h ..), so D = W X is laid out as pw_resident's: lane = pixel x0 + n, register q =
  // output channel 32 cw + 8 (q / 4) + 4 h + q % 4 -- each store instruction writes two whole 128-byte
  // channel rows (a D = X^T W^T layout, 4 pixels per lane, wrote 32 partial lines of 32 bytes and was
  // slower)
  half8 bwh[KS], bwl[KS];
  {
    const _Float16* ph = wh + (int64_t)(32 * cw + n) * cin_pad + 8 * h;
    const _Float16* pl = wl + (int64_t)(32 * cw + n) * cin_pad + 8 * h;
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      bwh[k] = *reinterpret_cast<const half8*>(ph + 16 * k);
      bwl[k] = *reinterpret_cast<const half8*>(pl + 16 * k);
    }
  }
  // the weights landed once, here: otherwise the compiler keeps their loads "in flight" into the row
  // loop and its per-k-step vmcnt waits there drain the previous row's stores every row
  __builtin_amdgcn_s_waitcnt(0);
  d2_barrier();  // taps / bias
  const float unscale = ldexpf(1.0f, -P.wexp);
  const uint32_t aoff = d2_aoff(n, h);
  const float* sb = sbias + 32 * cw + 4 * h;  // + 8 (q / 4) + q % 4
  bool bad = false;
  D2_T0();
  for (int k = 0; k < nstrip; ++k) {
    int b, ys, x0;
    strip_of(k, b, ys, x0);
    float* ob = P.out + (int64_t)b * P.out_bs + (int64_t)(32 * cw) * HW + x0 + n;
    const float* rb = RES ? P.res + (int64_t)b * P.res_bs + (int64_t)(32 * cw) * HW + x0 + n : nullptr;
    const bool col_ok = x0 + n < W;
    d2_barrier();  // the strip's A[0]
    D2_TS(2);
    for (int s = 0; s < R; ++s) {
      const char* a = sm + AIMG0 + (s & 1) * AB + aoff;
      const int y = ys + s;
      floatx16 acc;
      // the A fragments one k-step ahead of their MFMAs
      half8 ah = *reinterpret_cast<const half8*>(a);
      half8 al = *reinterpret_cast<const half8*>(a + 1024);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        half8 nh = ah, nl = al;
        if (ks + 1 < KS) {
          nh = *reinterpret_cast<const half8*>(a + (ks + 1) * 2048);
          nl = *reinterpret_cast<const half8*>(a + (ks + 1) * 2048 + 1024);
        }
        // pw_resident's term order: (W lo . X hi), (W hi . X lo), (W hi . X hi)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bwl[ks], ah, ks == 0 ? floatx16{} : acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bwh[ks], al, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bwh[ks], ah, acc, 0, 0, 0);
        ah = nh;
        al = nl;
      }
      D2_TS(0);
#if MLIC_D2_RESPOS == 1
      __builtin_amdgcn_sched_barrier(0);
#endif
      // epilogue of output row y (pw_resident's op sequence).  The residual: one coalesced dword per lane
      // and channel (whole 128-byte rows), loaded after the MFMAs (before them, its 16 registers beside
      // the weights, the accumulators and the prefetched fragments spill at the three-wave cap)
      float xr[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        xr[q] = 0.0f;
        if constexpr (RES) {
#if MLIC_D2_RESPOS == 2
          const bool rok = y < H && col_ok;
          xr[q] = *(rok ? rb + (int64_t)(8 * (q >> 2) + 4 * h + (q & 3)) * HW + (int64_t)y * W : d2_zeros);
#elif MLIC_D2_RESPOS == 3
          (void)rb;
#else
          if (y < H && col_ok) xr[q] = rb[(int64_t)(8 * (q >> 2) + 4 * h + (q & 3)) * HW + (int64_t)y * W];
#endif
        }
      }
#if MLIC_D2_RESPOS == 1
      __builtin_amdgcn_sched_barrier(0);
#endif
      if (y < H) {
        float* orow = ob + (int64_t)y * W;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 b4 = *reinterpret_cast<const float4*>(sb + 8 * g);
          const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int q = 4 * g + e;
            float tv = __builtin_fmaf(acc[q], unscale, bq[e]);
            if constexpr (MODE == 1) tv = gelu_erf(tv);
            tv = tv + xr[q];
            bad |= col_ok && !(__builtin_fabsf(tv) <= 3.4e38f);
            if (col_ok) orow[(int64_t)(8 * g + 4 * h + e) * HW] = tv;
          }
        }
      }
      D2_TS(1);
      d2_barrier();
      D2_TS(2);
    }
  }
  D2_TFLUSH(0);
  range_report(P.rflag, bad);
}

static int d2_num_cus() { return device_cu_count(); }

static int d2_mode(const ConvParams& P) {
  const int e = P.epi & ~EPI_RES;
  if (e == EPI_NONE) return 0;
  if (e == EPI_GELU) return 1;
  return -1;
}

// rows per strip: about 32, evened out over the image height
static int d2_rows(int H) {
  const int n = std::max(1, (H + 16) / 32);
  return (H + n - 1) / n;
}

// the A/B arm 1 of mlic_set_kernel_option("dwpw2") (the form selection is in conv_dwpw3.hip)
bool dwpw2_lds_ok(const ConvParams& P, int cin_pad) {
  if (P.K != 1 || P.stride != 1 || P.pad != 0 || P.nseg != 1 || P.seg[0].C != P.Cin || cin_pad < P.Cin) return false;
  if (P.Cin != P.Cout || (P.Cin != 96 && P.Cin != 128 && P.Cin != 160 && P.Cin != 192)) return false;
  if (d2_mode(P) < 0) return false;
  if (P.Ho != P.H || P.Wo != P.W || P.out_cs != (int64_t)P.H * P.W || (P.W % 4) != 0) return false;
  if ((int64_t)P.Cin * P.H * P.W * 4 >= (1ll << 31)) return false;
  return true;
}

template <int N, int M, bool RS>
static void launch_dwpw2(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                         const float* dwb, hipStream_t st) {
  const int R = d2_rows(P.H);
  const int64_t want = (int64_t)((P.W + D2_TC - 1) / D2_TC) * ((P.H + R - 1) / R) * P.B;
  const int64_t g = std::min<int64_t>(want, (int64_t)d2_num_cus());
  const dim3 grid((unsigned)((g + 7) / 8 * 8));  // a multiple of 8: the XCD-aware deal
  hipLaunchKernelGGL((dwpw2_kernel<N, M, RS>), grid, dim3(N / 16 * 64), 0, st, P, R, wh, wl, cin_pad, dww, dwb);
  HIP_OK(hipGetLastError());
}

void dwpw2_lds_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                       const float* dwb, hipStream_t st) {
  MLIC_CHECK(dwpw2_lds_ok(P, cin_pad) && dww, "dwpw2: unsupported shape");
  const int mode = d2_mode(P), res = (P.epi & EPI_RES) ? 1 : 0;
#define D2_RUN(NN)                                                                               \
  if (P.Cin == NN) {                                                                             \
    if (mode == 0 && !res) return launch_dwpw2<NN, 0, false>(P, wh, wl, cin_pad, dww, dwb, st); \
    if (mode == 0 && res) return launch_dwpw2<NN, 0, true>(P, wh, wl, cin_pad, dww, dwb, st);   \
    if (mode == 1 && !res) return launch_dwpw2<NN, 1, false>(P, wh, wl, cin_pad, dww, dwb, st); \
    return launch_dwpw2<NN, 1, true>(P, wh, wl, cin_pad, dww, dwb, st);                          \
  }
  D2_RUN(192) D2_RUN(160) D2_RUN(128) D2_RUN(96)
#undef D2_RUN
}

}  // namespace mlic
