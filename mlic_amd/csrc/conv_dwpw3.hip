// Fused depthwise-separable conv, register-row producer / consumer form ("dwpw3"): the fork's
// DepthWiseConv (modules/layers/conv.py:22-32, 46-63: depthwise 3x3 stride 1 pad 1 + bias, pointwise
// 1x1 + bias, then the block's GELU / residual; res_blk.py:62-154) in one kernel for the full-resolution
// g_a / g_s layers (Cin = Cout = N).  Bit for bit the arithmetic of dwpw_kernel / dwpw2_kernel: the
// depthwise in dw3x3's FMA order (acc = 0, taps row-major, + bias), the hi / lo split, the three
// split-fp16 MFMA terms per k-step in pw_resident's order, pw_resident's epilogue.
//
// dwpw2 (conv_dwpw2.hip) staged every input row in LDS and read it back three times per output, with the
// taps, from LDS: its producers issued ~6 LDS reads per channel and pixel and waited on each group of
// them, and the consumers sat at the barriers (tools/gpu/dwpw2_probe.hip).  Here a producer lane owns one
// PIXEL column of a 64-pixel strip and its 32 channels live in registers:
//   * the input row of each channel is one coalesced 256-byte dword load per wave (C), its horizontal
//     neighbours come from the lanes beside it by DPP wave shifts, and the two strip-edge pixels ride in
//     a second load (E) whose lanes 0 / 63 the shifts fall back to;
//   * the vertical window is two running partial sums per channel (pa: the output row two tap rows in,
//     pb: one tap row in), so each input row is read once and added to the three output rows it touches
//     in dw3x3's order;
//   * the taps are wave-uniform: scalar loads (s_load) straight from the weight tensor, FMAs with an SGPR
//     operand -- no LDS traffic for them;
//   * the next row's loads are issued channel by channel as soon as the current row's value is consumed,
//     a whole step of latency ahead.
// The only LDS traffic is the split depthwise image (two 64-pixel blocks per step, ds_write_b128) and the
// consumers' MFMA operand reads of it.
// Consumers (waves 0 .. N/32 - 1): wave w owns output channels 32 w .. 32 w + 31 with its split weights in
// registers (the A operand of v_mfma_f32_32x32x16_f16 for every k-step), B = the depthwise image; a step is
// one output row of the strip, two 32-pixel blocks one after the other.  One s_barrier per step: producers
// write A[(s + 1) & 1] while consumers read A[s & 1].
// Work unit: a strip of R rows x 64 columns (R ~ 32: 2 rows of vertical halo per R), strips dealt to
// workgroups in contiguous ranges per XCD.
// LDS: two A images [k-step][block][hi / lo][32 pixels x 32 bytes] + bias: 97.3 KB at N = 192.
#include "common.h"
#include "kernels.h"

#include <cstdlib>

namespace mlic {

namespace {
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));

constexpr int D3_TC = 64;  // strip width: one pixel per producer lane = two MFMA column blocks
constexpr int D3_G = 8;    // producer channels per A-image write (one 16-byte piece of hi and of lo)

#ifndef MLIC_D3_FAKETAPS
#define MLIC_D3_FAKETAPS 0
#endif
#ifndef MLIC_D3_ABL  // timing ablations (wrong results): 1 no producer row loads, 2 no consumer stores,
#define MLIC_D3_ABL 0  // 4 no MFMAs, 8 no depthwise FMAs (the raw value written), 16 no A writes
#endif
#ifndef MLIC_D3_ASYNC  // 1: producer / consumer hand-off by LDS counters instead of one s_barrier per step
#define MLIC_D3_ASYNC 0
#endif
#ifndef MLIC_D3_NBUF  // A images in the ring (2 or 3; the barrier form needs 2)
#define MLIC_D3_NBUF (MLIC_D3_ASYNC ? 3 : 2)
#endif
#ifndef MLIC_D3_PK  // consumer epilogue on channel pairs with packed-fp32 VALU (A/B: 0 = scalar)
#define MLIC_D3_PK 1
#endif
#ifndef MLIC_D3_PPK  // producer depthwise on channel pairs with packed-fp32 VALU (A/B: 0 = scalar)
#define MLIC_D3_PPK 0
#endif
#ifndef MLIC_D3_TPF  // producer taps prefetched one channel pair ahead (A/B: 0 = loaded at use)
#define MLIC_D3_TPF 0
#endif
#ifndef MLIC_D3_TG  // producer channels per scheduling group (2, 4, 8)
#define MLIC_D3_TG (MLIC_D3_TPF ? 2 : 4)
#endif
constexpr int D3_TG = MLIC_D3_TG;

// buffer resource over `bytes` bytes at a wave-uniform base (loads past the end return 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t d3_rsrc(const float* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

__device__ __forceinline__ void d3_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LDS hand-off counters (MLIC_D3_ASYNC): every lane of a wave adds 1 (no exec-masked LDS operations in
// the MFMA waves), so one wave's event counts 64.  The wait is bounded: a broken protocol reports
// through the range flag instead of hanging the GPU.
__device__ __forceinline__ void d3_signal(uint32_t* ctr) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's A writes / reads are done
  __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool d3_wait_geq(const uint32_t* ctr, uint32_t target) {
  uint32_t spins = 0;
  for (;;) {
    const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    if (v >= target) break;
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1u << 22)) return false;
  }
  asm volatile("" ::: "memory");
  return true;
}

// A image byte offset of pixel row n, channel half g (0: channels 0-7, 1: 8-15) in a 32 x 32-byte block;
// the 16-byte halves swapped when (n >> 3) & 1 (conflict-free ds_read_b128 for the consumers)
__device__ __forceinline__ uint32_t d3_aoff(int n, int g) { return (uint32_t)(n * 32 + ((g ^ ((n >> 3) & 1)) << 4)); }

// horizontal neighbours of v (this lane's pixel of one channel): L = lane - 1's (wave_shr:1), R = lane + 1's
// (wave_shl:1); at the strip edges (lanes 0 / 63, no source lane) the channel's edge pixels, which sit in
// lanes K / 63 - K of the packed edge register e and are moved into lanes 0 / 63 by row shifts
template <int K>
__device__ __forceinline__ void d3_neighbours(float e, float v, float& L, float& R) {
  const int ei = __builtin_bit_cast(int, e), vi = __builtin_bit_cast(int, v);
  int el = ei, er = ei;
  if constexpr (K > 0) {
    el = __builtin_amdgcn_mov_dpp(ei, 0x100 + K, 0xF, 0xF, true);  // row_shl:K: lane 0 <- lane K
    er = __builtin_amdgcn_mov_dpp(ei, 0x110 + K, 0xF, 0xF, true);  // row_shr:K: lane 63 <- lane 63 - K
  }
  L = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(el, vi, 0x138, 0xF, 0xF, false));
  R = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(er, vi, 0x130, 0xF, 0xF, false));
}
// d3_neighbours for a channel index known after unrolling (the DPP controls are immediates)
__device__ __forceinline__ void d3_neighbours_k(int k, float e, float v, float& L, float& R) {
  switch (k) {
#define D3_NB(K) \
  case K: return d3_neighbours<K>(e, v, L, R);
    D3_NB(0) D3_NB(1) D3_NB(2) D3_NB(3) D3_NB(4) D3_NB(5) D3_NB(6) D3_NB(7)
    D3_NB(8) D3_NB(9) D3_NB(10) D3_NB(11) D3_NB(12) D3_NB(13) D3_NB(14) D3_NB(15)
#undef D3_NB
  }
}
}  // namespace

// MODE: 0 = bias only, 1 = GELU (dwpw_kernel's modes), 2 = GDN, 3 = IGDN (pw_resident's: x * rsqrt(v),
// x * sqrt(v), the aux operand x = the conv input); RES: residual add last.  PW: the pointwise conv
// alone (no depthwise; MODE 2 / 3 convolve x * x) -- the full-resolution GDN / IGDN of g_a / g_s
template <int N, int MODE, bool RES, bool PW = false>
__global__ __launch_bounds__(N / 16 * 64) void dwpw3_kernel(ConvParams P, int R, const _Float16* __restrict__ wh,
                                                           const _Float16* __restrict__ wl, int cin_pad,
                                                           const float* __restrict__ dww,
                                                           const float* __restrict__ dwb) {
  constexpr int NC = N / 32;      // consumer waves (32 output channels each) = producer waves (32 inputs)
  constexpr int KS = N / 16;      // k-steps of 16 channels
  constexpr int AB = KS * 4096;   // one A image: [ks][block][hi / lo][1 KB]
  constexpr int NBUF = MLIC_D3_NBUF;
  constexpr int AIMG0 = 0, CTR0 = NBUF * AB, BIAS0 = CTR0 + 2 * NBUF * 4;
  constexpr int LDS = BIAS0 + N * 4;
  static_assert(LDS <= 160 * 1024, "dwpw3: LDS");
  static_assert(MLIC_D3_ASYNC || NBUF == 2, "dwpw3: the barrier form alternates two A images");
  __shared__ __attribute__((aligned(16))) char sm[LDS];
  float* sbias = reinterpret_cast<float*>(sm + BIAS0);
  // (ASYNC) filled[b]: 64 per producer that wrote A[b], freed[b]: 64 per consumer done reading it; the
  // t-th output row of the workgroup (strip-major) goes through A[t % NBUF], its (t / NBUF)-th use
  uint32_t* filled = reinterpret_cast<uint32_t*>(sm + CTR0);
  uint32_t* freed = filled + NBUF;
  if (threadIdx.x < 2 * NBUF) filled[threadIdx.x] = 0;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int r = tid; r < N; r += blockDim.x) sbias[r] = P.bias ? P.bias[r] : 0.0f;

  const int H = P.H, W = P.W, HW = H * W;
  const int nseg = (W + D3_TC - 1) / D3_TC;
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
    // (the divisions expand into VALU reciprocals: the results are pinned to scalars, otherwise every
    // address and row flag derived from them is carried per lane)
    b = __builtin_amdgcn_readfirstlane(b);
    ys = __builtin_amdgcn_readfirstlane(yb * R);
    x0 = __builtin_amdgcn_readfirstlane((r - yb * nseg) * D3_TC);
  };

  if (wave >= NC) {
    // ------------------------------------------------------------------------------ producers
    const int cb = 32 * (wave - NC);  // input channels cb .. cb + 31
    // this lane's A-image byte offsets (k-step cb / 16, its block and pixel row) for channel halves 0 / 1
    const uint32_t aw0 = AIMG0 + (uint32_t)(((cb >> 4) * 2 + (lane >> 5)) * 2048) + d3_aoff(lane & 31, 0);
    const uint32_t aw1 = aw0 - d3_aoff(lane & 31, 0) + d3_aoff(lane & 31, 1);
    float pa[32], pb[32];  // running sums of two output rows (two / one tap rows in, roles alternating)
    // the next input row: sc[j] = channel cb + j at this lane's pixel; the strip-edge pixels of 16 channels
    // share one register: se[i] lane k < 16 = channel cb + 16 i + k at x0 - 1, lane 63 - k = at x0 + 64
    float sc[32], se[2];
    // the strip's input channels cb .. cb + 31 as a buffer resource: a padding pixel (outside the row) is
    // read at an offset past the end of the buffer, which the hardware returns as 0
    __amdgpu_buffer_rsrc_t rs;
    uint32_t cxo = 0, exo = 0;  // this lane's pixel / edge pixel byte offsets in a row (or "outside")
    const uint32_t hw4 = (uint32_t)HW * 4u;
    // channel j of input row (byte offset so, advanced to channel j + 1) into sc[j], and the edges of
    // channels j .. j + 15 into se[j / 16] when j % 16 == 15 (so - 15 channels); the offset chain is opaque
    // to the compiler (it would precompute all 32 channel offsets out of the loops and spill them)
    auto load_ch = [&](int j, uint32_t& so) {
      asm volatile("" : "+s"(so));
      sc[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, cxo, so, 0));
      if (!PW && (j & 15) == 15)
        se[j >> 4] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, exo, so - 15u * hw4, 0));
      so += hw4;
    };
    // the byte offset of input row Y in the chain (rows outside the image: past the end of the buffer, so
    // that every load of the row returns 0 -- the padding rows, and the row after a strip's last)
    auto row_off = [&](int Y) {
      return (uint32_t)__builtin_amdgcn_readfirstlane(Y >= 0 && Y < H ? Y * W * 4 : 0x40000000);
    };
    auto load_row = [&](int Y) {
      uint32_t so = row_off(Y);
#pragma unroll
      for (int j = 0; j < 32; ++j) load_ch(j, so);
    };
    // feed the input row held in sc / se: tap row 2 into pa (finishing output row Y, written into A
    // `buf` when buf >= 0), tap row 1 into pb, tap row 0 starts the next; then load input row `ynext` in
    // its place (channel by channel: a step of latency ahead).  The same code for every row: in a strip's
    // first two rows the sums that are not started yet hold stale values and feed only outputs that are
    // never written (rows above the strip)
    // F: the sums two tap rows in (finished by this row), A: one tap row in.  After the row A holds the
    // sums two rows in and F the new ones: the caller swaps the roles (no register moves)
    bool pbad = false;
    auto feed = [&](float (&F)[32], float (&A)[32], int t, int ynext) {
      const int buf = t < 0 ? -1 : t % NBUF;
#if MLIC_D3_ASYNC
      // the image's previous use (row t - NBUF) read by every consumer
      if (t >= NBUF) pbad |= !d3_wait_geq(freed + buf, 64u * NC * (uint32_t)(t / NBUF));
#endif
      uint32_t so = row_off(ynext);
      uint32_t toff = (uint32_t)cb;
#if MLIC_D3_TPF
      // taps + bias of the current channel pair in scalar registers, the next pair's loaded one pair ahead
      // (the last pair of the row prefetches the first: the taps are the same every row)
      float tcur[20], tnxt[20];
      auto load_taps = [&](uint32_t t, float (&d)[20]) {
        const float* tp = dww + t * 9;
#pragma unroll
        for (int k = 0; k < 18; ++k) d[k] = tp[k];
        d[18] = dwb[t];
        d[19] = dwb[t + 1];
      };
      asm volatile("" : "+s"(toff));
      load_taps(toff, tcur);
#endif
#pragma unroll
      for (int g = 0; g < 32; g += D3_G) {
        half8 hv8, lv8;
#pragma unroll
        for (int e = 0; e < D3_G; e += 2) {
          // a scheduling fence per D3_TG channels, and the running channel index of the taps redefined
          // behind every fence by an opaque (volatile, ordered) statement: the scalar tap loads have no
          // memory dependences, and without this they float to the top of the row (320 scalar registers
          // for 32 channels) or out of the row loop altogether
          if (e % D3_TG == 0) __builtin_amdgcn_sched_barrier(0);
#if MLIC_D3_TPF
          uint32_t tnext = (g + e + 2 < 32) ? toff + 2 : (uint32_t)cb;
          asm volatile("" : "+s"(tnext));
          load_taps(tnext, tnxt);
          const float* tg = tcur;
          const float* bg = tcur + 18;
#else
          asm volatile("" : "+s"(toff));
#if MLIC_D3_FAKETAPS  // timing probe only (wrong results): the taps as constants, no scalar loads
          static constexpr float fk[20] = {.1f, .2f, .3f, .4f, .5f, .6f, .7f, .8f, .9f, .11f,
                                           .12f, .13f, .14f, .15f, .16f, .17f, .18f, .19f, .21f, .22f};
          const float* tg = fk;
          const float* bg = fk + 18;
#else
          const float* tg = dww + toff * 9;
          const float* bg = dwb + toff;
#endif
#endif
#if MLIC_D3_PPK
          // the channel pair (j, j + 1) as packed-fp32 VALU: each v_pk_fma_f32 is the two channels' fma,
          // element for element the scalar sequence (taps paired into scalar register pairs)
          const int j = g + e;
          float Ls[2], Rs[2];
          d3_neighbours_k(j & 15, se[j >> 4], sc[j], Ls[0], Rs[0]);
          d3_neighbours_k((j + 1) & 15, se[(j + 1) >> 4], sc[j + 1], Ls[1], Rs[1]);
          const mlic_float2 L2 = {Ls[0], Ls[1]}, C2 = {sc[j], sc[j + 1]}, R2 = {Rs[0], Rs[1]};
          auto tap = [&](int k) { return mlic_float2{tg[k], tg[9 + k]}; };
          mlic_float2 a2 = {F[j], F[j + 1]}, b2 = {A[j], A[j + 1]}, n2 = {0.0f, 0.0f};
          a2 = __builtin_elementwise_fma(tap(6), L2, a2);
          a2 = __builtin_elementwise_fma(tap(7), C2, a2);
          a2 = __builtin_elementwise_fma(tap(8), R2, a2);
          b2 = __builtin_elementwise_fma(tap(3), L2, b2);
          b2 = __builtin_elementwise_fma(tap(4), C2, b2);
          b2 = __builtin_elementwise_fma(tap(5), R2, b2);
          n2 = __builtin_elementwise_fma(tap(0), L2, n2);
          n2 = __builtin_elementwise_fma(tap(1), C2, n2);
          n2 = __builtin_elementwise_fma(tap(2), R2, n2);
          mlic_float2 o2 = a2 + mlic_float2{bg[0], bg[1]};
          asm volatile("" : "+v"(o2), "+v"(b2), "+v"(n2));
          A[j] = b2[0];
          A[j + 1] = b2[1];
          F[j] = n2[0];
          F[j + 1] = n2[1];
          load_ch(j, so);
          load_ch(j + 1, so);
          const float o[2] = {o2[0], o2[1]};
#else
          float o[2];
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            const int j = g + e + f;
            const float C = sc[j];
            float L, Rr;
            d3_neighbours_k(j & 15, se[j >> 4], C, L, Rr);
            const float* tp = tg + f * 9;
            float a = F[j], bs = A[j], nw = 0.0f;
#if MLIC_D3_ABL & 8
            a = C; bs = L; nw = Rr;
#else
            a = fmaf(tp[6], L, a);
            a = fmaf(tp[7], C, a);
            a = fmaf(tp[8], Rr, a);
            bs = fmaf(tp[3], L, bs);
            bs = fmaf(tp[4], C, bs);
            bs = fmaf(tp[5], Rr, bs);
            nw = fmaf(tp[0], L, nw);
            nw = fmaf(tp[1], C, nw);
            nw = fmaf(tp[2], Rr, nw);
#endif
            o[f] = a + bg[f];
            // the channel's results pinned here (opaque, ordered): the arithmetic has no chain of its own
            // and would otherwise sink to its uses (the A write, the next row) past the fences, keeping
            // every tap of the group live in scalar registers
            asm volatile("" : "+v"(o[f]), "+v"(bs), "+v"(nw));
            A[j] = bs;
            F[j] = nw;
#if !(MLIC_D3_ABL & 1)
            load_ch(j, so);
#endif
          }
#endif
          const float2v vv = {o[0], o[1]};
          const half2v hv = __builtin_convertvector(vv, half2v);
          const half2v lv = __builtin_convertvector(vv - __builtin_convertvector(hv, float2v), half2v);
          hv8[e] = hv[0];
          hv8[e + 1] = hv[1];
          lv8[e] = lv[0];
          lv8[e + 1] = lv[1];
          toff += 2;
#if MLIC_D3_TPF
          // the next pair's taps must have landed here, a pair of work after their loads (ordered use)
#pragma unroll
          for (int k = 0; k < 20; k += 4)
            asm volatile("" ::"s"(tnxt[k]), "s"(tnxt[k + 1]), "s"(tnxt[k + 2]), "s"(tnxt[k + 3]));
#pragma unroll
          for (int k = 0; k < 20; ++k) tcur[k] = tnxt[k];
#endif
        }
        if (buf >= 0) {  // (uniform)
          // k-step cb / 16 + g / 16, channel half (g / 8) & 1 (cb % 32 == 0)
          char* a = sm + buf * AB + (g >> 4) * 4096 + ((g >> 3) & 1 ? aw1 : aw0);
#if MLIC_D3_ABL & 16
          if (hv8[0] == (_Float16)12345.0f)  // (practically never: keeps the depthwise live)
#endif
          {
            *reinterpret_cast<half8*>(a) = hv8;
            *reinterpret_cast<half8*>(a + 1024) = lv8;
          }
        }
      }
#if MLIC_D3_ASYNC
      if (buf >= 0) d3_signal(filled + buf);
#endif
    };
    // PW: the input row held in sc (x, or x * x for GDN / IGDN), split into A `buf`; then input row `ynext`
    auto feed_pw = [&](int t, int ynext) {
      const int buf = t % NBUF;
      uint32_t so = row_off(ynext);
#pragma unroll
      for (int g = 0; g < 32; g += D3_G) {
        __builtin_amdgcn_sched_barrier(0);
        half8 hv8, lv8;
#pragma unroll
        for (int e = 0; e < D3_G; e += 2) {
          float o[2];
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            const int j = g + e + f;
            float v = sc[j];
            if constexpr (MODE == 2 || MODE == 3) v *= v;
            o[f] = v;
            load_ch(j, so);
          }
          const float2v vv = {o[0], o[1]};
          const half2v hv = __builtin_convertvector(vv, half2v);
          const half2v lv = __builtin_convertvector(vv - __builtin_convertvector(hv, float2v), half2v);
          hv8[e] = hv[0];
          hv8[e + 1] = hv[1];
          lv8[e] = lv[0];
          lv8[e + 1] = lv[1];
        }
        char* a = sm + buf * AB + (g >> 4) * 4096 + ((g >> 3) & 1 ? aw1 : aw0);
        *reinterpret_cast<half8*>(a) = hv8;
        *reinterpret_cast<half8*>(a + 1024) = lv8;
      }
    };
    d3_barrier();  // bias written by every wave
    if constexpr (PW) {
      // rows ys .. ys + R - 1, one per step; R + 1 barriers per strip as the consumers' (the strip's A
      // after row 0, then one per consumed row)
      for (int k = 0; k < nstrip; ++k) {
        int b, ys, x0;
        strip_of(k, b, ys, x0);
        rs = d3_rsrc(P.seg[0].p + (int64_t)b * P.seg[0].bs + (int64_t)cb * HW, 32u * hw4);
        const int xl = x0 + lane;
        cxo = xl < W ? (uint32_t)xl * 4u : 0x80000000u;
        load_row(ys);
        for (int u = 0; u <= R; ++u) {
          if (u < R) feed_pw(k * R + u, u + 1 < R ? ys + u + 1 : -1);
          d3_barrier();
        }
      }
      return;
    }
    for (int k = 0; k < nstrip; ++k) {
      int b, ys, x0;
      strip_of(k, b, ys, x0);
      rs = d3_rsrc(P.seg[0].p + (int64_t)b * P.seg[0].bs + (int64_t)cb * HW, 32u * hw4);
      const int xl = x0 + lane;
      cxo = xl < W ? (uint32_t)xl * 4u : 0x80000000u;
      // edge lanes: k < 16 the left edge of channel k, 63 - k the right edge of channel k (+ the load's
      // first channel); the other lanes read nothing
      const int xe = lane < 16 ? x0 - 1 : (lane >= 48 ? x0 + D3_TC : -1);
      const int ek = lane < 16 ? lane : 63 - lane;
      exo = xe >= 0 && xe < W ? (uint32_t)ek * hw4 + (uint32_t)xe * 4u : 0x80000000u;
      // input rows ys - 1 + u, u = 0 .. R + 1: row u >= 2 finishes output row ys + u - 2 into A[u & 1]; one
      // barrier after every u >= 2 (the consumers' strip barrier, then one per output row), plus the one
      // after the last row's consumption
      load_row(ys - 1);
      // the next row of step u: input row ys + u (none after the strip's last: a padding row)
      auto step = [&](int u, float (&F)[32], float (&A)[32]) {
        if (u <= R + 1) feed(F, A, u >= 2 ? k * R + u - 2 : -1, u + 1 <= R + 1 ? ys + u : -1);
#if !MLIC_D3_ASYNC
        if (u >= 2) d3_barrier();
#endif
      };
      for (int u = 0; u < R + 3; u += 2) {  // two steps per trip: the sum roles alternate
        step(u, pa, pb);
        if (u + 1 < R + 3) step(u + 1, pb, pa);
      }
    }
    range_report(P.rflag, pbad);
    return;
  }

  // -------------------------------------------------------------------------------- consumers
  const int cw = wave;
  const int n = lane & 31, h = lane >> 5;
  // weights: A operand of k-step k = W[32 cw .. +32][16 k .. +16]: lane holds row n (output channel
  // 32 cw + n), channels 16 k + 8 h .. + 8 of hi and of lo; B = the depthwise image (lane: pixel n of the
  // block, channels 8 h ..), so D = W X: lane = pixel, register q = output channel 32 cw + 8 (q / 4) +
  // 4 h + q % 4 -- each store instruction writes two whole 128-byte channel rows
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
  __builtin_amdgcn_s_waitcnt(0);  // the weights landed (no weight loads "in flight" inside the row loop)
  d3_barrier();  // bias
  const float unscale = ldexpf(1.0f, -P.wexp);
  const uint32_t aoff = d3_aoff(n, h);
  const float* sb = sbias + 32 * cw + 4 * h;  // + 8 (q / 4) + q % 4
  bool bad = false;
  const uint32_t hw4 = (uint32_t)HW * 4u;
  for (int k = 0; k < nstrip; ++k) {
    int b, ys, x0;
    strip_of(k, b, ys, x0);
    // the wave's 32 output channels (and residual channels) as buffer resources: a lane outside the image
    // stores / loads at an offset past the end (dropped / 0) -- no exec-masked memory operations beside
    // the MFMAs (dwpw2's masked residual loads there gave wrong results in some rows)
    const auto rs_o = d3_rsrc(P.out + (int64_t)b * P.out_bs + (int64_t)(32 * cw) * HW, 32u * hw4);
    const auto rs_r = RES ? d3_rsrc(P.res + (int64_t)b * P.res_bs + (int64_t)(32 * cw) * HW, 32u * hw4) : rs_o;
    constexpr bool GDN = MODE == 2 || MODE == 3;
    const auto rs_x = GDN ? d3_rsrc(P.aux + (int64_t)b * P.aux_bs + (int64_t)(32 * cw) * HW, 32u * hw4) : rs_o;
#if !MLIC_D3_ASYNC
    d3_barrier();  // the strip's A[0]
#endif
    for (int s = 0; s < R; ++s) {
      const int y = ys + s;
      const int t = k * R + s, buf = t % NBUF;
#if MLIC_D3_ASYNC
      bad |= !d3_wait_geq(filled + buf, 64u * NC * (uint32_t)(t / NBUF + 1));
#endif
#pragma unroll
      for (int bk = 0; bk < 2; ++bk) {
        __builtin_amdgcn_sched_barrier(0);  // the two blocks one after the other (one accumulator live)
        // this lane's output pixel and byte offset (pixel, channel 4 h); the residual of the block is loaded
        // before its MFMAs (16 dword loads in flight beside them)
        const int px = x0 + 32 * bk + n;
        const bool ok = y < H && px < W;
        const uint32_t vo = ok ? (uint32_t)(y * W + px) * 4u + (uint32_t)(4 * h) * hw4 : 0x80000000u;
        float xr[16], xa[16];
        if constexpr (GDN) {  // the GDN / IGDN input x of the block's output channels
          uint32_t so = 0;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            asm volatile("" : "+s"(so));
            xa[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_x, vo, so, 0));
            so += (q & 3) == 3 ? 5u * hw4 : hw4;
          }
        }
        if constexpr (RES) {
          uint32_t so = 0;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            asm volatile("" : "+s"(so));
            xr[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_r, vo, so, 0));
            so += (q & 3) == 3 ? 5u * hw4 : hw4;
          }
        }
        const char* a = sm + AIMG0 + buf * AB + bk * 2048 + aoff;
        floatx16 acc;
        // the B fragments one k-step ahead of their MFMAs
        half8 ah = *reinterpret_cast<const half8*>(a);
        half8 al = *reinterpret_cast<const half8*>(a + 1024);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          half8 nh = ah, nl = al;
          if (ks + 1 < KS) {
            nh = *reinterpret_cast<const half8*>(a + (ks + 1) * 4096);
            nl = *reinterpret_cast<const half8*>(a + (ks + 1) * 4096 + 1024);
          }
          // pw_resident's term order: (W lo . X hi), (W hi . X lo), (W hi . X hi)
#if MLIC_D3_ABL & 4
          if (ks == 0) acc = floatx16{};
          acc[ks & 15] += (float)ah[0] + (float)al[1] + (float)bwh[ks][0] + (float)bwl[ks][1];
#else
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bwl[ks], ah, ks == 0 ? floatx16{} : acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bwh[ks], al, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bwh[ks], ah, acc, 0, 0, 0);
#endif
          ah = nh;
          al = nl;
        }
        // epilogue of output row y, pixel x0 + 32 bk + n (pw_resident's op sequence; residual last).
        // Register q = output channel 32 cw + 8 (q / 4) + 4 h + q % 4: byte offset vo (pixel, 4 h) + the
        // uniform channel offset (8 (q / 4) + q % 4) HW 4, a running (opaque) chain
        uint32_t so = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 b4 = *reinterpret_cast<const float4*>(sb + 8 * g);
          const float bq[4] = {b4.x, b4.y, b4.z, b4.w};
          if constexpr (GDN) {
            // pw_resident's GDN epilogue: the range check on the pre-activation, x * rsqrt(v) / x * sqrt(v)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int q = 4 * g + e;
              asm volatile("" : "+s"(so));
              float tv = __builtin_fmaf(acc[q], unscale, bq[e]);
              bad |= ok && !(__builtin_fabsf(tv) <= 3.4e38f);
              tv = gdn_apply(xa[q], tv, MODE == 3);
              if constexpr (RES) tv = tv + xr[q];
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, tv), rs_o, vo, so, 0);
              so += hw4;
            }
          } else {
#if MLIC_D3_PK
          // channel pairs: the scale / bias FMA, GELU and residual add as packed-fp32 VALU (gelu_erf2: the
          // same operations element for element)
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const int q = 4 * g + e;
            mlic_float2 t2 = __builtin_elementwise_fma(mlic_float2{acc[q], acc[q + 1]}, mlic_float2{unscale, unscale},
                                                       mlic_float2{bq[e], bq[e + 1]});
            if constexpr (MODE == 1) t2 = gelu_erf2(t2);
            if constexpr (RES) t2 = t2 + mlic_float2{xr[q], xr[q + 1]};
#pragma unroll
            for (int f = 0; f < 2; ++f) {
              asm volatile("" : "+s"(so));
              // (the element copied out first: __builtin_bit_cast of the vector element lvalue t2[f] reads
              // element 0 whatever f is -- seen in the ISA)
              const float tv = t2[f];
              bad |= ok && !(__builtin_fabsf(tv) <= 3.4e38f);
#if MLIC_D3_ABL & 2
              if (tv == 12345.0f)
#endif
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, tv), rs_o, vo, so, 0);
              so += hw4;
            }
          }
#else
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int q = 4 * g + e;
            asm volatile("" : "+s"(so));
            float tv = __builtin_fmaf(acc[q], unscale, bq[e]);
            if constexpr (MODE == 1) tv = gelu_erf(tv);
            if constexpr (RES) tv = tv + xr[q];
            bad |= ok && !(__builtin_fabsf(tv) <= 3.4e38f);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, tv), rs_o, vo, so, 0);
            so += hw4;
          }
#endif
          }
          so += 4u * hw4;
        }
      }
#if MLIC_D3_ASYNC
      d3_signal(freed + buf);
#else
      d3_barrier();
#endif
    }
  }
  range_report(P.rflag, bad);
}

static int d3_num_cus() { return device_cu_count(); }

// rows per strip: the R in 8 .. 34 with the fewest steps for the busiest workgroup, rounds of strips over
// the CUs x (R + 2 halo rows + ~1 step of strip overhead).  544 x 960 x 8 keeps R = 32 (2040 strips,
// 8 rounds); 272 x 480 x 8 takes R = 34 (512 strips: 2 rounds of 37 steps, against 3 of 35 at R = 32) and
// 136 x 240 x 8 R = 17 (256 strips: every CU busy, against 128 at R = 34)
static int d3_rows(int B, int H, int W) {
  const int64_t ncu = d3_num_cus(), nseg = (W + D3_TC - 1) / D3_TC;
  int best = std::min(H, 32);
  int64_t best_cost = INT64_MAX;
  for (int R = std::min(H, 34); R >= std::min(H, 8); --R) {
    const int64_t strips = (int64_t)B * nseg * ((H + R - 1) / R);
    const int64_t cost = (strips + ncu - 1) / ncu * (R + 3);
    if (cost < best_cost) {
      best_cost = cost;
      best = R;
    }
  }
  return best;
}

bool dwpw3_shape_ok(const ConvParams& P, int cin_pad) {
  if (P.K != 1 || P.stride != 1 || P.pad != 0 || P.nseg != 1 || P.seg[0].C != P.Cin || cin_pad < P.Cin) return false;
  if (P.Cin != P.Cout || (P.Cin != 96 && P.Cin != 128 && P.Cin != 160 && P.Cin != 192)) return false;
  const int e = P.epi & ~EPI_RES;
  if (e != EPI_NONE && e != EPI_GELU) return false;
  if (P.Ho != P.H || P.Wo != P.W || P.out_cs != (int64_t)P.H * P.W) return false;
  if ((int64_t)P.Cin * P.H * P.W * 4 >= (1ll << 31)) return false;
  return true;
}
static bool d3_args_ok(const float* dww, const float* dwb) { return dww && dwb; }  // (the depthwise has a bias)

template <int N, int M, bool RS>
static void launch_dwpw3(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                         const float* dwb, hipStream_t st) {
  const int R = d3_rows(P.B, P.H, P.W);
  const int64_t want = (int64_t)((P.W + D3_TC - 1) / D3_TC) * ((P.H + R - 1) / R) * P.B;
  const int64_t g = std::min<int64_t>(want, (int64_t)d3_num_cus());
  const dim3 grid((unsigned)((g + 7) / 8 * 8));  // a multiple of 8: the XCD-aware deal
  hipLaunchKernelGGL((dwpw3_kernel<N, M, RS>), grid, dim3(N / 16 * 64), 0, st, P, R, wh, wl, cin_pad, dww, dwb);
  HIP_OK(hipGetLastError());
}

void dwpw3_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                   const float* dwb, hipStream_t st) {
  MLIC_CHECK(dwpw3_shape_ok(P, cin_pad) && d3_args_ok(dww, dwb), "dwpw3: unsupported shape");
  const int mode = (P.epi & EPI_GELU) ? 1 : 0, res = (P.epi & EPI_RES) ? 1 : 0;
#define D3_RUN(NN)                                                                               \
  if (P.Cin == NN) {                                                                             \
    if (mode == 0 && !res) return launch_dwpw3<NN, 0, false>(P, wh, wl, cin_pad, dww, dwb, st); \
    if (mode == 0 && res) return launch_dwpw3<NN, 0, true>(P, wh, wl, cin_pad, dww, dwb, st);   \
    if (mode == 1 && !res) return launch_dwpw3<NN, 1, false>(P, wh, wl, cin_pad, dww, dwb, st); \
    return launch_dwpw3<NN, 1, true>(P, wh, wl, cin_pad, dww, dwb, st);                          \
  }
  D3_RUN(192) D3_RUN(160) D3_RUN(128) D3_RUN(96)
#undef D3_RUN
}

// The fused depthwise + pointwise form for Cin = Cout: $MLIC_DWPW2 / mlic_set_kernel_option("dwpw2"):
//   2 (default) this register-row kernel (8 x 192 x 544 x 960 bias / GELU / GELU + residual 1.85 / 2.01 /
//     2.15 ms against dwpw_kernel's 2.31 / 2.45 / 2.98, profiles/r05/ab/dwpw3_ab.log);
//   0 dwpw_kernel (conv_dwpw.hip, rounds 3-4: one wave per SIMD, the same bits);
//   1 the row-pipelined LDS form dwpw2_kernel -- an A/B-only family since round 6 (ab/conv_dwpw2.hip,
//     linked by make AB=1 only: its masked-residual builds gave intermittent wrong rows).
static int g_dwpw2 = -1;
void dwpw2_set(int on) { g_dwpw2 = on; }
static int d2_form() {
  static const int env = [] {
    const char* e = std::getenv("MLIC_DWPW2");
    return e ? std::atoi(e) : 2;
  }();
  return g_dwpw2 < 0 ? env : g_dwpw2;
}
bool dwpw2_ok(const ConvParams& P, int cin_pad) {
  const int f = d2_form();
  if (f == 2) return dwpw3_shape_ok(P, cin_pad);
  if (f == 1) return dwpw2_lds_ok(P, cin_pad);
  return false;
}
void dwpw2_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                   const float* dwb, hipStream_t st) {
  if (d2_form() == 2) return dwpw3_forward(P, wh, wl, cin_pad, dww, dwb, st);
  dwpw2_lds_forward(P, wh, wl, cin_pad, dww, dwb, st);
}

// the pointwise form (PW) for the full-resolution 1x1 convs with Cin = Cout (pw_resident's MODE 0 - 3: bias,
// GELU, GDN, IGDN, with or without residual).  $MLIC_PW3 / mlic_set_kernel_option("pw3"): 0 off, 1 (default)
// from 256 K px per image (at 272 x 480 pw_resident measured faster: 0.45 vs 0.48 ms GELU, 0.64 vs 0.66 GDN;
// at 544 x 960 pw3's GDN / IGDN 2.07 vs 2.30), 2 at every grid (tests)
static int g_pw3 = -1;
void pw3_set(int on) { g_pw3 = on; }
static int pw3_setting() {
  static const int env = [] {
    const char* e = std::getenv("MLIC_PW3");
    return e ? std::atoi(e) : 1;
  }();
  return g_pw3 < 0 ? env : g_pw3;
}
static int pw3_mode(const ConvParams& P) {
  const int e = P.epi & ~EPI_RES;
  if (e == EPI_NONE) return 0;
  if (e == EPI_GELU) return 1;
  if (e == (EPI_GDN | EPI_SQUARE_IN)) return 2;
  if (e == (EPI_IGDN | EPI_SQUARE_IN)) return 3;
  return -1;
}
bool pw3_ok(const ConvParams& P, int cin_pad) {
  const int mode = pw3_mode(P), setting = pw3_setting();
  if (setting == 0 || mode < 0 || (mode >= 2 && !P.aux)) return false;
  if (setting == 1 && (int64_t)P.H * P.W < 262144) return false;
  if (P.K != 1 || P.stride != 1 || P.pad != 0 || P.nseg != 1 || P.seg[0].C != P.Cin || cin_pad < P.Cin) return false;
  if (P.Cin != P.Cout || (P.Cin != 96 && P.Cin != 128 && P.Cin != 160 && P.Cin != 192)) return false;
  if (P.Ho != P.H || P.Wo != P.W || P.out_cs != (int64_t)P.H * P.W) return false;
  if ((int64_t)P.Cin * P.H * P.W * 4 >= (1ll << 31)) return false;
  return true;
}
template <int N, int M, bool RS>
static void launch_pw3(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  const int R = d3_rows(P.B, P.H, P.W);
  const int64_t want = (int64_t)((P.W + D3_TC - 1) / D3_TC) * ((P.H + R - 1) / R) * P.B;
  const int64_t g = std::min<int64_t>(want, (int64_t)d3_num_cus());
  const dim3 grid((unsigned)((g + 7) / 8 * 8));
  hipLaunchKernelGGL((dwpw3_kernel<N, M, RS, true>), grid, dim3(N / 16 * 64), 0, st, P, R, wh, wl, cin_pad,
                     (const float*)nullptr, (const float*)nullptr);
  HIP_OK(hipGetLastError());
}
void pw3_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  MLIC_CHECK(pw3_ok(P, cin_pad), "pw3: unsupported shape");
  const int mode = pw3_mode(P), res = (P.epi & EPI_RES) ? 1 : 0;
#define P3_RUN(NN)                                                                \
  if (P.Cin == NN) {                                                              \
    if (mode == 0 && !res) return launch_pw3<NN, 0, false>(P, wh, wl, cin_pad, st); \
    if (mode == 0 && res) return launch_pw3<NN, 0, true>(P, wh, wl, cin_pad, st);   \
    if (mode == 1 && !res) return launch_pw3<NN, 1, false>(P, wh, wl, cin_pad, st); \
    if (mode == 1 && res) return launch_pw3<NN, 1, true>(P, wh, wl, cin_pad, st);   \
    if (mode == 2 && !res) return launch_pw3<NN, 2, false>(P, wh, wl, cin_pad, st); \
    if (mode == 2 && res) return launch_pw3<NN, 2, true>(P, wh, wl, cin_pad, st);   \
    if (mode == 3 && !res) return launch_pw3<NN, 3, false>(P, wh, wl, cin_pad, st); \
    return launch_pw3<NN, 3, true>(P, wh, wl, cin_pad, st);                          \
  }
  P3_RUN(192) P3_RUN(160) P3_RUN(128) P3_RUN(96)
#undef P3_RUN
}

}  // namespace mlic
