// Fused 1x1-conv chain ("chain"): 2-4 pointwise layers with bias + GELU between them in ONE kernel,
// the intermediates never leaving the chip.  Serves EntropyParameters (modules/transform/entropy.py:
// 7-29: in -> 320 -> 256 -> 128 -> 2 C, GELU between; called per slice and phase at
// models/mlicpp.py:111,124,146,160) and LocalContext's MLP (context.py:108-110 fc1 -> GELU -> fc2 + x).
//
// Arithmetic: split-fp16 as conv_f16x3.hip (v = hi + lo + r, a.b = lo_a.hi_b + hi_a.lo_b + hi_a.hi_b
// with fp32 accumulation) on v_mfma_f32_16x16x32_f16.
//
// Mapping (gfx950, one 256-thread workgroup per CU, 128 pixels per workgroup):
//   * each wave owns 32 pixels (two 16-column MFMA blocks) and EVERY output row of every layer, so a
//     layer's accumulators are, lane for lane, the next layer's B operand: the 16x16 C/D block holds
//     rows 4*(lane>>4)+e of column lane&15, and two such blocks (rows 32c+{0..15} and 32c+{16..31})
//     give lane group G = lane>>4 the 8 k-slots 8G..8G+7 of K-chunk c under the fixed permutation
//     slot s -> row 16*((s>>2)&1) + 4*(s>>3) + (s&3).  The next layer's weights are packed with that
//     K permutation, so bias + GELU + the hi/lo split happen in registers and nothing is staged; the
//     operands of K-chunk c + 1 are made while chunk c's MFMAs run (program-order interleave);
//   * weights: one K-step = 32 input channels x all output rows of the layer, pre-packed on the host
//     side into the exact LDS image (128-byte rows: hi of 32 k | lo of 32 k, 16-byte granule G of row
//     n at G ^ ((n >> 1) & 7): conflict-free ds_read_b128 fragments).  Staged through registers
//     (global_load_dwordx4, 1 KB per wave-instruction, L2-resident) one step ahead and stored with
//     ds_write_b128 into a 2-slot LDS ring: measured far cheaper to issue next to the MFMA/ds_read
//     stream than LDS-DMA pieces (tools/gpu/chain_probe.hip);
//   * layer 0's input (fp32 NCHW, a multi-segment channel concat) is loaded by each lane straight into
//     its B-fragment registers two K-steps ahead (a 2-deep register ring) and split in registers;
//   * one s_barrier per K-step; every global load is compiler-visible (its vmcnt is the compiler's).
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

#ifndef MLIC_CH_PK  // chain layer transitions: 1 = packed-fp32 bias + GELU of value pairs, 0 = scalar
#define MLIC_CH_PK 1
#endif

namespace mlic {

namespace {
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int CH_BN = 128;     // pixels per workgroup
// NJ = 16-pixel column blocks per wave: 2 = four waves of 32 pixels (one wave per SIMD, 512-register
// waves: rounds 2-5), 1 = eight waves of 16 pixels (two waves per SIMD, <= 256 registers each: one wave's
// bias / GELU / split VALU work runs beside the other's MFMAs instead of in its own MFMA shadow only)
template <int NJ>
constexpr int ch_threads() { return 64 * (8 / NJ); }

__device__ __forceinline__ int chswz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ half8 chain_frag(const char* base, int row, int granule) {
  return *reinterpret_cast<const half8*>(base + row * 128 + ((granule ^ chswz(row)) << 4));
}

// hi/lo split of 8 values.  The fp16 range guard needs no check here: a value with |v| >= 65520 splits
// to hi = +-inf (lo = -+inf or NaN), which makes every accumulator it reaches inf / NaN; GELU maps
// inf to NaN, NaN propagates through every later layer's split and MFMAs, and the output store
// checks that the chain's outputs are finite (one compare per output instead of a max per input)
__device__ __forceinline__ void split8(const float (&v)[8], half8& h, half8& l) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const _Float16 hv = (_Float16)v[e];
    h[e] = hv;
    l[e] = (_Float16)(v[e] - (float)hv);
  }
}
}  // namespace

#ifdef MLIC_CHAIN_TRACE
// step timestamps of two workgroups (tools/gpu/chain_probe.hip): [wg][wave][step][3] shader clocks
__device__ unsigned long long* g_chain_trace;
constexpr int CH_TR_STEPS = 64;
#endif

template <int C1, int C2, int C3, int C4, int NJ>
__global__ __launch_bounds__(ch_threads<NJ>()) void chain_kernel(ChainParams P) {
  constexpr int CH_T = ch_threads<NJ>(), NW = CH_T / 64, PW = 16 * NJ;  // threads, waves, pixels per wave
  constexpr int NL = C4 ? 4 : (C3 ? 3 : 2);
  constexpr int WSLOT = C1 * 128;  // layer 0 is the widest (checked by the host side)
  constexpr int B_OFF = 2 * WSLOT;
  constexpr int NB = C1 + C2 + C3 + C4;
  constexpr int WMAX = C1 / 32 * 4 / NW;  // 1-KB weight pieces per wave of the widest step
  static_assert(C1 % 32 == 0 && C2 % 32 == 0 && (C3 == 0 || C3 % 32 == 0) && (C4 == 0 || C4 % 16 == 0), "dims");
  static_assert(NJ == 2 || (C1 % 64 == 0 && C2 % 64 == 0 && C3 % 64 == 0 && C4 % 64 == 0), "8 waves: rows / 64 pieces");
  static_assert(C2 <= C1 && C3 <= C1 && C4 <= C1, "layer 0 is the widest");
  static_assert(B_OFF + NB * 4 <= 160 * 1024, "chain LDS");
  __shared__ __attribute__((aligned(1024))) char sm[B_OFF + NB * 4];
  float* sbias = reinterpret_cast<float*>(sm + B_OFF);
#ifdef MLIC_CHAIN_TRACE
  __shared__ unsigned long long str[NW][CH_TR_STEPS][3];
  const int tr_wg = (blockIdx.x == 0 && blockIdx.y == 0) ? 0
                    : (blockIdx.x == gridDim.x - 2 && blockIdx.y == gridDim.y - 1) ? 1 : -1;
#define CH_TR(t, k) \
  if (tr_wg >= 0 && (t) < CH_TR_STEPS) str[threadIdx.x >> 6][t][k] = __builtin_readcyclecounter()
#else
#define CH_TR(t, k)
#endif

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = lane >> 4, l16 = lane & 15;
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * CH_BN;
  const int HW = P.HW;
  const int NQ = P.ckbd ? HW >> 1 : HW;  // pixels of this launch (the phase's half under ckbd)
  // plane offset of the launch's pixel q (clamped: a ragged last tile loads the last pixel, stores nothing)
  auto px_of = [&](int q) {
    q = min(q, NQ - 1);
    if (!P.ckbd) return q;
    const int w2 = P.W >> 1, y = q / w2, x = 2 * (q - y * w2) + ((y + (P.ckbd == 1 ? 1 : 0)) & 1);
    return y * P.W + x;
  };
  // the lane's pixels, one per 16-pixel column block: in the input / residual / aux planes (squeezed
  // planes of NQ pixels under sq_in) and in the output planes
  const int HWi = P.sq_in ? NQ : HW;
  int pxj[NJ], pxo[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int q = p0 + PW * wv + 16 * j + l16;
    pxo[j] = px_of(q);
    pxj[j] = P.sq_in ? min(q, NQ - 1) : pxo[j];
  }
  const int S0 = P.cin0 / 32;
  constexpr int S1 = C1 / 32, S2 = C2 / 32, S3 = C3 / 32;
  const int T = S0 + S1 + (NL > 2 ? S2 : 0) + (NL > 3 ? S3 : 0);

  {
    constexpr int CS[4] = {C1, C2, C3, C4};
    int off = 0;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      for (int i = tid; i < CS[l]; i += CH_T) sbias[off + i] = P.bias[l] ? P.bias[l][i] : 0.0f;
      off += CS[l];
    }
  }
  __syncthreads();

  // rows (output channels) of the layer that K-step t belongs to; 0 past the end
  auto rows_of = [&](int t) -> int {
    if (t >= T) return 0;
    if (t < S0) return C1;
    t -= S0;
    if (t < S1) return C2;
    t -= S1;
    if (NL > 2 && t < S2) return C3;
    return C4;
  };

  // weights of step u: wave wv moves 1-KB pieces wv*n .. wv*n + n - 1 (n = rows / 32 / (NW / 4)) through wr
  u32x4 wr[WMAX];
  int64_t w_off = 0;  // halves: the image of the next step to load
  auto wload = [&](int u) {
    const int R = rows_of(u), n = R / 32 * 4 / NW;
    const _Float16* src = P.wimg + w_off + (int64_t)(wv * n) * 512 + lane * 8;
#pragma unroll
    for (int i = 0; i < WMAX; ++i)
      if (i < n) wr[i] = *reinterpret_cast<const u32x4*>(src + i * 512);
    w_off += (int64_t)R * 64;
  };
  auto wstore = [&](int u) {
    const int n = rows_of(u) / 32 * 4 / NW;
    char* dst = sm + (u & 1) * WSLOT + (wv * n) * 1024 + lane * 16;
#pragma unroll
    for (int i = 0; i < WMAX; ++i)
      if (i < n) *reinterpret_cast<u32x4*>(dst + i * 1024) = wr[i];
  };
  // top of step t: this wave's stores of W(t) done, then the barrier (W(t) visible to all waves; slot
  // (t + 1) & 1, read in step t - 1, free); then W(t + 1) registers -> LDS and W(t + 2) -> registers
  auto step_begin = [&](int t) {
    CH_TR(t, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    CH_TR(t, 1);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    CH_TR(t, 2);
    if (t + 1 < T) wstore(t + 1);
    if (t + 2 < T) wload(t + 2);
  };

  // layer-0 input, 2 K-steps ahead in registers: lane (G, l16) loads exactly its B fragments,
  // channels 32t + 8G .. +7 at pixels p0 + PW wv + 16 j + l16 (8 NJ dword loads; the 32 channels of a
  // K-step lie in one input segment, segments being multiples of 32).  Every L0 step issues its
  // loads (the last two re-load chunk S0 - 1), so the ring's vmcnt stays a plain count.
  auto load_f = [&](int t, float (&f)[NJ][8]) {
    t = min(t, S0 - 1);
    const int ch = 32 * t;
    int s = 0, c0 = 0;
    while (s + 1 < P.nseg && ch >= c0 + P.seg[s].C) { c0 += P.seg[s].C; ++s; }
    const float* src = P.seg[s].p + (int64_t)b * P.seg[s].bs + (int64_t)(ch - c0 + 8 * G) * HWi;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) f[j][kk] = src[(int64_t)kk * HWi + pxj[j]];
    }
  };

  auto mfma3 = [](floatx4& acc, const half8& ah, const half8& al, const half8& bh, const half8& bl) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
  };
  // one K-step of COUT rows against B operands in registers; the A fragments of row block i + 2 are
  // read while block i's MFMAs issue (12 MFMAs of cover for the LDS latency); hook(i) runs after
  // block i's MFMAs (program-order interleave of independent VALU work)
  auto kstep = [&](auto& acc, const char* As, const half8 (&bh)[NJ], const half8 (&bl)[NJ], auto cout_c, auto&& hook) {
    constexpr int COUT = decltype(cout_c)::value, NBK = COUT / 16, D = 2, R = D + 1;
    half8 ah[R], al[R];
#pragma unroll
    for (int i = 0; i < D && i < NBK; ++i) {
      ah[i] = chain_frag(As, 16 * i + l16, G);
      al[i] = chain_frag(As, 16 * i + l16, G + 4);
    }
#pragma unroll
    for (int i = 0; i < NBK; ++i) {
      if (i + D < NBK) {
        ah[(i + D) % R] = chain_frag(As, 16 * (i + D) + l16, G);
        al[(i + D) % R] = chain_frag(As, 16 * (i + D) + l16, G + 4);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) mfma3(acc[i][j], ah[i % R], al[i % R], bh[j], bl[j]);
      hook(i);
    }
  };
  auto no_hook = [](int) {};

  int bad = 0;  // fp16 range guard (common.h)
  // ------------------------------------------------------------------ layer 0 (input prefetched)
  floatx4 acc0[C1 / 16][NJ];
  if (P.aux) {
    // the hoisted part of layer 0 (EntropyParameters' hyper columns, one wide GEMM per image) starts
    // the accumulators, in the prescaled domain of this layer's weights (exact)
    const float* ax = P.aux + (int64_t)b * P.aux_bs;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int px = pxj[j];
#pragma unroll
      for (int i = 0; i < C1 / 16; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc0[i][j][e] = ldexpf(ax[(int64_t)(16 * i + 4 * G + e) * HWi + px], P.wexp[0]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < C1 / 16; ++i)
      for (int j = 0; j < NJ; ++j) acc0[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  auto step0 = [&](int t, float (&f)[NJ][8]) {
    step_begin(t);
    half8 bh[NJ], bl[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) split8(f[j], bh[j], bl[j]);
    // keep the reload of f below its last use, so the ring slot stays in the same registers (an
    // overlap would make the register allocator rotate the ring with copies that wait for the loads)
    __builtin_amdgcn_sched_barrier(0);
    load_f(t + 2, f);
    kstep(acc0, sm + (t & 1) * WSLOT, bh, bl, std::integral_constant<int, C1>{}, no_hook);
  };
  // prologue: W(0) -> LDS, W(1) -> registers, F(0), F(1); then the L0 steps as a do-while (S0 even),
  // so the 2-deep input ring has a single entry path and stays in place across iterations
  wload(0);
  wstore(0);
  if (T > 1) wload(1);
  if (S0 > 0) {
    float fa[NJ][8], fb[NJ][8];
    load_f(0, fa);
    load_f(1, fb);
    int t = 0;
    do {
      step0(t, fa);
      step0(t + 1, fb);
      t += 2;
    } while (t < S0);
  }

  using I1 = std::integral_constant<int, S1>;
  using I2 = std::integral_constant<int, S2>;
  using I3 = std::integral_constant<int, S3>;
  // K-chunk c of a layer's accumulators -> the next layer's B operands (bias + GELU + split, in
  // registers; 2^-wexp is exact, so the fma equals ldexp + add), one value pair at a time: pair pi =
  // (j = pi >> 2, q = (pi >> 1) & 1, e = 2 (pi & 1)); the split of column block j follows its 4th pair
  auto chunk_pair = [&](auto& acc, int c, int pi, float (&v)[NJ][8], half8 (&oh)[NJ], half8 (&ol)[NJ], int boff,
                        float unscale) {
    const int j = pi >> 2, q = (pi >> 1) & 1, e = 2 * (pi & 1);
    const float* bq = sbias + boff + 32 * c + 16 * q + 4 * G + e;
#if MLIC_CH_PK
    // the pair through the packed GELU (gelu_erf2 == gelu_erf element for element) and one packed fma
    const mlic_float2 a2 = __builtin_elementwise_fma(mlic_float2{acc[2 * c + q][j][e], acc[2 * c + q][j][e + 1]},
                                                     mlic_float2{unscale, unscale}, mlic_float2{bq[0], bq[1]});
    const mlic_float2 g2 = gelu_erf2(a2);
    v[j][4 * q + e] = g2.x;
    v[j][4 * q + e + 1] = g2.y;
#else
    // scalar VALU beside the MFMAs (packed fp32 there costs more than its scalar pair: MI355X_MICROARCH)
    v[j][4 * q + e] = gelu_erf(__builtin_fmaf(acc[2 * c + q][j][e], unscale, bq[0]));
    v[j][4 * q + e + 1] = gelu_erf(__builtin_fmaf(acc[2 * c + q][j][e + 1], unscale, bq[1]));
#endif
    if ((pi & 3) == 3) split8(v[j], oh[j], ol[j]);
  };

  // one layer fed from the previous layer's accumulators: NCH K-chunks, COUT rows, steps t0 .. t0 +
  // NCH - 1.  Chunk c + 1's operands are made during step c, spread over its MFMA blocks (VALU work
  // independent of those MFMAs); chunk 0's before the first step.
  auto layer_regs = [&](auto& acc, auto& prev, auto nch_c, auto cout_c, int t0, int boff, int wexp) {
    constexpr int NCH = decltype(nch_c)::value, COUT = decltype(cout_c)::value, NBK = COUT / 16;
    constexpr int NP = 4 * NJ;  // value pairs of a K-chunk per lane
    constexpr int PER = NBK >= NP ? NBK / NP : 1, PPB = NBK >= NP ? 1 : NP / NBK;  // blocks per pair, pairs per block
    const float unscale = ldexpf(1.0f, -wexp);
#pragma unroll
    for (int i = 0; i < COUT / 16; ++i)
      for (int j = 0; j < NJ; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    half8 nh[NJ], nl[NJ];
    float v[NJ][8];
#pragma unroll
    for (int pi = 0; pi < NP; ++pi) chunk_pair(prev, 0, pi, v, nh, nl, boff, unscale);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int t = t0 + c;
      step_begin(t);
      half8 b_h[NJ], b_l[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        b_h[j] = nh[j];
        b_l[j] = nl[j];
      }
      kstep(acc, sm + (t & 1) * WSLOT, b_h, b_l, cout_c, [&](int i) {
        if (c + 1 < NCH && i % PER == 0)
#pragma unroll
          for (int k = 0; k < PPB; ++k) chunk_pair(prev, c + 1, (i / PER) * PPB + k, v, nh, nl, boff, unscale);
      });
    }
  };
  // the output of the last layer: bias (+ residual), fp32 NCHW store
  auto store = [&](auto& acc, auto cout_c, int boff, int wexp) {
    constexpr int COUT = decltype(cout_c)::value;
#ifdef MLIC_CHAIN_TRACE
    if (tr_wg >= 0 && lane == 0) {
      CH_TR(T < CH_TR_STEPS ? T : CH_TR_STEPS - 1, 0);
      for (int i = 0; i < CH_TR_STEPS * 3; ++i)
        g_chain_trace[((int64_t)tr_wg * 4 + wv) * CH_TR_STEPS * 3 + i] = (&str[wv][0][0])[i];
    }
#endif
    const float unscale = ldexpf(1.0f, -wexp);
#pragma unroll
    for (int i = 0; i < COUT / 16; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (p0 + PW * wv + 16 * j + l16 >= NQ) continue;
        const int px = pxo[j], pxi = pxj[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 16 * i + 4 * G + e;
          float v = __builtin_fmaf(acc[i][j][e], unscale, sbias[boff + co]);
          bad |= !(__builtin_fabsf(v) <= 3.4e38f) ? 1 : 0;
          if (P.res) v += P.res[(int64_t)b * P.res_bs + (int64_t)co * HWi + pxi];
          P.out[(int64_t)b * P.out_bs + (int64_t)co * HW + px] = v;
        }
      }
    range_report(P.rflag, bad != 0);
  };

  floatx4 acc1[C2 / 16][NJ];
  layer_regs(acc1, acc0, I1{}, std::integral_constant<int, C2>{}, S0, 0, P.wexp[0]);
  if constexpr (NL == 2) {
    store(acc1, std::integral_constant<int, C2>{}, C1, P.wexp[1]);
  } else {
    floatx4 acc2[C3 / 16][NJ];
    layer_regs(acc2, acc1, I2{}, std::integral_constant<int, C3>{}, S0 + S1, C1, P.wexp[1]);
    if constexpr (NL == 3) {
      store(acc2, std::integral_constant<int, C3>{}, C1 + C2, P.wexp[2]);
    } else {
      floatx4 acc3[C4 / 16][NJ];
      layer_regs(acc3, acc2, I3{}, std::integral_constant<int, C4>{}, S0 + S1 + S2, C1 + C2, P.wexp[2]);
      store(acc3, std::integral_constant<int, C4>{}, C1 + C2 + C3, P.wexp[3]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// weights: split hi/lo [Cout][cin_pad] -> [step][Cout rows][64 halves] LDS images (granule swizzle;
// permute = 1: K order of a layer fed from the previous layer's accumulators)
__global__ void chain_pack_kernel(const _Float16* __restrict__ wh, const _Float16* __restrict__ wl, int Cout, int Cin,
                                  int cin_pad, int permute, _Float16* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int e = (int)(i % 64);
  const int row = (int)((i / 64) % Cout);
  const int step = (int)(i / (64 * (int64_t)Cout));
  const int Gp = e >> 3, G = Gp ^ chswz(row);
  const int s = (G & 3) * 8 + (e & 7);  // k-slot
  const int k = permute ? 16 * ((s >> 2) & 1) + 4 * (s >> 3) + (s & 3) : s;
  const int ch = step * 32 + k;
  _Float16 v = (_Float16)0.0f;
  if (ch < Cin) v = G < 4 ? wh[(int64_t)row * cin_pad + ch] : wl[(int64_t)row * cin_pad + ch];
  dst[i] = v;
}

int64_t chain_layer_halves(int Cout, int Cin) { return (int64_t)((Cin + 31) / 32) * Cout * 64; }

void chain_pack(const _Float16* wh, const _Float16* wl, int Cout, int Cin, int cin_pad, int permute, _Float16* dst,
                hipStream_t st) {
  const int64_t n = chain_layer_halves(Cout, Cin);
  hipLaunchKernelGGL(chain_pack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, wh, wl, Cout, Cin, cin_pad,
                     permute, dst, n);
  HIP_OK(hipGetLastError());
}

bool chain_supported(int nl, const int* cout) {
  if (nl == 4) return cout[0] == 320 && cout[1] == 256 && cout[2] == 128 && (cout[3] == 64 || cout[3] == 128);
  if (nl == 2) return cout[0] == 128 && cout[1] == 64;
  return false;
}

// $MLIC_CHAIN_NJ / mlic_set_kernel_option("chain_nj"): 16-pixel column blocks per wave (1: eight waves
// of 16 pixels, 2: four waves of 32); the same MFMA order per accumulator and the same K order, so both
// give the same bits
static int g_chain_nj = -1;
void chain_set_nj(int nj) { g_chain_nj = nj; }
static int chain_nj() {
  static const int env = [] {
    const char* e = std::getenv("MLIC_CHAIN_NJ");
    return e ? std::atoi(e) : 1;
  }();
  const int v = g_chain_nj > 0 ? g_chain_nj : env;
  return v == 2 ? 2 : 1;
}

// $MLIC_EP_HALF / mlic_set_kernel_option("ep_half"): EntropyParameters' chains run on their own
// phase's checkerboard half only (ChainParams::ckbd); 0 = the whole grid (A/B, the same bits at every
// pixel a consumer reads)
static int g_ep_half = -1;
void chain_set_ep_half(int on) { g_ep_half = on; }
bool chain_ep_half() {
  static const int env = [] {
    const char* e = std::getenv("MLIC_EP_HALF");
    return e ? std::atoi(e) : 1;
  }();
  return (g_ep_half >= 0 ? g_ep_half : env) != 0;
}

template <int NJ>
static void launch_chain(const ChainParams& P, int nl, const int* cout, hipStream_t st) {
  dim3 grid(((P.ckbd ? P.HW / 2 : P.HW) + CH_BN - 1) / CH_BN, P.B);
  constexpr int T = ch_threads<NJ>();
  if (nl == 4 && cout[3] == 64)
    hipLaunchKernelGGL((chain_kernel<320, 256, 128, 64, NJ>), grid, dim3(T), 0, st, P);
  else if (nl == 4)
    hipLaunchKernelGGL((chain_kernel<320, 256, 128, 128, NJ>), grid, dim3(T), 0, st, P);
  else
    hipLaunchKernelGGL((chain_kernel<128, 64, 0, 0, NJ>), grid, dim3(T), 0, st, P);
  HIP_OK(hipGetLastError());
}

void chain_forward(const ChainParams& P, int nl, const int* cout, hipStream_t st) {
  MLIC_CHECK(chain_supported(nl, cout), "chain: unsupported layer widths");
  MLIC_CHECK(P.cin0 % 64 == 0 && (P.cin0 > 0 || P.aux) && P.HW % 4 == 0 && P.HW >= 4,
             "chain: Cin multiple of 64 (or 0 with aux), HW of 4");
  MLIC_CHECK(P.ckbd == 0 || (P.ckbd <= 2 && P.W > 0 && P.W % 2 == 0 && P.HW % P.W == 0), "chain: checkerboard half needs W even");
  MLIC_CHECK(!P.sq_in || P.ckbd, "chain: squeezed inputs need a checkerboard half");
  if (chain_nj() == 2) launch_chain<2>(P, nl, cout, st);
  else launch_chain<1>(P, nl, cout, st);
}

}  // namespace mlic
