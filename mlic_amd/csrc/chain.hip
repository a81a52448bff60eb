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
//     K permutation, so bias + GELU + the hi/lo split happen in registers and nothing is staged;
//   * weights stream through LDS: one K-step = 32 input channels x all output rows of the layer,
//     pre-packed on the host side into the exact LDS image (128-byte rows: hi of 32 k | lo of 32 k,
//     16-byte granule G of row n at G ^ ((n >> 1) & 7): conflict-free ds_read_b128 fragments), moved
//     by global_load_lds_dwordx4 (LDS-DMA) into a 3-slot ring, two steps ahead;
//   * layer 0's input (fp32 NCHW, a multi-segment channel concat) is loaded by each lane straight into
//     its B-fragment registers, three K-steps ahead (HBM latency), and split in registers;
//   * the K-step sequence of all layers is one pipeline: one counted `s_waitcnt vmcnt` (weights of
//     this step landed; the younger input loads and weight DMAs stay in flight) and one raw s_barrier
//     per step.
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <type_traits>

namespace mlic {

namespace {
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int CH_T = 256;      // threads (4 waves)
constexpr int CH_BN = 128;     // pixels per workgroup

__device__ __forceinline__ int chswz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void chain_glds(const void* src, const void* lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)lds));
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(l) : "m0");
}

__device__ __forceinline__ half8 chain_frag(const char* base, int row, int granule) {
  return *reinterpret_cast<const half8*>(base + row * 128 + ((granule ^ chswz(row)) << 4));
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (over-waits for n outside the cases)
__device__ __forceinline__ void chain_wait(int n) {
  switch (n) {
#define MLIC_CW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MLIC_CW(1) MLIC_CW(2) MLIC_CW(3) MLIC_CW(4) MLIC_CW(5) MLIC_CW(6) MLIC_CW(7) MLIC_CW(8) MLIC_CW(9)
    MLIC_CW(10) MLIC_CW(11) MLIC_CW(12) MLIC_CW(13) MLIC_CW(14) MLIC_CW(15) MLIC_CW(16)
#undef MLIC_CW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void split8(const float (&v)[8], half8& h, half8& l, bool& bad) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bad |= f16_unsafe(v[e]);
    const _Float16 hv = (_Float16)v[e];
    h[e] = hv;
    l[e] = (_Float16)(v[e] - (float)hv);
  }
}
}  // namespace

template <int C1, int C2, int C3, int C4>
__global__ __launch_bounds__(CH_T) void chain_kernel(ChainParams P) {
  constexpr int NL = C4 ? 4 : (C3 ? 3 : 2);
  constexpr int CMAX = C1;  // layer 0 is the widest (checked by the host side)
  constexpr int WSLOT = CMAX * 128;
  constexpr int B_OFF = 3 * WSLOT;
  constexpr int NB = C1 + C2 + C3 + C4;
  static_assert(C1 % 32 == 0 && C2 % 16 == 0 && (C3 == 0 || C3 % 16 == 0) && (C4 == 0 || C4 % 16 == 0), "dims");
  static_assert(B_OFF + NB * 4 <= 160 * 1024, "chain LDS");
  static_assert(NL == 2 || C2 % 32 == 0, "inner layers feed whole K chunks");
  __shared__ __attribute__((aligned(1024))) char sm[B_OFF + NB * 4];
  float* sbias = reinterpret_cast<float*>(sm + B_OFF);

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int G = lane >> 4, l16 = lane & 15;
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * CH_BN;
  const int HW = P.HW;
  const int S0 = P.cin0 / 32;
  constexpr int S1 = C1 / 32, S2 = C2 / 32, S3 = C3 / 32;
  const int T = S0 + S1 + (NL > 2 ? S2 : 0) + (NL > 3 ? S3 : 0);

  // biases to LDS (before any DMA: the loop below must see no compiler-visible global load)
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

  // weight DMA: step w_next -> slot w_next % 3; each wave moves rows/32 KB-sized pieces
  int w_next = 0;
  int64_t w_off = 0;  // halves
  auto issue_w = [&]() {
    const int R = rows_of(w_next);
    const int n = R / 32;
    char* dst = sm + (w_next % 3) * WSLOT;
    const _Float16* src = P.wimg + w_off + lane * 8;
    for (int i = 0; i < n; ++i) {
      const int ci = wv * n + i;
      chain_glds(src + (int64_t)ci * 512, dst + ci * 1024);
    }
    w_off += (int64_t)R * 64;
    ++w_next;
  };
  // layer-0 input: prefetched into registers 3 K-steps ahead (a 3-deep register ring, the loop below
  // is unrolled by 3 so the ring index is static).  Lane (G, l16) loads exactly its B fragments:
  // channels 32t + 8G .. +7 at pixels p0 + 32 wv + 16 j + l16 (16 dword loads; the 32 channels of a
  // K-step lie in one input segment, segments being multiples of 32).  These loads are compiler-
  // visible: the compiler's own vmcnt for them only over-waits (it does not see the DMAs), and the
  // explicit per-step wait below counts them (NF per step).
  constexpr int NF = 16;
  auto load_f = [&](int t, float (&f)[2][8]) {
    if (t >= S0) return;
    const int ch = 32 * t;
    int s = 0, c0 = 0;
    while (s + 1 < P.nseg && ch >= c0 + P.seg[s].C) { c0 += P.seg[s].C; ++s; }
    const float* src = P.seg[s].p + (int64_t)b * P.seg[s].bs + (int64_t)(ch - c0 + 8 * G) * HW;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int px = min(p0 + 32 * wv + 16 * j + l16, HW - 1);  // ragged last tile: outputs dropped
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) f[j][kk] = src[(int64_t)kk * HW + px];
    }
  };
  auto nf_of = [&](int t) { return t < S0 ? NF : 0; };
  // at the top of step u only W(u) must have landed; issued after it: F(u+1), W(u+1), F(u+2)
  auto step_begin = [&](int t) {
    chain_wait(nf_of(t + 1) + rows_of(t + 1) / 32 + nf_of(t + 2));
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 2 < T) issue_w();
  };

  auto mfma3 = [](floatx4& acc, const half8& ah, const half8& al, const half8& bh, const half8& bl) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
  };
  // one K-step of COUT rows against B operands in registers; the A fragments of row block i + 1 are
  // read while block i's MFMAs issue
  auto kstep = [&](auto& acc, const char* As, const half8 (&bh)[2], const half8 (&bl)[2], auto cout_c) {
    constexpr int COUT = decltype(cout_c)::value;
    half8 ah[2], al[2];
    ah[0] = chain_frag(As, l16, G);
    al[0] = chain_frag(As, l16, G + 4);
#pragma unroll
    for (int i = 0; i < COUT / 16; ++i) {
      if (i + 1 < COUT / 16) {
        ah[(i + 1) & 1] = chain_frag(As, 16 * (i + 1) + l16, G);
        al[(i + 1) & 1] = chain_frag(As, 16 * (i + 1) + l16, G + 4);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) mfma3(acc[i][j], ah[i & 1], al[i & 1], bh[j], bl[j]);
    }
  };

  bool bad = false;  // fp16 range guard (common.h)
  // prologue, issued in the per-step order (step u issues W(u+2), then F(u+3)): F(0) W(0) F(1) W(1) F(2)
  float fr[3][2][8];
  load_f(0, fr[0]);
  issue_w();
  load_f(1, fr[1]);
  if (T > 1) issue_w();
  load_f(2, fr[2]);

  // ------------------------------------------------------------------ layer 0 (input prefetched)
  floatx4 acc0[C1 / 16][2];
  if (P.aux) {
    // the hoisted part of layer 0 (EntropyParameters' hyper columns, one wide GEMM per image) starts
    // the accumulators, in the prescaled domain of this layer's weights (exact)
    const float* ax = P.aux + (int64_t)b * P.aux_bs;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int px = min(p0 + 32 * wv + 16 * j + l16, HW - 1);
#pragma unroll
      for (int i = 0; i < C1 / 16; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc0[i][j][e] = ldexpf(ax[(int64_t)(16 * i + 4 * G + e) * HW + px], P.wexp[0]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < C1 / 16; ++i)
      for (int j = 0; j < 2; ++j) acc0[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  auto step0 = [&](int t, float (&f)[2][8]) {
    if (t >= S0) return;
    step_begin(t);
    half8 bh[2], bl[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) split8(f[j], bh[j], bl[j], bad);
    load_f(t + 3, f);  // the ring slot is free once split
    kstep(acc0, sm + (t % 3) * WSLOT, bh, bl, std::integral_constant<int, C1>{});
  };
  for (int t = 0; t < S0; t += 3) {
    step0(t, fr[0]);
    step0(t + 1, fr[1]);
    step0(t + 2, fr[2]);
  }

  using I1 = std::integral_constant<int, S1>;
  using I2 = std::integral_constant<int, S2>;
  using I3 = std::integral_constant<int, S3>;
  // accumulators of a layer -> the next layer's B operands (bias + GELU + split, in registers)
  auto to_operands = [&](auto& acc, half8 (*oh)[2], half8 (*ol)[2], auto nch_c, int boff, bool gelu, int wexp) {
    constexpr int NCH = decltype(nch_c)::value;
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = boff + 32 * c + 16 * q + 4 * G + e;
            float x = ldexpf(acc[2 * c + q][j][e], -wexp) + sbias[r];
            v[4 * q + e] = gelu ? gelu_erf(x) : x;
          }
        split8(v, oh[c][j], ol[c][j], bad);
      }
  };

  // one layer fed from registers: NCH K-chunks, COUT rows, steps t0 .. t0 + NCH - 1
  auto layer_regs = [&](auto& acc, half8 (*bh)[2], half8 (*bl)[2], auto nch_c, auto cout_c, int t0) {
    constexpr int NCH = decltype(nch_c)::value, COUT = decltype(cout_c)::value;
#pragma unroll
    for (int i = 0; i < COUT / 16; ++i)
      for (int j = 0; j < 2; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int t = t0 + c;
      step_begin(t);
      const half8 b_h[2] = {bh[c][0], bh[c][1]}, b_l[2] = {bl[c][0], bl[c][1]};
      kstep(acc, sm + (t % 3) * WSLOT, b_h, b_l, cout_c);
    }
  };
  // the output of the last layer: bias (+ residual), fp32 NCHW store
  auto store = [&](auto& acc, auto cout_c, int boff, int wexp) {
    constexpr int COUT = decltype(cout_c)::value;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    range_report(P.rflag, bad);
#pragma unroll
    for (int i = 0; i < COUT / 16; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int px = p0 + 32 * wv + 16 * j + l16;
        if (px >= HW) continue;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 16 * i + 4 * G + e;
          float v = ldexpf(acc[i][j][e], -wexp) + sbias[boff + co];
          if (P.res) v += P.res[(int64_t)b * P.res_bs + (int64_t)co * HW + px];
          P.out[(int64_t)b * P.out_bs + (int64_t)co * HW + px] = v;
        }
      }
  };

  half8 b1h[C1 / 32][2], b1l[C1 / 32][2];
  to_operands(acc0, b1h, b1l, I1{}, 0, (P.gelu_mask & 1) != 0, P.wexp[0]);
  floatx4 acc1[C2 / 16][2];
  layer_regs(acc1, b1h, b1l, I1{}, std::integral_constant<int, C2>{}, S0);
  if constexpr (NL == 2) {
    store(acc1, std::integral_constant<int, C2>{}, C1, P.wexp[1]);
  } else {
    half8 b2h[C2 / 32 > 0 ? C2 / 32 : 1][2], b2l[C2 / 32 > 0 ? C2 / 32 : 1][2];
    to_operands(acc1, b2h, b2l, I2{}, C1, (P.gelu_mask & 2) != 0, P.wexp[1]);
    floatx4 acc2[C3 / 16][2];
    layer_regs(acc2, b2h, b2l, I2{}, std::integral_constant<int, C3>{}, S0 + S1);
    if constexpr (NL == 3) {
      store(acc2, std::integral_constant<int, C3>{}, C1 + C2, P.wexp[2]);
    } else {
      half8 b3h[C3 / 32][2], b3l[C3 / 32][2];
      to_operands(acc2, b3h, b3l, I3{}, C1 + C2, (P.gelu_mask & 4) != 0, P.wexp[2]);
      floatx4 acc3[C4 / 16][2];
      layer_regs(acc3, b3h, b3l, I3{}, std::integral_constant<int, C4>{}, S0 + S1 + S2);
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

void chain_forward(const ChainParams& P, int nl, const int* cout, hipStream_t st) {
  MLIC_CHECK(chain_supported(nl, cout), "chain: unsupported layer widths");
  MLIC_CHECK(P.cin0 % 32 == 0 && (P.cin0 > 0 || P.aux) && P.HW % 4 == 0 && P.HW >= 4,
             "chain: Cin multiple of 32 (or 0 with aux), HW of 4");
  dim3 grid((P.HW + CH_BN - 1) / CH_BN, P.B);
  if (nl == 4 && cout[3] == 64)
    hipLaunchKernelGGL((chain_kernel<320, 256, 128, 64>), grid, dim3(CH_T), 0, st, P);
  else if (nl == 4)
    hipLaunchKernelGGL((chain_kernel<320, 256, 128, 128>), grid, dim3(CH_T), 0, st, P);
  else
    hipLaunchKernelGGL((chain_kernel<128, 64, 0, 0>), grid, dim3(CH_T), 0, st, P);
  HIP_OK(hipGetLastError());
}

}  // namespace mlic
