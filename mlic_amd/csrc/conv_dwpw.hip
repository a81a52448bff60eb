// Fused depthwise-separable conv ("dwpw"): the fork's DepthWiseConv (modules/layers/conv.py:22-32 and
// 46-63: depthwise 3x3 stride 1 pad 1 + bias, then pointwise 1x1 + bias, then the block's GELU /
// residual) in ONE kernel, so the depthwise output never goes to HBM.  g_a / g_s run it on every
// stride-1 dwsep conv of their residual blocks (res_blk.py:62-154: ResidualBlock conv1 / conv2,
// ResidualBlockWithStride conv2, ResidualBlockUpsample conv): Cin = Cout = N.
//
// Barrier-free, like the resident pointwise kernel (conv_pw.hip pw_resident_kernel).  One workgroup
// of 4 waves (one per SIMD) per CU keeps, for its whole life, in LDS:
//   * the split hi/lo pointwise weights as an MFMA A-fragment image, [k-step][row][64 B] with the four
//     16-byte granules (hi k0-7 | hi k8-15 | lo k0-7 | lo k8-15) XOR-swizzled by (row >> 2) & 3:
//     conflict-free ds_read_b128 for both lane groups (no padding, so N = 192 fits beside the taps);
//   * the depthwise taps + bias, [C][12] floats, read by broadcast ds_read_b128.
// Every lane owns TWO adjacent pixels of one row: its activation loads are dwordx2 (8 B per lane per
// channel and row), and the two pixels are the columns of two v_mfma_f32_32x32x16_f16 B fragments
// (e = 0, 1: column n <-> pixel xl + e; lane half h holds channels 8h..8h+7 of a 16-deep k-step), whose
// accumulators hold, lane for lane, the same output channel of both pixels -- the epilogue stores them
// as dwordx2 too.  A wave row segment is 64 loaded columns (lane n: xl = x0 - 2 + 2n) for 60 output
// columns: lanes 0 and 31 of each lane half only supply the halo (x0 - 1 via lane 0's second pixel,
// x0 + 60 via lane 31's first) and store nothing, so the horizontal neighbours are plain DPP wave
// shifts with no edge loads (what a halo lane receives across the lane-half seam is never used); MFMA
// columns wasted: 2 of 32.  Out-of-image taps read 0 through an out-of-range buffer offset.
// The depthwise sum is dw3x3_s1_vec_kernel's order (acc = 0, taps row-major by fma, + bias), the hi /
// lo split and the MFMA k order are pw_resident's, and the epilogue is pw_resident's op sequence
// (gelu_erf2 is gelu_erf element for element): the fused output equals depthwise + resident pointwise
// bit for bit (tests/test_gpu_conv.py::test_dwpw_fused).
// Pipeline: k-step j + 1's depthwise + split runs interleaved with k-step j's MFMAs in program order,
// and refills a one-slot register ring with k-step j + 2 channel by channel; the ring and the B
// fragments carry across tiles.  The accumulators of all Cout rows (CT x 2 x 16 registers, AGPRs)
// take one wave per SIMD.  Workgroup tile = 4 rows x 60 columns (wave w: row y0 + w); tiles ordered
// (image, row block, segment) and dealt XCD-aware (the workgroups of one XCD, blockIdx % 8 under
// round-robin placement, take one contiguous eighth of them: speed only).  Needs W even (a lane's
// pixel pair is either inside the row or entirely outside it).
// HBM bytes per pixel: 4 * (Cin + Cout [+ Cout residual]) -- the pointwise conv's alone; the unfused
// pair moves 4 * (3 Cin + Cout [+ Cout]).  Measured (8 x 192 x 544 x 960, GELU): 2.42-2.49 ms against
// 2.98 ms for depthwise + resident pointwise.  Rejected: the lane-per-pixel form (b32 main + edge loads,
// 8 waves: 3.2 ms); the same kernel without its depthwise stage as a pointwise conv (1.81 vs 1.68 ms
// for pw_resident, one wave per SIMD cannot hide the epilogue); a barrier per k-step to keep the four
// row waves in step for L1 reuse (-16 % L2 requests, +5 % time).
#include "common.h"
#include "kernels.h"

#include <type_traits>

namespace mlic {

namespace {
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int DR_DWP = 12;                 // floats per depthwise channel in LDS: 9 taps, bias, 2 pad
constexpr uint32_t DR_OOB = 0x80000000u;   // buffer offset past any image: the load returns 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dr_rsrc(const float* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  float* pb = reinterpret_cast<float*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, 0, bytes, 0x00020000);
}

__device__ __forceinline__ void dr_opaque(uint32_t& v) { asm volatile("" : "+s"(v)); }
__device__ __forceinline__ int dr_swz(int row) { return (row >> 2) & 3; }

}  // namespace

#ifndef MLIC_DWPW_ROLLED_ALL  // A/B build: 1 = the k-steps of the bias-only form as a loop too
#define MLIC_DWPW_ROLLED_ALL 0
#endif
#ifndef MLIC_DPABL  // diagnostics build: 1 = one MFMA per k-step, 2 = no depthwise math, 4 = no output stores,
                    // 16 = the three tap rows all read the centre row (one L1 miss per pixel instead of three)
#define MLIC_DPABL 0
#endif
constexpr int DP_WAVES = 4;
constexpr int DP_THREADS = DP_WAVES * 64;
constexpr int DP_SEG = 60;
constexpr int DPP_WAVE_SHL1 = 0x130, DPP_WAVE_SHR1 = 0x138;

namespace {
typedef float float2v __attribute__((ext_vector_type(2)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
// lane - 1 (SHR) / lane + 1 (SHL) of the whole wave; lane 0 / 63 receive 0 (never used)
template <int CTRL>
__device__ __forceinline__ float wave_nb(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
}  // namespace

// MODE: 0 = bias only, 1 = GELU, 4 = 0.5 tanh + the checkerboard mask of P.epi (the LRP head), as
// pw_resident's MODE; residual add (RES) last
template <int CIN, int CT, int MODE, bool RES>
__global__ __launch_bounds__(DP_THREADS) void dwpw_kernel(ConvParams P, const _Float16* __restrict__ wh,
                                                         const _Float16* __restrict__ wl, int cin_pad,
                                                         const float* __restrict__ dww, const float* __restrict__ dwb) {
  constexpr int KS = CIN / 16;
  constexpr int ROWS = CT * 32;
  constexpr int TAPB = CIN * DR_DWP * 4 + ROWS * 4;
  constexpr int LDS = TAPB + KS * ROWS * 64;
  static_assert(CIN % 16 == 0 && LDS <= 160 * 1024, "dwpw: LDS");
  __shared__ __attribute__((aligned(16))) char sm[LDS];
  float* sdw = reinterpret_cast<float*>(sm);
  float* sbias = sdw + CIN * DR_DWP;
  char* sa = sm + TAPB;

  const int tid = threadIdx.x;
  {  // prologue: the A image (dwpw_kernel's layout), every load in flight before the first store
    constexpr int NG = KS * ROWS * 4;
    constexpr int NIT = (NG + DP_THREADS - 1) / DP_THREADS;
    u32x4 st[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int id = tid + it * DP_THREADS;
      const int q = id & 3, row = (id >> 2) % ROWS, j = (id >> 2) / ROWS;
      st[it] = u32x4{0u, 0u, 0u, 0u};
      if (id < NG && row < P.Cout)
        st[it] = *reinterpret_cast<const u32x4*>((q < 2 ? wh : wl) + (int64_t)row * cin_pad + 16 * j + 8 * (q & 1));
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int id = tid + it * DP_THREADS;
      const int q = id & 3, row = (id >> 2) % ROWS, j = (id >> 2) / ROWS;
      if (id < NG) *reinterpret_cast<u32x4*>(sa + (j * ROWS + row) * 64 + ((q ^ dr_swz(row)) << 4)) = st[it];
    }
  }
  for (int i = tid; i < CIN * DR_DWP; i += DP_THREADS) {
    const int c = i / DR_DWP, k = i - c * DR_DWP;
    sdw[i] = k < 9 ? dww[c * 9 + k] : (k == 9 && dwb ? dwb[c] : 0.0f);
  }
  for (int r = tid; r < ROWS; r += DP_THREADS) sbias[r] = (P.bias && r < P.Cout) ? P.bias[r] : 0.0f;
  __syncthreads();  // the only barrier

  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 31, h = lane >> 5;
  const int H = P.H, W = P.W, HW = H * W;
  const int nseg = (W + DP_SEG - 1) / DP_SEG;
  const int nyb = (H + DP_WAVES - 1) / DP_WAVES;
  const int tpi = nseg * nyb;
  const int ntiles = tpi * P.B;
  const int xcd = (int)blockIdx.x & 7, nslot = (int)gridDim.x >> 3;
  const int t_end = (int)((int64_t)(xcd + 1) * ntiles / 8);
  int tile = (int)((int64_t)xcd * ntiles / 8) + ((int)blockIdx.x >> 3);
  if (tile >= t_end) return;  // the whole workgroup: no barrier follows

  const uint32_t hw4 = (uint32_t)HW * 4u;
  const uint32_t img_bytes = (uint32_t)CIN * hw4;
  const float* xbase = P.seg[0].p;
  const int64_t xbs = P.seg[0].bs;

  struct Seg2 {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t vo[3];
  };
  auto seg_of = [&](int t) {
    Seg2 s;
    const int b = t / tpi;
    const int r = t - b * tpi;
    const int yb = r / nseg;
    const int y = yb * DP_WAVES + wave;  // rows past the image read 0 and store nothing
    const int xl = (r - yb * nseg) * DP_SEG - 2 + 2 * n;
    s.rs = dr_rsrc(xbase + (int64_t)b * xbs, img_bytes);
    const uint32_t ch = (uint32_t)(8 * h) * hw4;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const int yy = y + dy - 1;
      s.vo[dy] = yy >= 0 && yy < H && xl >= 0 && xl < W ? (uint32_t)(yy * W + xl) * 4u + ch : DR_OOB;
    }
    if (MLIC_DPABL & 16) s.vo[0] = s.vo[2] = s.vo[1];  // diagnostics: every tap row is the centre row (L1 hits)
    return s;
  };
  // one k-step: the lane's 8 channels x 3 rows as pixel pairs (24 dwordx2 loads)
  auto load_ks = [&](float2v (&r)[8][3], const Seg2& s, uint32_t so) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
        r[i][dy] = __builtin_bit_cast(float2v, __builtin_amdgcn_raw_buffer_load_b64(s.rs, s.vo[dy], so, 0));
      so += hw4;
      dr_opaque(so);
    }
  };

  // LDS offsets (kept as integers so the LDS address space survives the opaque redefinitions below)
  uint32_t tapo = 8 * h * DR_DWP;  // floats: the lane half's channels 8h.. of each k-step
  uint32_t abo = n * 64;           // bytes: A image row n of k-step 0
  // depthwise 3x3 of channel 16j + 8h + i (k-step j) at the lane's two pixels (dw3x3's order); the
  // channel's ring registers are refilled, as soon as they are read, with the same channel of the
  // k-step two ahead (segment s, channel offset so)
  auto dw_channel = [&](float2v (&rk)[3], int j, int i, const Seg2& s, uint32_t so) {
    const float4* tq = reinterpret_cast<const float4*>(sdw + tapo + (16 * j + i) * DR_DWP);
    const float4 w0 = tq[0], w1 = tq[1];
    const float2 w2 = *reinterpret_cast<const float2*>(tq + 2);
    const float tw[10] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y};
    float a0 = 0.0f, a1 = 0.0f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float p0 = rk[dy].x, p1 = rk[dy].y;
      a0 = fmaf(tw[3 * dy + 0], wave_nb<DPP_WAVE_SHR1>(p1), a0);
      a0 = fmaf(tw[3 * dy + 1], p0, a0);
      a0 = fmaf(tw[3 * dy + 2], p1, a0);
      a1 = fmaf(tw[3 * dy + 0], p0, a1);
      a1 = fmaf(tw[3 * dy + 1], p1, a1);
      a1 = fmaf(tw[3 * dy + 2], wave_nb<DPP_WAVE_SHL1>(p0), a1);
    }
    float2v v = float2v{a0 + tw[9], a1 + tw[9]};
    if (MLIC_DPABL & 2) v = rk[1];  // diagnostics: no depthwise math
    // the refill stays below the last read of the slot (as the chain kernel's input ring): hoisted
    // above it, the loads land in fresh registers that the loop back-edge copies into the ring's --
    // copies that wait for the loads (s_waitcnt vmcnt(0) at the end of every k-step)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
      rk[dy] = __builtin_bit_cast(float2v, __builtin_amdgcn_raw_buffer_load_b64(s.rs, s.vo[dy], so, 0));
    return v;
  };
  // channels i, i + 1 of k-step j split into the hi / lo B fragments of pixel e = 0, 1: one packed
  // conversion per fragment register (v_cvt_pk_f16_f32), the residual of both in one packed add
  auto dw_pair = [&](float2v (&r0)[3], float2v (&r1)[3], int j, int i, half8 (&bh)[2], half8 (&bl)[2], const Seg2& s,
                     uint32_t so) {
    uint32_t so1 = so + hw4;
    dr_opaque(so1);
    const float2v c0 = dw_channel(r0, j, i, s, so);
    const float2v c1 = dw_channel(r1, j, i + 1, s, so1);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float2v v = {c0[e], c1[e]};
      const half2v hv = __builtin_convertvector(v, half2v);
      const half2v lv = __builtin_convertvector(v - __builtin_convertvector(hv, float2v), half2v);
      bh[e][i] = hv[0];
      bh[e][i + 1] = hv[1];
      bl[e][i] = lv[0];
      bl[e][i + 1] = lv[1];
    }
  };

  // pipeline: k-step j + 1's depthwise + split runs interleaved with k-step j's MFMAs (a channel pair
  // per CT * 6 / 4 MFMAs, in program order) and refills the one-slot register ring with k-step j + 2
  // (of this tile, or of the next one: the ring and the B fragments carry across tiles)
  float2v ring[8][3];
  Seg2 cur = seg_of(tile);
  int nt = tile + nslot < t_end ? tile + nslot : tile;
  Seg2 nxt = seg_of(nt);
  load_ks(ring, cur, 0);
  half8 bh[2], bl[2];
#pragma unroll
  for (int i = 0; i < 8; i += 2)
    dw_pair(ring[i], ring[i + 1], 0, i, bh, bl, KS > 1 ? cur : nxt, (uint32_t)(KS > 1 ? 16 + i : i) * hw4);

  const int swz = dr_swz(n);
  const int gh = (h ^ swz) << 4, gl = ((2 + h) ^ swz) << 4;
  bool bad = false;
  floatx16 acc[CT][2];
  // k-step j: its MFMAs (the first k-step of a tile starts from a zero accumulator: an inline-constant
  // C operand, no zeroing moves) interleaved with k-step j + 1's depthwise
  auto kstep = [&](int j, auto first) {
    // the ring holds k-step j + 1 (of this tile, or the next tile's k-step 0 when j = KS - 1); its
    // refill is k-step j + 2 (wrapping into the next tile the same way)
    const int j1 = (j + 1) % KS, j2 = j + 2;
    const Seg2& s2 = j2 < KS ? cur : nxt;
    const uint32_t so2 = (uint32_t)(16 * (j2 < KS ? j2 : j2 - KS)) * hw4;
    half8 nbh[2], nbl[2];
    if (MLIC_DPABL & 8) __builtin_amdgcn_s_barrier();  // experiment: keep the 4 row waves in step (L1 reuse)
    // the LDS offsets are redefined per k-step: otherwise the compiler hoists the tap and A-fragment
    // reads of later k-steps (LDS is never written here) and spills them
    asm volatile("" : "+v"(tapo), "+v"(abo));
    const char* ab = sa + abo + j * ROWS * 64;
    constexpr int NM = MLIC_DPABL & 1 ? 1 : CT * 6;  // MFMAs per k-step
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      dw_pair(ring[i], ring[i + 1], j1, i, nbh, nbl, s2, so2 + (uint32_t)i * hw4);
#pragma unroll
      for (int t = (i / 2) * NM / 4; t < (i / 2 + 1) * NM / 4; ++t) {
        const int c = (MLIC_DPABL & 1) ? 0 : t / 6, r = t % 6, e = r & 1;
        // pw_resident's term order per accumulator: lo.hi, hi.lo, hi.hi
        const half8 av = *reinterpret_cast<const half8*>(ab + c * 32 * 64 + (r < 2 ? gl : gh));
        half8 bv = r >= 2 && r < 4 ? bl[e] : bh[e];
        if (MLIC_DPABL & 1) bv = bh[0] + bl[0] + bh[1] + bl[1];  // diagnostics: one MFMA per k-step
        const bool zero = decltype(first)::value && r < 2;
        acc[c][e] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, zero ? floatx16{} : acc[c][e], 0, 0, 0);
      }
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      bh[e] = nbh[e];
      bl[e] = nbl[e];
    }
  };
  for (;;) {
    kstep(0, std::true_type{});
    // the rolled loop's back-edge rotates the register ring with copies that wait for the ring's own
    // refill loads (s_waitcnt vmcnt(0) closing every k-step).  Fully unrolled, the bias-only form runs
    // 2.30 instead of 2.42 ms (8 x 192 x 544 x 960); the GELU forms do not gain (GELU 2.38 / 2.35, GELU +
    // residual 3.33 / 2.93: the unrolled body spills SGPRs into lanes), so they keep the loop
    if constexpr (MODE == 0 && !RES && !MLIC_DWPW_ROLLED_ALL) {
#pragma unroll
      for (int j = 1; j < KS; ++j) kstep(j, std::false_type{});
    } else {
#pragma nounroll
      for (int j = 1; j < KS; ++j) kstep(j, std::false_type{});
    }

    // epilogue (pw_resident's op sequence): bias, range guard, GELU, residual; pixel pairs as dwordx2
    {
      const int b = tile / tpi;
      const int r = tile - b * tpi;
      const int yb = r / nseg;
      const int y = yb * DP_WAVES + wave;
      const int xl = (r - yb * nseg) * DP_SEG - 2 + 2 * n;
      if (n >= 1 && n <= 30 && xl < W && y < H) {
        const uint32_t cs4 = (uint32_t)P.out_cs * 4u;
        const uint32_t vo_out = (uint32_t)(y * W + xl) * 4u + (uint32_t)(4 * h) * cs4;
        const auto rs_out = dr_rsrc(P.out + (int64_t)b * P.out_bs, (uint32_t)P.Cout * cs4);
        const auto rs_res = dr_rsrc(RES ? P.res + (int64_t)b * P.res_bs : P.out, RES ? (uint32_t)P.Cout * cs4 : 0u);
        const float* sb = sbias + 4 * h;
        const float unscale = ldexpf(1.0f, -P.wexp);
        // checkerboard mask (MODE 4): keep a pixel where its anchor-ness matches the flag
        bool keep[2] = {true, true};
        if (MODE == 4 && (P.epi & (EPI_MASK_ANCHOR | EPI_MASK_NONANCHOR))) {
#pragma unroll
          for (int e = 0; e < 2; ++e) keep[e] = is_anchor(y, xl + e) == ((P.epi & EPI_MASK_ANCHOR) != 0);
        }
        uint32_t so_o = 0;
#pragma unroll
        for (int c = 0; c < CT; ++c) {
          float2v xr[16];
          uint32_t oo = so_o;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            if (q > 0) {
              oo += (((q & 3) == 0) ? 5u : 1u) * cs4;  // co_u = 32c + (q&3) + 8(q>>2)
              dr_opaque(oo);
            }
            xr[q] = RES ? __builtin_bit_cast(float2v, __builtin_amdgcn_raw_buffer_load_b64(rs_res, vo_out, oo, 0))
                        : float2v{0.0f, 0.0f};
          }
          float4 bq[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) bq[g] = *reinterpret_cast<const float4*>(sb + c * 32 + 8 * g);
          oo = so_o;
          float2v vv[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const float4 b4 = bq[q >> 2];
            const float bv = (q & 3) == 0 ? b4.x : (q & 3) == 1 ? b4.y : (q & 3) == 2 ? b4.z : b4.w;
            // acc * 2^-wexp + bias as one packed fma: the product by an exact power of two is exact (a
            // subnormal result aside), so this equals ldexp then add (pw_resident does the same)
            float2v t = __builtin_elementwise_fma(float2v{acc[c][0][q], acc[c][1][q]}, float2v{unscale, unscale},
                                                  float2v{bv, bv});
            if constexpr (MODE == 1) t = gelu_erf2(t);
            if constexpr (MODE == 4) {
#pragma unroll
              for (int e = 0; e < 2; ++e) t[e] = keep[e] ? 0.5f * tanhf(t[e]) : 0.0f;
            }
            vv[q] = t + xr[q];
          }
          // range guard: a split operand beyond fp16 makes its accumulator inf / NaN, which survives
          // the epilogue and this fixed-order sum of the co-tile's outputs (a finite overflow of the
          // sum only errs to the safe side: the exact-fp32 fallback)
          float2v sum = vv[0];
#pragma unroll
          for (int q = 1; q < 16; ++q) sum += vv[q];
          bad |= !(fabsf(sum.x) <= 3.4e38f) || !(fabsf(sum.y) <= 3.4e38f);
          if (MLIC_DPABL & 4) {  // diagnostics: epilogue math without the stores
#pragma unroll
            for (int q = 0; q < 16; ++q) asm volatile("" ::"v"(vv[q][0]), "v"(vv[q][1]));
          } else if (c * 32 + 32 <= P.Cout) {  // uniform: a whole co-tile, straight-line stores
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              if (q > 0) {
                oo += (((q & 3) == 0) ? 5u : 1u) * cs4;
                dr_opaque(oo);
              }
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, vv[q]), rs_out, vo_out, oo, 0);
            }
          } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              if (q > 0) {
                oo += (((q & 3) == 0) ? 5u : 1u) * cs4;
                dr_opaque(oo);
              }
              if (c * 32 + (q & 3) + 8 * (q >> 2) + 4 * h < P.Cout)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, vv[q]), rs_out, vo_out, oo, 0);
            }
          }
          so_o += 32 * cs4;
          dr_opaque(so_o);
        }
      }
    }
    if (nt == tile) break;
    tile = nt;
    cur = nxt;
    nt = tile + nslot < t_end ? tile + nslot : tile;
    nxt = seg_of(nt);
  }
  range_report(P.rflag, bad);
}

static int dr_num_cus() { return device_cu_count(); }

// epilogue mode of P (the kernel's MODE), -1 when the kernel has none for it
static int dw_mode(const ConvParams& P) {
  const int e = P.epi & ~EPI_RES;
  if (e == EPI_NONE) return 0;
  if (e == EPI_GELU) return 1;
  if (e == EPI_TANH_HALF || e == (EPI_TANH_HALF | EPI_MASK_ANCHOR) || e == (EPI_TANH_HALF | EPI_MASK_NONANCHOR))
    return 4;
  return -1;
}

// instantiated (CIN, CT, MODE, RES): Cin = Cout = N of g_a / g_s with every epilogue they use (MLICPP_L
// 192, M 160, S2 128, S 96, the small-decoder model's N / 4 = 48); and the single-input dwsep convs of
// the latent-resolution stacks (MLICPP_L, slice_ch 32): the LRP's 224 -> 128 GELU and 128 -> 32 head
// (0.5 tanh, checkerboard mask, residual into y_hat; quantization.py:30-45), the channel context's
// 192 -> 128 GELU (context.py:115-138) -- for the kernel-level tests and A/B only: at the latent grid
// (8 K pixels per image) the per-workgroup weight prologue outweighs the saved bytes (LRP: 4.14 vs
// 4.3 ms unfused per 8 images, channel context slower), so the model fuses only grids of >= 16 K
// pixels per image (dwpw_grid_ok)
// Round 6: the Cin = Cout = 96 .. 192 forms are served by dwpw3_kernel (conv_dwpw3.hip) in the product;
// their dwpw_kernel instantiations (the "dwpw2" option's form 0) are built into the A/B library only
// (make AB=1 defines MLIC_AB_BUILD)
#define DR_ALL(X, CIN, CT) X(CIN, CT, 0, 0) X(CIN, CT, 0, 1) X(CIN, CT, 1, 0) X(CIN, CT, 1, 1)
#if MLIC_AB_BUILD
#define DR_EQ(X) DR_ALL(X, 192, 6) DR_ALL(X, 160, 5) DR_ALL(X, 128, 4) DR_ALL(X, 96, 3)
#else
#define DR_EQ(X)
#endif
#define DR_COMBOS(X) DR_EQ(X) DR_ALL(X, 48, 2) X(224, 4, 1, 0) X(128, 1, 4, 1) X(192, 4, 1, 0)

bool dwpw_grid_ok(const ConvParams& P) { return (int64_t)P.H * P.W >= 16384; }

bool dwpw_ok(const ConvParams& P, int cin_pad) {
  if (P.K != 1 || P.stride != 1 || P.pad != 0 || P.nseg != 1 || P.seg[0].C != P.Cin || cin_pad < P.Cin) return false;
  const int mode = dw_mode(P);
  if (mode < 0) return false;
  if (P.Ho != P.H || P.Wo != P.W || P.out_cs != (int64_t)P.H * P.W || (P.W % 2) != 0) return false;
  const int64_t HW = (int64_t)P.H * P.W;
  if ((int64_t)P.Cin * HW * 4 >= (1ll << 31) || (int64_t)P.Cout * HW * 4 >= (1ll << 31)) return false;
  if (dwpw2_ok(P, cin_pad)) return true;  // the Cin = Cout forms of the "dwpw2" option (dwpw3 by default)
  const int ct = (P.Cout + 31) / 32, res = (P.epi & EPI_RES) ? 1 : 0;
#define DR_OK(CIN, CT, M, R) \
  if (P.Cin == CIN && ct == CT && mode == M && res == R) return true;
  DR_COMBOS(DR_OK)
#undef DR_OK
  return false;
}

template <int CIN, int CT, int M, bool R>
static void launch_dwpw(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                        const float* dwb, hipStream_t st) {
  const int64_t want = (int64_t)((P.W + DP_SEG - 1) / DP_SEG) * ((P.H + DP_WAVES - 1) / DP_WAVES) * P.B;
  const int64_t g = std::min<int64_t>(want, (int64_t)dr_num_cus());
  const dim3 grid((unsigned)((g + 7) / 8 * 8));  // a multiple of 8: the XCD-aware deal
  hipLaunchKernelGGL((dwpw_kernel<CIN, CT, M, R>), grid, dim3(DP_THREADS), 0, st, P, wh, wl, cin_pad, dww, dwb);
  HIP_OK(hipGetLastError());
}

void dwpw_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                  const float* dwb, hipStream_t st) {
  MLIC_CHECK(dwpw_ok(P, cin_pad) && dww, "dwpw: unsupported shape");
  if (dwb && dwpw2_ok(P, cin_pad)) return dwpw2_forward(P, wh, wl, cin_pad, dww, dwb, st);
  const int ct = (P.Cout + 31) / 32, mode = dw_mode(P), res = (P.epi & EPI_RES) ? 1 : 0;
#define DR_RUN(CIN, CT, M, R)                                        \
  if (P.Cin == CIN && ct == CT && mode == M && res == R) {           \
    launch_dwpw<CIN, CT, M, R != 0>(P, wh, wl, cin_pad, dww, dwb, st); \
    return;                                                          \
  }
  DR_COMBOS(DR_RUN)
#undef DR_RUN
  throw Error("mlic: dwpw_kernel for this shape is an A/B-only instantiation (the dwpw2 option's form 0: make AB=1)");
}

}  // namespace mlic
