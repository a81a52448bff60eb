// Specialised convolution kernels for the shapes the generic implicit-GEMM tiles handle badly.
//
// 1. pw_resident_kernel — 1x1 stride-1 convs whose split weight matrix fits in LDS (Cin = Cout = N
//    of g_a / g_s: the dwsep point convs and GDN/IGDN at full and half resolution, K = 96..192).
//    With K = 192 a tiled GEMM spends most of its time in prologue/epilogue latency (6 K-tiles per
//    block).  Here each CU keeps the whole hi/lo weight matrix resident in LDS for the life of the
//    block (loaded once), and each of its 8 waves streams its own 32-pixel columns: the B fragments
//    of v_mfma_f32_32x32x16_f16 (lane l: pixel l&31, channels 8(l>>5)..+7 of each 16-deep k-step)
//    come straight from HBM into VGPRs with buffer loads (32 consecutive pixels per half-wave =
//    128-byte lines, every activation read exactly once), are split into hi/lo in registers, and
//    the next column's loads are issued as soon as a k-step's registers are consumed, so a whole
//    tile of loads is always in flight behind the MFMAs.  No barriers after the weight load.
//    Per 32-pixel tile: Cout/32 x K/16 x 3 MFMAs; A reads 4*Cout*K bytes of LDS (85 B/clk/CU at
//    K = Cout = 192, under the 128 B/clk LDS rate), so the kernel is HBM-bound:
//    bytes/pixel = 4*(Cin + Cout [+ Cout for the GDN/residual operand]).  Stride 2 (the 1x1 skip of
//    ResidualBlockWithStride) only changes the per-lane input offset.
//
// 2. conv3x3_narrow_kernel — 3x3 stride-1 convs with Cout <= 16 (g_s's last subpel conv, N -> 12).
//    On MFMA a 12-row output wastes >80 % of a 64-row tile; as a direct convolution on the fp32
//    VALU (exact fp32, packed 2-pixel FMAs) it needs 12*9 FMAs per input value, with a 16x32 output
//    tile's input patch (+1 halo) and the chunk's weights (as duplicated pairs, read by broadcast
//    ds_read_b128 straight into v_pk_fma_f32 operands) staged through LDS in 8-channel chunks.
//
// 3. conv1x1_smallcin_kernel — 1x1 (and 3x3 pad 1) convs with Cin <= 4 (g_a's first point conv and
//    skip, 3 -> N; the small-decoder model's dense first conv): write-bound; one pixel per lane (four
//    per lane with 16-byte stores where rows allow), Cout outputs from scalar weights.
#include "common.h"
#include "kernels.h"

namespace mlic {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int PW_WAVES = 8;
constexpr int PW_THREADS = PW_WAVES * 64;
constexpr int LDS_BYTES = 160 * 1024;

// buffer descriptor from a wave-uniform base (readfirstlane makes the uniformity provable: no
// waterfall loops around the buffer ops)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  float* pb = reinterpret_cast<float*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, 0, bytes, 0x00020000);
}

// hides a scalar from loop-invariant hoisting / rematerialisation (96 live SGPR offsets would spill)
__device__ __forceinline__ void opaque(uint32_t& v) { asm volatile("" : "+s"(v)); }

template <int CIN>
constexpr int pw_apitch() { return CIN + 8; }  // halves; +16 B per row spreads rows over the banks

// MODE: 0 = bias only, 1 = GELU, 2 = GDN (x * rsqrt), 3 = IGDN (x * sqrt), 4 = 0.5 tanh + the
// checkerboard mask of P.epi (the LRP head); residual add (RES) last
template <int CIN, int CT, int MODE, bool RES>
__global__ __launch_bounds__(PW_THREADS) void pw_resident_kernel(ConvParams P, const _Float16* __restrict__ wh,
                                                                  const _Float16* __restrict__ wl, int cin_pad) {
  constexpr int KS = CIN / 16;
  constexpr int APITCH = pw_apitch<CIN>();
  constexpr int ROWS = CT * 32;
  constexpr int A_SZ = ROWS * APITCH;
  static_assert(CIN % 16 == 0 && 2 * A_SZ * 2 + ROWS * 4 <= LDS_BYTES, "pw_resident: weights must fit in LDS");
  __shared__ __attribute__((aligned(16))) _Float16 sm[2 * A_SZ + 2 * ROWS];  // + fp32 bias[ROWS]
  float* sbias = reinterpret_cast<float*>(sm + 2 * A_SZ);

  const int tid = threadIdx.x;
  constexpr int QPR = CIN / 8;  // 16-byte chunks per weight row
  // every weight load issued before the first LDS store: one memory latency for the whole prologue
  // (a load -> store loop pays one per iteration, which is most of a latent-resolution launch)
  constexpr int NIT = (ROWS * QPR + PW_THREADS - 1) / PW_THREADS;
  uint4 wst[2 * NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int id = tid + it * PW_THREADS;
    const int row = id / QPR, q = id - row * QPR;
    wst[2 * it] = wst[2 * it + 1] = make_uint4(0, 0, 0, 0);
    if (id < ROWS * QPR && row < P.Cout) {
      wst[2 * it] = *reinterpret_cast<const uint4*>(wh + (int64_t)row * cin_pad + 8 * q);
      wst[2 * it + 1] = *reinterpret_cast<const uint4*>(wl + (int64_t)row * cin_pad + 8 * q);
    }
  }
  const float bias_v = (tid < ROWS && P.bias && tid < P.Cout) ? P.bias[tid] : 0.0f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int id = tid + it * PW_THREADS;
    const int row = id / QPR, q = id - row * QPR;
    if (id < ROWS * QPR) {
      *reinterpret_cast<uint4*>(sm + row * APITCH + 8 * q) = wst[2 * it];
      *reinterpret_cast<uint4*>(sm + A_SZ + row * APITCH + 8 * q) = wst[2 * it + 1];
    }
  }
  static_assert(ROWS <= PW_THREADS, "one bias per thread");
  if (tid < ROWS) sbias[tid] = bias_v;
  __syncthreads();

  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int HW = P.Ho * P.Wo;
  const int tpi = (HW + 31) >> 5;  // 32-pixel tiles per image
  const int ntiles = tpi * P.B;
  const int tstride = gridDim.x * PW_WAVES;
  int tile = blockIdx.x * PW_WAVES + wave;
  if (tile >= ntiles) return;  // no barrier follows

  constexpr bool square = MODE == 2 || MODE == 3;  // GDN/IGDN convolve x*x
  const float* xbase = P.seg[0].p;
  const int64_t xbs = P.seg[0].bs;
  const uint32_t hw4 = (uint32_t)(P.H * P.W) * 4u;  // input plane (stride 2: the full-resolution plane)
  const uint32_t ho4 = (uint32_t)HW * 4u;           // output / aux plane
  const uint32_t img_bytes = (uint32_t)CIN * hw4;
  const int S = P.stride;

  // per-tile buffer descriptor over one image's CIN planes; per-lane pixel offset in voffset,
  // the (uniform) channel offset in soffset
  auto rsrc_of = [&](int t) { return make_rsrc(xbase + (int64_t)(t / tpi) * xbs, img_bytes); };
  auto voff_of = [&](int t) {
    const int b = t / tpi;
    const int p = min(((t - b * tpi) << 5) + l32, HW - 1);
    const int pin = S == 1 ? p : (p / P.Wo) * S * P.W + (p % P.Wo) * S;
    return (uint32_t)pin * 4u + (uint32_t)(8 * h) * hw4;
  };

  // load ring: D = KS/2 k-steps ahead.  Slot j % D holds k-step j of the current tile until it is
  // consumed, then receives k-step j + D (of this tile, or of the next one for j >= KS - D).
  // (measured: a ring of 3/4 or all of KS, and non-temporal loads / stores, change nothing: the
  // TA -> TCP path is the limit, busy ~80 % of the launch with the TCP's pending-miss stall ~85 %)
  constexpr int D = KS / 2;
  float ring[D][8];
  {
    const auto rs = rsrc_of(tile);
    const uint32_t vo = voff_of(tile);
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        ring[j][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, (16 * j + i) * hw4, 0));
  }

  const _Float16* Ah = sm + l32 * APITCH + 8 * h;
  const _Float16* Al = Ah + A_SZ;
  bool bad = false;  // fp16 range guard (common.h)
  for (; tile < ntiles; tile += tstride) {
    int nt = tile + tstride;
    if (nt >= ntiles) nt = tile;  // last tile: reload the current one (keeps every load unconditional)
    const auto rsc = rsrc_of(tile);
    const uint32_t voc = voff_of(tile);
    const auto rsn = rsrc_of(nt);
    const uint32_t von = voff_of(nt);

    floatx16 acc[CT];
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[c][r] = 0.0f;
    uint32_t so = (uint32_t)(16 * D) * hw4;  // channel byte offset of the next load, advanced load by load
    opaque(so);

#pragma unroll
    for (int j = 0; j < KS; ++j) {
      half8 bh, bl;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v = ring[j % D][i];
        if (square) v *= v;
        const _Float16 hv = (_Float16)v;
        bh[i] = hv;
        bl[i] = (_Float16)(v - (float)hv);
      }
      if (j == KS - D) {  // switch the stream to the next tile's k-step 0
        so = 0;
        opaque(so);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        ring[j % D][i] = __builtin_bit_cast(float, j + D < KS ? __builtin_amdgcn_raw_buffer_load_b32(rsc, voc, so, 0)
                                                              : __builtin_amdgcn_raw_buffer_load_b32(rsn, von, so, 0));
        so += (i == 7) ? 9 * hw4 : hw4;
        opaque(so);
      }
      // keep the reload here: the scheduler would otherwise hoist the ring's loads above the MFMAs
      __builtin_amdgcn_sched_barrier(0);
#ifndef MLIC_PW_ABL  // diagnostics: 1 = one MFMA per k-step, 2 = no output stores, 3 = both
#define MLIC_PW_ABL 0
#endif
      if (MLIC_PW_ABL & 1) {
        const half8 ah0 = *reinterpret_cast<const half8*>(Ah + 16 * j);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0, bh + bl, acc[0], 0, 0, 0);
        continue;
      }
      // co-tiles in pairs so consecutive MFMAs never chain on one accumulator
#pragma unroll
      for (int c = 0; c < CT; c += 2) {
        const int c1 = (c + 1 < CT) ? c + 1 : c;
        const half8 ah0 = *reinterpret_cast<const half8*>(Ah + c * 32 * APITCH + 16 * j);
        const half8 al0 = *reinterpret_cast<const half8*>(Al + c * 32 * APITCH + 16 * j);
        const half8 ah1 = *reinterpret_cast<const half8*>(Ah + c1 * 32 * APITCH + 16 * j);
        const half8 al1 = *reinterpret_cast<const half8*>(Al + c1 * 32 * APITCH + 16 * j);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al0, bh, acc[c], 0, 0, 0);
        if (c1 != c) acc[c1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al1, bh, acc[c1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0, bl, acc[c], 0, 0, 0);
        if (c1 != c) acc[c1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1, bl, acc[c1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0, bh, acc[c], 0, 0, 0);
        if (c1 != c) acc[c1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1, bh, acc[c1], 0, 0, 0);
      }
    }

    // epilogue: buffer ops whose per-lane part is (pixel, lane half) and whose channel part is a
    // uniform SGPR offset, so 96 stores need no 64-bit VGPR addresses
    const int b = tile / tpi;
    const int p = ((tile - b * tpi) << 5) + l32;
    const uint32_t cs4 = (uint32_t)P.out_cs * 4u;
    const uint32_t vo_out = (uint32_t)p * 4u + (uint32_t)(4 * h) * cs4;
    const auto rs_out = make_rsrc(P.out + (int64_t)b * P.out_bs, (uint32_t)P.Cout * cs4);
    constexpr bool gdn = MODE == 2 || MODE == 3, igdn = MODE == 3, gelu = MODE == 1, tanh_mask = MODE == 4;
    // checkerboard mask: keep v where this pixel's anchor-ness matches the flag (MODE 4 only)
    bool keep = true;
    if (tanh_mask && (P.epi & (EPI_MASK_ANCHOR | EPI_MASK_NONANCHOR))) {
      const int oh = p / P.Wo, ow = p - oh * P.Wo;
      keep = is_anchor(oh, ow) == ((P.epi & EPI_MASK_ANCHOR) != 0);
    }
    constexpr bool res = RES;
    const auto rs_aux = make_rsrc(gdn ? P.aux + (int64_t)b * P.aux_bs : P.out, gdn ? (uint32_t)P.Cout * ho4 : 0u);
    const uint32_t vo_aux = (uint32_t)p * 4u + (uint32_t)(4 * h) * ho4;
    const auto rs_res = make_rsrc(res ? P.res + (int64_t)b * P.res_bs : P.out, res ? (uint32_t)P.Cout * cs4 : 0u);
    const float* sb = sbias + 4 * h;  // per-lane base; the channel part folds into the ds_read offset
    const float unscale = ldexpf(1.0f, -P.wexp);
    // per co-tile: issue the 16 aux / residual loads together, then one wait, then 16 stores
    uint32_t so_o = 0, so_a = 0;  // channel byte offsets co_u * out_cs * 4 and co_u * HW * 4
    if (p < HW) {
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        float xa[16], xr[16];
        uint32_t oo = so_o, oa = so_a;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (r > 0) {
            const uint32_t step = ((r & 3) == 0) ? 5u : 1u;  // co_u = 32c + (r&3) + 8(r>>2)
            oo += step * cs4;
            oa += step * ho4;
            opaque(oo);
            opaque(oa);
          }
          if (gdn) xa[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_aux, vo_aux, oa, 0));
          xr[r] = res ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_res, vo_out, oo, 0)) : 0.0f;
        }
        // biases of this co-tile: rows 32c + 8g + 4h .. +3 as four 16-byte LDS reads
        float4 bq[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) bq[g] = *reinterpret_cast<const float4*>(sb + c * 32 + 8 * g);
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float4 b4 = bq[r >> 2];
          const float bv = (r & 3) == 0 ? b4.x : (r & 3) == 1 ? b4.y : (r & 3) == 2 ? b4.z : b4.w;
          float x = __builtin_fmaf(acc[c][r], unscale, bv);  // == ldexp(acc, -wexp) + bias (exact product)
          // fp16 range guard on the accumulator (an input beyond fp16 splits to inf/NaN and poisons it;
          // checked before GDN, whose rsqrt(inf) = 0 would hide it); cheaper here than in the ring
          bad |= !(fabsf(x) <= 3.4e38f);
          if (gelu) x = gelu_erf(x);
          if (gdn) x = gdn_apply(xa[r], x, igdn);
          if (tanh_mask) x = keep ? 0.5f * tanhf(x) : 0.0f;
          v[r] = x + xr[r];
        }
        // straight-line stores for a full co-tile (the uniform common case); per-row guards only on
        // the ragged last one
        oo = so_o;
        if ((MLIC_PW_ABL & 2) && P.Cout > 0) {  // uniform: keeps the stores in the code, skips them
          asm volatile("" :: "v"(v[0]), "v"(v[5]), "v"(v[10]), "v"(v[15]));
        } else
        if (c * 32 + 32 <= P.Cout) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if (r > 0) {
              oo += (((r & 3) == 0) ? 5u : 1u) * cs4;
              opaque(oo);
            }
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[r]), rs_out, vo_out, oo, 0);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if (r > 0) {
              oo += (((r & 3) == 0) ? 5u : 1u) * cs4;
              opaque(oo);
            }
            if (c * 32 + (r & 3) + 8 * (r >> 2) + 4 * h < P.Cout)
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[r]), rs_out, vo_out, oo, 0);
          }
        }
        so_o += 32 * cs4;
        so_a += 32 * ho4;
        opaque(so_o);
        opaque(so_a);
      }
    }
  }
  range_report(P.rflag, bad);
}

static int num_cus() { return device_cu_count(); }

// epilogue mode of P (see the kernel's MODE), -1 when the kernel has none for it
static int pw_mode(const ConvParams& P) {
  const int e = P.epi & ~EPI_RES;
  if (e == EPI_NONE) return 0;
  if (e == EPI_GELU) return 1;
  if (e == (EPI_GDN | EPI_SQUARE_IN)) return 2;
  if (e == (EPI_IGDN | EPI_SQUARE_IN)) return 3;
  if (e == EPI_TANH_HALF || e == (EPI_TANH_HALF | EPI_MASK_ANCHOR) || e == (EPI_TANH_HALF | EPI_MASK_NONANCHOR))
    return 4;
  return -1;
}

// instantiated (CIN, CT, MODE, RES) tuples.  PW_ALL: Cin = Cout = 32 CT, every epilogue (g_a / g_s
// point convs, GDN / IGDN, at full and half resolution).  The single tuples are the latent-resolution
// 1x1 convs of the context models and the LRP (MLICPP_L, slice_ch 32): there the generic tiles
// hold one output tile per CU and spend the launch in load latency, while this kernel streams
// 32-pixel columns from every wave of every CU.
#define PW_ALL(X, CIN, CT) \
  X(CIN, CT, 0, 0) X(CIN, CT, 0, 1) X(CIN, CT, 1, 0) X(CIN, CT, 1, 1) \
  X(CIN, CT, 2, 0) X(CIN, CT, 2, 1) X(CIN, CT, 3, 0) X(CIN, CT, 3, 1)
#define PW_COMBOS(X)                                                                              \
  PW_ALL(X, 96, 3) PW_ALL(X, 128, 4) PW_ALL(X, 160, 5) PW_ALL(X, 192, 6)                          \
  /* MLICPP_M_SMALL_DEC's g_s (N / 4 = 48 channels at full resolution) */                         \
  PW_ALL(X, 48, 2)                                                                                \
  /* g_s's output conv as per-tap partials: N -> 9 x 12 = 108 rows */                             \
  X(192, 4, 0, 0) X(96, 4, 0, 0) X(48, 4, 0, 0)                                                   \
  /* LRP: 224 -> 128 GELU; head 128 -> 32 (0.5 tanh, checkerboard mask, residual into y_hat) */   \
  X(224, 4, 1, 0) X(128, 1, 4, 1)                                                                 \
  /* channel context (dwsep): 32i -> 192 GELU, 192 -> 128 GELU */                                 \
  X(32, 6, 1, 0) X(64, 6, 1, 0) X(96, 6, 1, 0) X(128, 6, 1, 0) X(160, 6, 1, 0) X(192, 4, 1, 0)   \
  /* inter/intra q/k/v (dim -> dim), local qkv_proj 32 -> 96, proj 64 -> 64 */                   \
  X(32, 1, 0, 0) X(64, 2, 0, 0) X(32, 3, 0, 0)                                                    \
  /* global contexts: mlp.0 GELU (96 -> 128, 64 -> 128), mlp.4 + residual 128 -> 64, skip */      \
  X(96, 4, 1, 0) X(64, 4, 1, 0) X(128, 2, 0, 1) X(96, 2, 0, 0)

bool pw_resident_ok(const ConvParams& P, int cin_pad) {
  if (P.K != 1 || (P.stride != 1 && P.stride != 2) || P.pad != 0 || P.nseg != 1) return false;
  const int mode = pw_mode(P);
  if (mode < 0) return false;
  if (P.Ho != (P.H - 1) / P.stride + 1 || P.Wo != (P.W - 1) / P.stride + 1) return false;
  // the weight rows are read with stride cin_pad (>= Cin; padding columns are zeros)
  if (P.seg[0].C != P.Cin || cin_pad < P.Cin) return false;
  if (P.stride != 1 && (mode == 2 || mode == 3 || mode == 4)) return false;  // GDN aux is the conv input; mask grid
  const int64_t HW = (int64_t)P.H * P.W;
  if ((int64_t)P.Cin * HW * 4 >= (1ll << 31) || (int64_t)P.Cout * HW * 4 >= (1ll << 31)) return false;
  const int ct = (P.Cout + 31) / 32;
  const int res = (P.epi & EPI_RES) ? 1 : 0;
#define MLIC_PW_OK(CIN, CT, M, R) \
  if (P.Cin == CIN && ct == CT && mode == M && res == R) return true;
  PW_COMBOS(MLIC_PW_OK)
#undef MLIC_PW_OK
  return false;
}

template <int CIN, int CT, int M, bool R>
static void launch_pw(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  const int64_t ntiles = (int64_t)((P.Ho * P.Wo + 31) / 32) * P.B;
  const int64_t want = (ntiles + PW_WAVES - 1) / PW_WAVES;
  const dim3 grid((unsigned)std::min<int64_t>(want, (int64_t)num_cus()));
  hipLaunchKernelGGL((pw_resident_kernel<CIN, CT, M, R>), grid, dim3(PW_THREADS), 0, st, P, wh, wl, cin_pad);
  HIP_OK(hipGetLastError());
}

void pw_resident_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st) {
  MLIC_CHECK(pw_resident_ok(P, cin_pad), "pw_resident: unsupported shape");
  if (pw3_ok(P, cin_pad)) return pw3_forward(P, wh, wl, cin_pad, st);  // full-resolution GDN / IGDN
  const int mode = pw_mode(P);
  const int ct = (P.Cout + 31) / 32;
  const int res = (P.epi & EPI_RES) ? 1 : 0;
#define MLIC_PW_RUN(CIN, CT, M, R)                                  \
  if (P.Cin == CIN && ct == CT && mode == M && res == R) {          \
    launch_pw<CIN, CT, M, R != 0>(P, wh, wl, cin_pad, st);          \
    return;                                                         \
  }
  PW_COMBOS(MLIC_PW_RUN)
#undef MLIC_PW_RUN
}

// ---------------------------------------------------------------------------------------------
// 3x3 stride-1 pad-1 conv, Cout = COUT <= 16, exact fp32 on the VALU (packed v_pk_fma_f32).
// Tile 16 rows x 128 columns, 256 threads, each thread one row of 8 pixels x COUT outputs (4 pixel
// pairs x COUT float2 accumulators), so every broadcast weight read (w, w, w', w') feeds 8 packed
// FMAs.  Input staged per 2-channel chunk (LDS for 2 blocks / CU) with aligned float4 loads (patch column 0 = input column
// ow0 - 4), weights per chunk as duplicated pairs; both double-buffered in LDS.  Outputs leave as
// 16-byte stores (4 pixels of a channel, or under the pixel shuffle 2 pixels x 2 channels).
constexpr int NR_TH = 16, NR_TW = 128, NR_CC = 2;
constexpr int NR_PH = NR_TH + 2, NR_PQ = NR_TW / 4 + 2;  // patch rows, float4 per patch row
constexpr int NR_PITCH = NR_PQ * 4;                      // floats
constexpr int NR_PATCH4 = NR_CC * NR_PH * NR_PQ;         // float4 per chunk patch
constexpr int NR_STAGE = (NR_PATCH4 + 255) / 256;

template <int COUT>
__global__ __launch_bounds__(256) void conv3x3_narrow_kernel(ConvParams P) {
  typedef float float2v __attribute__((ext_vector_type(2)));
  typedef float float4v __attribute__((ext_vector_type(4)));
  constexpr int NW = NR_CC * 9 * COUT / 2;  // (w, w, w', w') float4 per chunk
  static_assert(COUT % 2 == 0, "Cout pairs");
  __shared__ __attribute__((aligned(16))) float4v sp[2][NR_PATCH4];
  __shared__ __attribute__((aligned(16))) float4v swp[2][NW];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;  // pixels ow0 + 8 tx .. + 7 of row oh0 + ty
  const int ow0 = blockIdx.x * NR_TW, oh0 = blockIdx.y * NR_TH;
  const int b = blockIdx.z;
  const int H = P.H, W = P.W, W4 = W >> 2;
  const int64_t HW = (int64_t)H * W;
  const float4v* x4 = reinterpret_cast<const float4v*>(P.seg[0].p + (int64_t)b * P.seg[0].bs);
  const int nchunk = (P.Cin + NR_CC - 1) / NR_CC;
  const float* w = P.wpk;  // [9][Cin][COUT]
  constexpr int WSTAGE = (NW + 255) / 256;

  float4v stage[NR_STAGE];
  float4v wst[WSTAGE];
  auto load = [&](int ch) {
#pragma unroll
    for (int s = 0; s < NR_STAGE; ++s) {
      const int e = tid + s * 256;
      float4v v = {0.f, 0.f, 0.f, 0.f};
      if (e < NR_PATCH4) {
        const int c = e / (NR_PH * NR_PQ), rem = e - c * (NR_PH * NR_PQ);
        const int py = rem / NR_PQ, pq = rem - py * NR_PQ;
        const int ci = ch * NR_CC + c, ih = oh0 + py - 1, iq = (ow0 >> 2) - 1 + pq;
        if (ci < P.Cin && ih >= 0 && ih < H && iq >= 0 && iq < W4) v = x4[(ci * HW >> 2) + (int64_t)ih * W4 + iq];
      }
      stage[s] = v;
    }
#pragma unroll
    for (int s = 0; s < WSTAGE; ++s) {
      const int e = tid + s * 256;  // (c, tap, co pair)
      float4v v = {0.f, 0.f, 0.f, 0.f};
      if (e < NW) {
        const int c = e / (9 * COUT / 2), rem = e - c * (9 * COUT / 2);
        const int tap = rem / (COUT / 2), cp = rem - tap * (COUT / 2);
        const int ci = ch * NR_CC + c;
        if (ci < P.Cin) {
          const float* wr = w + ((int64_t)tap * P.Cin + ci) * COUT + 2 * cp;
          v = float4v{wr[0], wr[0], wr[1], wr[1]};
        }
      }
      wst[s] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int s = 0; s < NR_STAGE; ++s) {
      const int e = tid + s * 256;
      if (e < NR_PATCH4) sp[buf][e] = stage[s];
    }
#pragma unroll
    for (int s = 0; s < WSTAGE; ++s) {
      const int e = tid + s * 256;
      if (e < NW) swp[buf][e] = wst[s];
    }
  };

  float2v acc[COUT][4];
#pragma unroll
  for (int co = 0; co < COUT; ++co)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[co][q] = float2v{0.0f, 0.0f};

  load(0);
  store(0);
  __syncthreads();
  for (int ch = 0; ch < nchunk; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < nchunk) load(ch + 1);
    const float* pb = reinterpret_cast<const float*>(sp[cur]) + ty * NR_PITCH + 8 * tx + 3;
    const int cmax = min(NR_CC, P.Cin - ch * NR_CC);
    for (int c = 0; c < cmax; ++c) {
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        // input columns 8tx-1 .. 8tx+8 <-> patch columns 8tx+3 .. 8tx+12
        const float* rp = pb + (c * NR_PH + dy) * NR_PITCH;
        const float4v m0 = *reinterpret_cast<const float4v*>(rp + 1);
        const float4v m1 = *reinterpret_cast<const float4v*>(rp + 5);
        const float xw[10] = {rp[0], m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w, rp[9]};
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const float4v* wq = &swp[cur][(c * 9 + dy * 3 + dx) * (COUT / 2)];
#pragma unroll
          for (int cp = 0; cp < COUT / 2; ++cp) {
            const float4v ww = wq[cp];  // all lanes read the same address: broadcast
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float2v xv = {xw[2 * q + dx], xw[2 * q + 1 + dx]};
              acc[2 * cp][q] = __builtin_elementwise_fma(xv, float2v{ww.x, ww.y}, acc[2 * cp][q]);
              acc[2 * cp + 1][q] = __builtin_elementwise_fma(xv, float2v{ww.z, ww.w}, acc[2 * cp + 1][q]);
            }
          }
        }
      }
    }
    if (ch + 1 < nchunk) store(cur ^ 1);
    __syncthreads();
  }

  const int oh = oh0 + ty, ow = ow0 + 8 * tx;
  if (oh >= P.Ho || ow >= P.Wo) return;
  const int p = oh * P.Wo + ow;
  const bool shuf = (P.epi & EPI_SHUFFLE) != 0;
  const bool full = ow + 7 < P.Wo && conv_vec_ok(P) && !(P.epi & (EPI_GDN | EPI_IGDN | EPI_MASK_ANCHOR | EPI_MASK_NONANCHOR));
  if (full && !shuf) {
#pragma unroll
    for (int co = 0; co < COUT; ++co)
#pragma unroll
      for (int h4 = 0; h4 < 2; ++h4)
        conv_store4(P, b, co, p + 4 * h4,
                    make_float4(acc[co][2 * h4].x, acc[co][2 * h4].y, acc[co][2 * h4 + 1].x, acc[co][2 * h4 + 1].y));
  } else if (full) {
#pragma unroll
    for (int cp = 0; cp < COUT / 2; ++cp)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        conv_store_shuf4(P, b, 2 * cp, p + 2 * q,
                         make_float4(acc[2 * cp][q].x, acc[2 * cp + 1][q].x, acc[2 * cp][q].y, acc[2 * cp + 1][q].y));
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if (ow + 2 * q + e >= P.Wo) continue;
#pragma unroll
        for (int co = 0; co < COUT; ++co) conv_store(P, b, co, p + 2 * q + e, e ? acc[co][q].y : acc[co][q].x);
      }
  }
}

bool conv_narrow_ok(const ConvParams& P) {
  // float4 patch loads: W % 4 == 0 and 16-byte aligned channel planes
  return P.K == 3 && P.stride == 1 && P.pad == 1 && P.nseg == 1 && P.Cout == 12 && P.Ho == P.H && P.Wo == P.W &&
         !(P.epi & EPI_SQUARE_IN) && (P.W % 4) == 0 && ((int64_t)P.H * P.W) % 4 == 0 && (P.seg[0].bs % 4) == 0 &&
         (reinterpret_cast<uintptr_t>(P.seg[0].p) % 16) == 0;
}

void conv_narrow_forward(const ConvParams& P, hipStream_t st) {
  MLIC_CHECK(conv_narrow_ok(P), "conv_narrow: unsupported shape");
  dim3 grid((P.Wo + NR_TW - 1) / NR_TW, (P.Ho + NR_TH - 1) / NR_TH, P.B);
  hipLaunchKernelGGL(conv3x3_narrow_kernel<12>, grid, dim3(256), 0, st, P);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// The N -> 12 3x3 output conv of g_s as a 1x1 conv N -> 9 x 12 (per-tap partial products, on the
// resident MFMA kernel) plus this gather: out = bias + sum over the 9 taps (fixed order) of the
// shifted partials, written through the PixelShuffle(2) (channel c = 4 c' + 2 dy + dx) as float2 pairs
// (dx = 0, 1).  part [B][9 * 12][H][W] (row tap * 12 + c), out [B][3][2H][2W].
__global__ __launch_bounds__(256) void taps_gather_kernel(const float* __restrict__ part, int64_t part_bs,
                                                          const float* __restrict__ bias, float* __restrict__ out,
                                                          int64_t out_bs, int H, int W) {
  constexpr int C = 12;
  const int w = blockIdx.x * 64 + (threadIdx.x & 63), h = blockIdx.y * 4 + (threadIdx.x >> 6), b = blockIdx.z;
  if (w >= W || h >= H) return;
  const int64_t HW = (int64_t)H * W;
  const float* pb = part + (int64_t)b * part_bs;
  float acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) acc[c] = 0.0f;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int y = h + t / 3 - 1, x = w + t % 3 - 1;
    if (y < 0 || y >= H || x < 0 || x >= W) continue;
    const float* q = pb + (int64_t)t * C * HW + (int64_t)y * W + x;
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] += q[c * HW];
  }
  float* ob = out + (int64_t)b * out_bs;
  const int W2 = 2 * W;
  const int64_t HW4 = 4 * HW;
#pragma unroll
  for (int cq = 0; cq < 3; ++cq)
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int c = 4 * cq + 2 * dy;
      const float b0 = bias ? bias[c] : 0.0f, b1 = bias ? bias[c + 1] : 0.0f;
      *reinterpret_cast<float2*>(ob + cq * HW4 + (int64_t)(2 * h + dy) * W2 + 2 * w) =
          make_float2(acc[c] + b0, acc[c + 1] + b1);
    }
}

void taps_gather(const float* part, int64_t part_bs, const float* bias, float* out, int64_t out_bs, int H, int W,
                 int B, hipStream_t st) {
  hipLaunchKernelGGL(taps_gather_kernel, dim3((W + 63) / 64, (H + 3) / 4, B), dim3(256), 0, st, part, part_bs, bias,
                     out, out_bs, H, W);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// KxK conv (K = 1 pad 0, or K = 3 pad 1; any stride) with Cin <= 4: one output pixel per lane, exact
// fp32, taps outer and channels inner (the [tap][Cin][Cout] packing order); K = 3 serves
// MLICPP_M_SMALL_DEC's dense first conv (3 -> N, stride 2)
template <int CIN, int K>
__device__ __forceinline__ float smallcin_in(const ConvParams& P, const float* xb, int64_t HWi, int c, int iy, int ix) {
  if (K > 1 && (iy < 0 || iy >= P.H || ix < 0 || ix >= P.W)) return 0.0f;
  float v = xb[c * HWi + (int64_t)iy * P.W + ix];
  if (P.epi & EPI_SQUARE_IN) v *= v;
  return v;
}

template <int CIN, int K>
__global__ __launch_bounds__(256) void conv1x1_smallcin_kernel(ConvParams P) {
  constexpr int KK = K * K;
  const int HWo = P.Ho * P.Wo;
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= HWo) return;
  const int oh = p / P.Wo, ow = p - oh * P.Wo;
  const int64_t HWi = (int64_t)P.H * P.W;
  const float* xb = P.seg[0].p + (int64_t)b * P.seg[0].bs;
  float xv[KK][CIN];
#pragma unroll
  for (int t = 0; t < KK; ++t)
#pragma unroll
    for (int c = 0; c < CIN; ++c)
      xv[t][c] = smallcin_in<CIN, K>(P, xb, HWi, c, oh * P.stride + t / K - P.pad, ow * P.stride + t % K - P.pad);
  const float* w = P.wpk;  // [K*K][Cin][Cout]
  for (int co = 0; co < P.Cout; ++co) {
    float v = 0.0f;
#pragma unroll
    for (int t = 0; t < KK; ++t)
#pragma unroll
      for (int c = 0; c < CIN; ++c) v = fmaf(xv[t][c], w[(t * CIN + c) * P.Cout + co], v);
    conv_store(P, b, co, p, v);
  }
}

// the same with four consecutive output pixels of one row per lane and 16-byte stores (the layer is
// write-bound: Cout = N outputs per input pixel); identical per-element arithmetic
template <int CIN, int K>
__global__ __launch_bounds__(256) void conv1x1_smallcin_vec_kernel(ConvParams P) {
  constexpr int KK = K * K;
  const int HWo = P.Ho * P.Wo;
  const int p = 4 * (blockIdx.x * 256 + threadIdx.x);
  const int b = blockIdx.y;
  if (p >= HWo) return;
  const int oh = p / P.Wo, ow = p - oh * P.Wo;
  const int64_t HWi = (int64_t)P.H * P.W;
  const int S = P.stride;
  const float* xb = P.seg[0].p + (int64_t)b * P.seg[0].bs;
  float xv[KK][CIN][4];
#pragma unroll
  for (int t = 0; t < KK; ++t)
#pragma unroll
    for (int c = 0; c < CIN; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        xv[t][c][e] = smallcin_in<CIN, K>(P, xb, HWi, c, oh * S + t / K - P.pad, (ow + e) * S + t % K - P.pad);
  const float* w = P.wpk;  // [K*K][Cin][Cout]
  for (int co = 0; co < P.Cout; ++co) {
    float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < KK; ++t)
#pragma unroll
      for (int c = 0; c < CIN; ++c) {
        const float wc = w[(t * CIN + c) * P.Cout + co];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(xv[t][c][e], wc, v[e]);
      }
    conv_store4(P, b, co, p, make_float4(v[0], v[1], v[2], v[3]));
  }
}

bool conv_smallcin_ok(const ConvParams& P) {
  return ((P.K == 1 && P.pad == 0) || (P.K == 3 && P.pad == 1)) && P.nseg == 1 && P.Cin >= 1 && P.Cin <= 4;
}

template <int K>
static void launch_smallcin(const ConvParams& P, hipStream_t st) {
  if ((P.Wo & 3) == 0 && conv_vec_ok(P) && !(P.epi & EPI_SHUFFLE)) {
    dim3 grid((P.Ho * P.Wo / 4 + 255) / 256, P.B);
    switch (P.Cin) {
      case 1: hipLaunchKernelGGL((conv1x1_smallcin_vec_kernel<1, K>), grid, dim3(256), 0, st, P); break;
      case 2: hipLaunchKernelGGL((conv1x1_smallcin_vec_kernel<2, K>), grid, dim3(256), 0, st, P); break;
      case 3: hipLaunchKernelGGL((conv1x1_smallcin_vec_kernel<3, K>), grid, dim3(256), 0, st, P); break;
      default: hipLaunchKernelGGL((conv1x1_smallcin_vec_kernel<4, K>), grid, dim3(256), 0, st, P); break;
    }
    HIP_OK(hipGetLastError());
    return;
  }
  dim3 grid((P.Ho * P.Wo + 255) / 256, P.B);
  switch (P.Cin) {
    case 1: hipLaunchKernelGGL((conv1x1_smallcin_kernel<1, K>), grid, dim3(256), 0, st, P); break;
    case 2: hipLaunchKernelGGL((conv1x1_smallcin_kernel<2, K>), grid, dim3(256), 0, st, P); break;
    case 3: hipLaunchKernelGGL((conv1x1_smallcin_kernel<3, K>), grid, dim3(256), 0, st, P); break;
    default: hipLaunchKernelGGL((conv1x1_smallcin_kernel<4, K>), grid, dim3(256), 0, st, P); break;
  }
  HIP_OK(hipGetLastError());
}

void conv_smallcin_forward(const ConvParams& P, hipStream_t st) {
  MLIC_CHECK(conv_smallcin_ok(P), "conv_smallcin: unsupported shape");
  if (P.K == 1) launch_smallcin<1>(P, st);
  else launch_smallcin<3>(P, st);
}

}  // namespace mlic
