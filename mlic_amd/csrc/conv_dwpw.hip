// Fused depthwise-separable conv ("dwpw"): the fork's DepthWiseConv (modules/layers/conv.py:22-32:
// depthwise 3x3 stride 1 pad 1 + bias, then pointwise 1x1 + bias, then the block's epilogue) in ONE
// kernel, so the depthwise output never goes to HBM.  g_a / g_s run it on every stride-1 dwsep conv
// of their residual blocks (res_blk.py ResidualBlock conv1/conv2, ResidualBlockWithStride conv2,
// ResidualBlockUpsample conv): Cin = Cout = N.
//
// Block = 8 rows x 32 columns of one image, 8 waves (wave w: row y0 + w, lane l32: column x0 + l32,
// lane half h: channels 8h..8h+7 of a 16-channel k-step -- the B fragment of
// v_mfma_f32_32x32x16_f16), all Cout rows per wave.  Per k-step, through a 2-slot LDS ring:
//   * the input patch, 16 channels x 10 rows x 34 columns (the block + its 1-pixel halo), staged
//     through registers by coalesced buffer loads (out-of-image positions read 0 via an
//     out-of-range offset) one k-step ahead and stored with ds_write_b32;
//   * the k-step's pointwise weights, split hi/lo, 64-byte rows [hi k0-7 | hi k8-15 | lo | lo] with
//     the 16-byte granule XOR-swizzled by (row >> 2) & 3 (conflict-free ds_read_b128 A fragments),
//     staged the same way from the L2-resident split weights;
// and the depthwise taps + bias stay resident ([C][12] floats, broadcast ds_read_b128).  The
// depthwise sum is acc = 0, 9 taps row-major by fma, + bias (dw3x3's order: the fused B operand
// equals the unfused depthwise output bit for bit), then the hi/lo split in registers; one barrier
// per k-step.  A persistent grid walks the blocks; the staging stream runs across block boundaries.
// HBM bytes per pixel: 4 * (Cin + Cout [+ Cout residual]) -- the pointwise conv's alone.
#include "common.h"
#include "kernels.h"

namespace mlic {

namespace {
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int DP_WAVES = 8;
constexpr int DP_THREADS = DP_WAVES * 64;
constexpr int DP_TW = 32;                      // block columns
constexpr int DP_PR = DP_WAVES + 2;            // patch rows
constexpr int DP_PC = DP_TW + 2;               // patch columns
constexpr int DP_CH = DP_PR * DP_PC;           // floats per channel plane of the patch
constexpr int DP_KC = 32;                     // channels per k-step (two 16-deep MFMA k-slices)
constexpr int DP_PSZ = DP_KC * DP_CH;          // floats per k-step patch
constexpr int DP_DWP = 12;                     // floats per depthwise channel: 9 taps, bias, 2 pad
constexpr uint32_t DP_OOB = 0x80000000u;       // buffer offset past any image: the load returns 0

__device__ __forceinline__ __amdgpu_buffer_rsrc_t dp_rsrc(const float* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  float* pb = reinterpret_cast<float*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, 0, bytes, 0x00020000);
}

__device__ __forceinline__ void dp_opaque(uint32_t& v) { asm volatile("" : "+s"(v)); }
}  // namespace

#ifdef MLIC_DP_TRACE  // diagnostic builds (tools/gpu/dwpw_probe.hip): phase stamps of workgroup 0
__device__ unsigned long long* g_dp_trace;
#define DP_TR(slot) \
  if (blockIdx.x == 0 && threadIdx.x < 64 && (slot) < 512) tr[(slot)] = __builtin_readcyclecounter()
#else
#define DP_TR(slot)
#endif
namespace {
__device__ __forceinline__ int dp_swz(int row) { return (row >> 1) & 7; }
}  // namespace

template <int CIN, int CT, bool GELU, bool RES>
__global__ __launch_bounds__(DP_THREADS) void dwpw_kernel(ConvParams P, const _Float16* __restrict__ wh,
                                                        const _Float16* __restrict__ wl, int cin_pad,
                                                        const float* __restrict__ dww, const float* __restrict__ dwb) {
  constexpr int KS = CIN / DP_KC;
  constexpr int ROWS = CT * 32;
  constexpr int WSZ = ROWS * 128;                      // bytes per k-step weight slot
  constexpr int NWQ = ROWS * 8;                        // 16-byte weight chunks per k-step
  constexpr int NWL = (NWQ + DP_THREADS - 1) / DP_THREADS;
  constexpr int LDS = 2 * DP_PSZ * 4 + 2 * WSZ + CIN * DP_DWP * 4 + ROWS * 4;
  static_assert(LDS <= 160 * 1024, "dwpw LDS");
  __shared__ __attribute__((aligned(16))) char sm[LDS];
#ifdef MLIC_DP_TRACE
  __shared__ unsigned long long tr[512];
#endif
  float* sin = reinterpret_cast<float*>(sm);
  char* sw = sm + 2 * DP_PSZ * 4;
  float* sdw = reinterpret_cast<float*>(sw + 2 * WSZ);
  float* sbias = sdw + CIN * DP_DWP;

  const int tid = threadIdx.x;
  for (int i = tid; i < CIN * DP_DWP; i += DP_THREADS) {
    const int c = i / DP_DWP, k = i - c * DP_DWP;
    sdw[i] = k < 9 ? dww[c * 9 + k] : (k == 9 && dwb ? dwb[c] : 0.0f);
  }
  for (int r = tid; r < ROWS; r += DP_THREADS) sbias[r] = (P.bias && r < P.Cout) ? P.bias[r] : 0.0f;

  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, h = lane >> 5;
  const int H = P.H, W = P.W, HW = H * W;
  const int nseg = (W + DP_TW - 1) / DP_TW;
  const int nyb = (H + DP_WAVES - 1) / DP_WAVES;
  const int nblk = nseg * nyb * P.B;
  if ((int)blockIdx.x >= nblk) return;  // before any barrier: the whole workgroup leaves
  const int nmine = (nblk - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int G = nmine * KS;  // k-steps of this workgroup
  const uint32_t hw4 = (uint32_t)HW * 4u;
  const uint32_t img_bytes = (uint32_t)CIN * hw4;

  auto block_of = [&](int n, int& b, int& y0, int& x0) {
    const int t = (int)blockIdx.x + n * (int)gridDim.x;
    b = t / (nseg * nyb);
    const int r = t - b * nseg * nyb;
    const int yb = r / nseg;
    y0 = yb * DP_WAVES;
    x0 = (r - yb * nseg) * DP_TW;
  };

  // ---- staging cursor (loads run 2 k-steps ahead of the compute, across block boundaries): thread
  // t < DP_CH owns patch position t (row t / DP_PC, column t % DP_PC) for all DP_KC channels
  float rin[DP_KC];
  u32x4 rw[NWL];
  uint32_t vpos = DP_OOB;  // byte offset of this thread's patch position in the load block's image
  __amdgpu_buffer_rsrc_t rs_in = dp_rsrc(P.seg[0].p, img_bytes);
  auto set_block = [&](int n) {
    int b, y0, x0;
    block_of(n, b, y0, x0);
    rs_in = dp_rsrc(P.seg[0].p + (int64_t)b * P.seg[0].bs, img_bytes);
    const int r = tid / DP_PC, c = tid - r * DP_PC;
    const int gy = y0 - 1 + r, gx = x0 - 1 + c;
    vpos = (tid < DP_CH && gy >= 0 && gy < H && gx >= 0 && gx < W) ? (uint32_t)(gy * W + gx) * 4u : DP_OOB;
  };
  auto gload = [&](int g) {
    const int n = g / KS, k = g - n * KS;
    if (k == 0) set_block(n);
    if (tid < DP_CH) {
      uint32_t so = (uint32_t)(DP_KC * k) * hw4;
      dp_opaque(so);
#pragma unroll
      for (int q = 0; q < DP_KC; ++q) {
        rin[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_in, vpos, so, 0));
        so += hw4;
        dp_opaque(so);
      }
    }
#pragma unroll
    for (int q = 0; q < NWL; ++q) {
      const int c = tid + q * DP_THREADS;
      if (NWQ % DP_THREADS == 0 || c < NWQ) {
        const int row = c >> 3, g8 = c & 7;
        const _Float16* src = (g8 < 4 ? wh : wl) + (int64_t)min(row, P.Cout - 1) * cin_pad + DP_KC * k + 8 * (g8 & 3);
        rw[q] = *reinterpret_cast<const u32x4*>(src);
      }
    }
  };
  auto lstore = [&](int g) {
    if (tid < DP_CH) {
      float* pin = sin + (g & 1) * DP_PSZ + tid;
#pragma unroll
      for (int q = 0; q < DP_KC; ++q) pin[q * DP_CH] = rin[q];
    }
    char* pw = sw + (g & 1) * WSZ;
#pragma unroll
    for (int q = 0; q < NWL; ++q) {
      const int c = tid + q * DP_THREADS;
      if (NWQ % DP_THREADS == 0 || c < NWQ) {
        const int row = c >> 3, g8 = c & 7;
        *reinterpret_cast<u32x4*>(pw + row * 128 + ((g8 ^ dp_swz(row)) << 4)) = rw[q];
      }
    }
  };

  gload(0);
  lstore(0);
  if (G > 1) gload(1);

  const float4* sdw4 = reinterpret_cast<const float4*>(sdw + (8 * h) * DP_DWP);  // this half's channels
  const int swz = dp_swz(l32);  // rows 32c + l32 share the swizzle of l32
  bool bad = false;
  for (int n = 0; n < nmine; ++n) {
  floatx16 acc[CT];
#pragma unroll
  for (int c = 0; c < CT; ++c)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.0f;
#pragma unroll 1
  for (int k = 0; k < KS; ++k) {
    const int g = n * KS + k;
    DP_TR(8 * g + 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // step g's slot complete; step g-1's reads of the other slot done
    asm volatile("" ::: "memory");
    DP_TR(8 * g + 1);
    if (g + 1 < G) lstore(g + 1);
    DP_TR(8 * g + 2);
    if (g + 2 < G) gload(g + 2);
    DP_TR(8 * g + 3);
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      // depthwise 3x3 of channels 32k + 16sub + 8h + i at (row y0 + wave, column x0 + l32)
      const float* pin = sin + (g & 1) * DP_PSZ + (16 * sub + 8 * h) * DP_CH + wave * DP_PC + l32;
      half8 bh, bl;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4* wq = sdw4 + (DP_KC * k + 16 * sub + i) * 3;
        const float4 w0 = wq[0], w1 = wq[1], w2 = wq[2];
        const float tw[10] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y};
        const float* pc = pin + i * DP_CH;
        float a = 0.0f;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) a = fmaf(tw[3 * dy + dx], pc[dy * DP_PC + dx], a);
        const float v = a + tw[9];
        const _Float16 hv = (_Float16)v;
        bh[i] = hv;
        bl[i] = (_Float16)(v - (float)hv);
      }
      const int gh = (2 * sub + h) ^ swz, gl = (4 + 2 * sub + h) ^ swz;  // A-fragment granules
      const char* pw = sw + (g & 1) * WSZ + l32 * 128;
#pragma unroll
      for (int c = 0; c < CT; c += 2) {
        const int c1 = (c + 1 < CT) ? c + 1 : c;
        const half8 ah0 = *reinterpret_cast<const half8*>(pw + c * 32 * 128 + (gh << 4));
        const half8 al0 = *reinterpret_cast<const half8*>(pw + c * 32 * 128 + (gl << 4));
        const half8 ah1 = *reinterpret_cast<const half8*>(pw + c1 * 32 * 128 + (gh << 4));
        const half8 al1 = *reinterpret_cast<const half8*>(pw + c1 * 32 * 128 + (gl << 4));
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al0, bh, acc[c], 0, 0, 0);
        if (c1 != c) acc[c1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al1, bh, acc[c1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0, bl, acc[c], 0, 0, 0);
        if (c1 != c) acc[c1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1, bl, acc[c1], 0, 0, 0);
        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah0, bh, acc[c], 0, 0, 0);
        if (c1 != c) acc[c1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah1, bh, acc[c1], 0, 0, 0);
      }
    }
  }

    DP_TR(8 * (n * KS + KS - 1) + 4);
    // epilogue (pw_resident's): bias, range guard, GELU, residual, one row of 32 columns per wave
    int b, y0, x0;
    block_of(n, b, y0, x0);
    const int y = y0 + wave, x = x0 + l32;
    if (y >= H || x >= W) continue;
    const uint32_t cs4 = (uint32_t)P.out_cs * 4u;
    const uint32_t vo_out = (uint32_t)(y * W + x) * 4u + (uint32_t)(4 * h) * cs4;
    const auto rs_out = dp_rsrc(P.out + (int64_t)b * P.out_bs, (uint32_t)P.Cout * cs4);
    const auto rs_res = dp_rsrc(RES ? P.res + (int64_t)b * P.res_bs : P.out, RES ? (uint32_t)P.Cout * cs4 : 0u);
    const float* sb = sbias + 4 * h;
    const int wexp = P.wexp;
    uint32_t so_o = 0;
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      float xr[16];
      uint32_t oo = so_o;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r > 0) {
          oo += (((r & 3) == 0) ? 5u : 1u) * cs4;  // co_u = 32c + (r&3) + 8(r>>2)
          dp_opaque(oo);
        }
        xr[r] = RES ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_res, vo_out, oo, 0)) : 0.0f;
      }
      oo = so_o;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = c * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (r > 0) {
          oo += (((r & 3) == 0) ? 5u : 1u) * cs4;
          dp_opaque(oo);
        }
        float v = ldexpf(acc[c][r], -wexp);
        v += sb[c * 32 + (r & 3) + 8 * (r >> 2)];
        bad |= !(fabsf(v) <= 3.4e38f);
        if (GELU) v = gelu_erf(v);
        v += xr[r];
        if (c * 32 + 32 <= P.Cout || co < P.Cout)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), rs_out, vo_out, oo, 0);
      }
      so_o += 32 * cs4;
      dp_opaque(so_o);
    }
  }
  range_report(P.rflag, bad);
#ifdef MLIC_DP_TRACE
  if (blockIdx.x == 0 && tid == 0)
    for (int i = 0; i < 512; ++i) g_dp_trace[i] = tr[i];
#endif
}

static int dp_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    HIP_OK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return n;
}

bool dwpw_ok(const ConvParams& P, int cin_pad) {
  if (P.K != 1 || P.stride != 1 || P.pad != 0 || P.nseg != 1 || P.seg[0].C != P.Cin || cin_pad != P.Cin) return false;
  if (P.epi & ~(EPI_GELU | EPI_RES)) return false;
  if (P.Ho != P.H || P.Wo != P.W || P.out_cs != (int64_t)P.H * P.W) return false;
  const int64_t HW = (int64_t)P.H * P.W;
  if ((int64_t)P.Cin * HW * 4 >= (1ll << 31) || (int64_t)P.Cout * HW * 4 >= (1ll << 31)) return false;
  const int ct = (P.Cout + 31) / 32;
  return (P.Cin == 192 && ct == 6) || (P.Cin == 128 && ct == 4) || (P.Cin == 96 && ct == 3) ||
         (P.Cin == 160 && ct == 5);
}

template <int CIN, int CT>
static void launch_dwpw(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                        const float* dwb, hipStream_t st) {
  const int64_t nblk = (int64_t)((P.W + DP_TW - 1) / DP_TW) * ((P.H + DP_WAVES - 1) / DP_WAVES) * P.B;
  const dim3 grid((unsigned)std::min<int64_t>(nblk, (int64_t)dp_num_cus()));
  const bool gelu = (P.epi & EPI_GELU) != 0, res = (P.epi & EPI_RES) != 0;
#define MLIC_DP(G, R) \
  hipLaunchKernelGGL((dwpw_kernel<CIN, CT, G, R>), grid, dim3(DP_THREADS), 0, st, P, wh, wl, cin_pad, dww, dwb)
  if (gelu && res) MLIC_DP(true, true);
  else if (gelu) MLIC_DP(true, false);
  else if (res) MLIC_DP(false, true);
  else MLIC_DP(false, false);
#undef MLIC_DP
  HIP_OK(hipGetLastError());
}

void dwpw_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                  const float* dwb, hipStream_t st) {
  MLIC_CHECK(dwpw_ok(P, cin_pad) && dww, "dwpw: unsupported shape");
  switch (P.Cin) {
    case 192: launch_dwpw<192, 6>(P, wh, wl, cin_pad, dww, dwb, st); break;
    case 160: launch_dwpw<160, 5>(P, wh, wl, cin_pad, dww, dwb, st); break;
    case 128: launch_dwpw<128, 4>(P, wh, wl, cin_pad, dww, dwb, st); break;
    default: launch_dwpw<96, 3>(P, wh, wl, cin_pad, dww, dwb, st); break;
  }
}

}  // namespace mlic
