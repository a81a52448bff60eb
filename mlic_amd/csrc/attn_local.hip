// LocalContext 5x5 window attention (context.py:75-107) on the split-fp16 MFMA pipe.
//
// For every latent pixel p and head, the 25 cells of its 5x5 window attend to each other:
// S = Q K^T * scale + rel-pos bias + checkerboard mask (-100 unless query and key cell are both
// anchors inside the image), P = softmax over keys, O = P V; output row (head*hd + d)*25 + i of the
// unfolded map the 5x5 "fusion" conv contracts over.  Per (pixel, head) that is a 25x25xhd and a
// 25xhdx25 product — one wave does it with v_mfma_f32_32x32x16_f16 (cells padded to 32):
//   S^T = K . Q^T   A = K (lane = key cell j, 8 dims), B = Q^T (lane = query cell i, 8 dims);
//                   the accumulator holds key rows j in registers and query i on the lane, so the
//                   softmax over keys is 16 registers + one exchange with lane ^ 32;
//   O^T = V^T . P^T P^T is used straight from the accumulator as the B operand (registers 8s..8s+7
//                   = k-step s, key order 16s + 8(e>>2) + 4h + (e&3)); A = V^T gathered in that order.
// Every product is split-fp16 (hi.hi + hi.lo + lo.hi, fp32 accumulation) like the conv kernels.
// The workgroup stages the q/k/v channels of its pixel tile plus a 2-cell halo in LDS once.  For
// hd = 16 the tile is a 1 x 32 strip and each head's 400 x 32 output block is staged in LDS and
// written as 128-byte rows (the per-lane results are 25 different rows of one pixel — written
// directly they are 4-byte scattered stores); hd = 32 (MLICPP_S2) uses 8 x 8 tiles, direct stores.
#include "common.h"
#include "kernels.h"

namespace mlic {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

namespace {
// 8 waves: the 120 KB of LDS admits one workgroup per CU, so the block itself must bring 2 waves per SIMD
constexpr int LA_THREADS = 512;
constexpr int LA_WAVES = LA_THREADS / 64;

template <int HD>
struct LaTile {
  static constexpr bool STAGE = HD == 16;
  static constexpr int TH = STAGE ? 1 : 8, TW = STAGE ? 32 : 8;
  static constexpr int LH = TH + 4, LW = TW + 4, NCELL = LH * LW, NPIX = TH * TW;
  static constexpr int OPITCH = NPIX + 1;  // staged output row pitch (conflict-free lane writes)
  static constexpr size_t lds_floats(int C) { return (size_t)3 * C * NCELL + (STAGE ? HD * 25 * OPITCH : 0); }
};

__device__ __forceinline__ void split8(const float (&v)[8], half8& hi, half8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const _Float16 h = (_Float16)v[e];
    hi[e] = h;
    lo[e] = (_Float16)(v[e] - (float)h);
  }
}

__device__ __forceinline__ floatx16 mfma3(const half8& ah, const half8& al, const half8& bh, const half8& bl,
                                          floatx16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, c, 0, 0, 0);
}
}  // namespace

template <int HD>
__global__ __launch_bounds__(LA_THREADS) void local_attn_mfma_kernel(LocalAttnParams P) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  using T = LaTile<HD>;
  constexpr int C = 2 * HD, LT_H = T::TH, LT_W = T::TW, LW = T::LW, NCELL = T::NCELL;
  const int H = P.H, W = P.W, HW = H * W;
  const int b = blockIdx.y;
  const int ntx = (W + LT_W - 1) / LT_W;
  const int x0 = (blockIdx.x % ntx) * LT_W, y0 = (blockIdx.x / ntx) * LT_H;
  const float* src = P.qkv + (int64_t)b * P.qkv_bs;
  {  // all of this thread's loads in flight together, then the stores (see local_attn_packed_kernel)
    constexpr int NSTG = 3 * C * NCELL, NQ = (NSTG + LA_THREADS - 1) / LA_THREADS;
    float stg[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = threadIdx.x + q * LA_THREADS;
      const int ch = i / NCELL, cell = i - ch * NCELL;
      const int gy = y0 - 2 + cell / LW, gx = x0 - 2 + cell % LW;
      stg[q] = (i < NSTG && gy >= 0 && gy < H && gx >= 0 && gx < W) ? src[(int64_t)ch * HW + gy * W + gx] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = threadIdx.x + q * LA_THREADS;
      if (i < NSTG) sm[i] = stg[q];
    }
  }
  float* ostage = sm + 3 * C * NCELL;  // [HD * 25][OPITCH] (STAGE only)
  __syncthreads();
  const float* qs = sm;
  const float* ks = sm + C * NCELL;
  const float* vs = sm + 2 * C * NCELL;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const bool lvalid = l32 < 25;  // this lane's window cell (query i for S^T's B, key j for its A)
  const int cy = lvalid ? l32 / 5 : 0, cx = lvalid ? l32 % 5 : 0;

  // relative-position bias for (query i = l32, key j of register r), both heads: item-invariant
  float bias[2][16];
  int ridx[16];  // the index loads in flight together, then the table loads
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int j = (r & 3) + 8 * (r >> 2) + 4 * h;
    ridx[r] = (lvalid && j < 25) ? P.rel_index[l32 * 25 + j] : -1;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) bias[hh][r] = ridx[r] >= 0 ? P.rel_table[ridx[r] * 2 + hh] : 0.0f;

#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
  for (int pl = wave; pl < T::NPIX; pl += LA_WAVES) {
    const int ly = pl / LT_W, lx = pl - (pl / LT_W) * LT_W;
    const int py = y0 + ly, px = x0 + lx;
    if (py >= H || px >= W) continue;  // wave-uniform
    const int cell = (ly + cy) * LW + (lx + cx);

    // ---- S^T = K Q^T (k = head dims, 16 per MFMA k-step)
    floatx16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.0f;
#pragma unroll
    for (int k0 = 0; k0 < HD; k0 += 16) {
      float kv[8], qv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = (k0 + 8 * h + e) * 2 + hh;  // interleaved head split: channel = d * heads + head
        kv[e] = lvalid ? ks[ch * NCELL + cell] : 0.0f;
        qv[e] = lvalid ? qs[ch * NCELL + cell] * P.scale : 0.0f;
      }
      half8 kh_, kl_, qh_, ql_;
      split8(kv, kh_, kl_);
      split8(qv, qh_, ql_);
      s = mfma3(kh_, kl_, qh_, ql_, s);
    }

    // ---- bias, checkerboard mask, softmax over keys (registers + partner lane)
    const int par = py + px;
    const int qgy = py + cy - 2, qgx = px + cx - 2;
    const bool qa = lvalid && qgy >= 0 && qgy < H && qgx >= 0 && qgx < W && ((par + cy + cx) & 1);
    float mx = -3.0e38f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int jy = j / 5, jx = j - 5 * (j / 5);
      const int kgy = py + jy - 2, kgx = px + jx - 2;
      const bool ka = kgy >= 0 && kgy < H && kgx >= 0 && kgx < W && ((par + jy + jx) & 1);
      const float v = s[r] + bias[hh][r] + ((qa && ka) ? 0.0f : -100.0f);
      s[r] = j < 25 ? v : -3.0e38f;
      mx = fmaxf(mx, s[r]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float sum = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = (r & 3) + 8 * (r >> 2) + 4 * h;
      s[r] = j < 25 ? softmax_exp(s[r] - mx) : 0.0f;
      sum += s[r];
    }
    sum += __shfl_xor(sum, 32);
    const float inv = 1.0f / sum;

    // ---- O^T = V^T P^T (k = keys; P^T registers 8t..8t+7 are k-step t)
    floatx16 o;
#pragma unroll
    for (int r = 0; r < 16; ++r) o[r] = 0.0f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float pv[8], vv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pv[e] = s[8 * t + e] * inv;
        const int j = 16 * t + 8 * (e >> 2) + 4 * h + (e & 3);
        const int jy = j / 5, jx = j - 5 * (j / 5);
        const int d = l32;  // A row = head dim
        vv[e] = (j < 25 && d < HD) ? vs[((d * 2) + hh) * NCELL + (ly + jy) * LW + (lx + jx)] : 0.0f;
      }
      half8 ph, pl_, vh, vl;
      split8(pv, ph, pl_);
      split8(vv, vh, vl);
      o = mfma3(vh, vl, ph, pl_, o);
    }

    // ---- O^T[d][i] -> T row (head * hd + d) * 25 + i at pixel p
    if (lvalid) {
      if constexpr (T::STAGE) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int d = (r & 3) + 8 * (r >> 2) + 4 * h;
          ostage[(d * 25 + l32) * T::OPITCH + pl] = o[r];
        }
      } else {
        float* dst = P.out + (int64_t)b * P.out_bs + (int64_t)py * W + px;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = (r & 3) + 8 * (r >> 2) + 4 * h;
          dst[(int64_t)((hh * HD + d) * 25 + l32) * HW] = o[r];
        }
      }
    }
  }
  if constexpr (T::STAGE) {  // coalesced write of this head's rows (one 32-pixel strip each)
    __syncthreads();
    const int nvalid = min(LT_W, W - x0);
    float* dst = P.out + (int64_t)b * P.out_bs + (int64_t)(hh * HD * 25) * HW + (int64_t)y0 * W + x0;
    for (int idx = threadIdx.x; idx < HD * 25 * T::NPIX; idx += LA_THREADS) {
      const int row = idx / T::NPIX, pix = idx - row * T::NPIX;
      if (pix < nvalid) dst[(int64_t)row * HW + pix] = ostage[row * T::OPITCH + pix];
    }
    __syncthreads();
  }
  }
}

// ---------------------------------------------------------------------------------------------
// hd = 16 (MLICPP_L/M/S): the same attention, writing the fusion conv's B operand directly in
// conv_x4's packed split layout  out[b][i][pos][64 halves]: chunk = query cell i (25 chunks),
// channel k = head*16 + d (hi at k, lo at 32 + k), pos = flat pixel (K = 1 folding of conv_x4).
// The fusion weights are permuted to that order once at load (k' = i*32 + head*16 + d), so the
// 5x5 "fusion" conv runs on conv_x4 with no fp32 round trip of the 800-row map and no packing pass.
// Both heads are processed in one pass (two independent MFMA / softmax chains per pixel); loads
// are branch-free (lanes outside the 25-cell window read a zero cell), q is pre-scaled at staging.
#ifndef MLIC_LA_STAGE_V1  // A/B build: 1 = the element-per-thread staging of rounds 4-5
#define MLIC_LA_STAGE_V1 0
#endif
namespace {
constexpr int LP_TW = 32, LP_LW = LP_TW + 4, LP_NCELL = 5 * LP_LW, LP_NCP = LP_NCELL + 1;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t la_rsrc(const float* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}
// key cell j of S^T accumulator register r in lane half h; its mask tables
constexpr int la_j(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
constexpr uint32_t la_jbits(int h) {
  uint32_t b = 0;
  for (int r = 0; r < 16; ++r) b |= la_j(r, h) < 25 ? 1u << r : 0u;
  return b;
}
constexpr uint32_t la_kbits(int h, int par) {  // key cells that are anchors at pixel parity par
  uint32_t b = 0;
  for (int r = 0; r < 16; ++r) {
    const int j = la_j(r, h);
    b |= (j < 25 && ((j / 5 + j % 5 + 1) & 1) == par) ? 1u << r : 0u;  // (par + jy + jx) odd
  }
  return b;
}
constexpr int la_voff(int t, int e, int h) {  // window-cell offset of key 16t + 8(e>>2) + 4h + (e&3), -1 past 25
  const int j = 16 * t + 8 * (e >> 2) + 4 * h + (e & 3);
  return j < 25 ? (j / 5) * LP_LW + j % 5 : -1;
}
}

// Operands are split once at staging (not per use): q (pre-scaled) and k as [head][hi|lo][cell][16 d]
// (a lane's 8 dims of one cell are one 16-byte read per half), v as hi / lo planes [head*16 + d][cell]
// gathered 2 bytes at a time straight into the fragment.  Interior pixels take the checkerboard /
// window mask from per-lane bit masks (parity only); the two rows / columns at the border compute
// the in-image tests.
__global__ __launch_bounds__(LA_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void local_attn_packed_kernel(LocalAttnParams P, _Float16* __restrict__ outp,
                                                                     int npos) {
  constexpr int QKP = LP_NCP * 16;       // halves per (tensor, head, hi|lo) plane
  constexpr int QK_H = 2 * 2 * 2 * QKP;  // q, k x heads x hi|lo
  constexpr int VP = 32 * LP_NCP;        // v as (hi, lo) half pairs, one 32-bit word per (channel, cell)
  __shared__ __attribute__((aligned(16))) _Float16 sm[QK_H + 2 * VP];
  // relative-position bias of (query l32, key j of register r), per lane: [head][r][lane] (8 KB;
  // held in registers it pushed the kernel past 128 VGPRs, i.e. one workgroup per CU)
  __shared__ float sbias[2 * 16 * 64];
  const int H = P.H, W = P.W, HW = H * W;
  const int b = blockIdx.y;
  const int ntx = (W + LP_TW - 1) / LP_TW;
  const int x0 = (blockIdx.x % ntx) * LP_TW, y0 = blockIdx.x / ntx;
  const float* src = P.qkv + (int64_t)b * P.qkv_bs;
#if MLIC_LA_STAGE_V1
  // all of this thread's staging loads first (independent, in flight together), then the stores:
  // a load -> convert -> store loop serialises one full memory latency per element
  constexpr int NSTG = 3 * 32 * LP_NCP, NQ = (NSTG + LA_THREADS - 1) / LA_THREADS;
  float stg[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int i = threadIdx.x + q * LA_THREADS;
    const int ch = i / LP_NCP, cell = i - ch * LP_NCP;
    stg[q] = 0.0f;
    if (i < NSTG && cell < LP_NCELL) {
      const int gy = y0 - 2 + cell / LP_LW, gx = x0 - 2 + cell % LP_LW;
      if (gy >= 0 && gy < H && gx >= 0 && gx < W) stg[q] = src[(int64_t)ch * HW + gy * W + gx];
    }
  }
  for (int i = threadIdx.x; i < 2 * 16 * 64; i += LA_THREADS) {
    const int hh = i >> 10, r = (i >> 6) & 15, ln = i & 63, q32 = ln & 31;
    const int j = (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
    sbias[i] = (q32 < 25 && j < 25) ? P.rel_table[P.rel_index[q32 * 25 + j] * 2 + hh] : 0.0f;
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int i = threadIdx.x + q * LA_THREADS;
    if (i >= NSTG) break;
    const int ch = i / LP_NCP, cell = i - ch * LP_NCP;
    float v = stg[q];
    if (ch < 32) v *= P.scale;
    const _Float16 hv = (_Float16)v, lv = (_Float16)(v - (float)hv);
    const int which = ch >> 5, c = ch & 31, d = c >> 1, hh = c & 1;  // channel = d * heads + head
    if (which < 2) {
      _Float16* dst = sm + ((which * 2 + hh) * 2) * QKP + cell * 16 + d;
      dst[0] = hv;
      dst[QKP] = lv;
    } else {
      reinterpret_cast<uint32_t*>(sm + QK_H)[(hh * 16 + d) * LP_NCP + cell] =
          (uint32_t)__builtin_bit_cast(uint16_t, hv) | ((uint32_t)__builtin_bit_cast(uint16_t, lv) << 16);
    }
  }
#else
  // thread t < 2 * LP_NCP stages window cell t % LP_NCP of the 48 channels of head t / LP_NCP
  // (channel = d * heads + head, so channel c0 + 2q is tensor q >> 4, dim q & 15): one bounds test per
  // thread, the 48 loads branch-free (an out-of-image cell reads 0 through an out-of-range buffer
  // offset; the channel is the scalar offset) and in flight together, then q / k as two 16-byte hi and
  // two lo rows and v as (hi, lo) words.  (Element per thread, the form before round 6: a bounds test,
  // a branch and two 2-byte LDS stores per element -- 40 % of the kernel's VALU instructions.)
  if (threadIdx.x < 2 * LP_NCP) {
    const int c0 = threadIdx.x >= LP_NCP ? 1 : 0, cell = (int)threadIdx.x - c0 * LP_NCP;
    const int gy = y0 - 2 + cell / LP_LW, gx = x0 - 2 + cell % LP_LW;
    const bool in = cell < LP_NCELL && gy >= 0 && gy < H && gx >= 0 && gx < W;
    const __amdgpu_buffer_rsrc_t rs = la_rsrc(src, (uint32_t)(96 * HW) * 4u);
    const uint32_t vo = in ? (uint32_t)(c0 * HW + gy * W + gx) * 4u : 0x80000000u;
    float v[48];
#pragma unroll
    for (int q = 0; q < 48; ++q)
      v[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, (uint32_t)(2 * q * HW) * 4u, 0));
#pragma unroll
    for (int t = 0; t < 2; ++t) {  // q (pre-scaled), k
      half8 hv[2], lv[2];
#pragma unroll
      for (int d = 0; d < 16; ++d) {
        const float x = t == 0 ? v[d] * P.scale : v[16 + d];
        const _Float16 hx = (_Float16)x;
        hv[d >> 3][d & 7] = hx;
        lv[d >> 3][d & 7] = (_Float16)(x - (float)hx);
      }
      _Float16* dst = sm + ((t * 2 + c0) * 2) * QKP + cell * 16;
      *reinterpret_cast<half8*>(dst) = hv[0];
      *reinterpret_cast<half8*>(dst + 8) = hv[1];
      *reinterpret_cast<half8*>(dst + QKP) = lv[0];
      *reinterpret_cast<half8*>(dst + QKP + 8) = lv[1];
    }
    uint32_t* vdst = reinterpret_cast<uint32_t*>(sm + QK_H) + c0 * 16 * LP_NCP + cell;
#pragma unroll
    for (int d = 0; d < 16; ++d) {
      const float x = v[32 + d];
      const _Float16 hx = (_Float16)x, lx_ = (_Float16)(x - (float)hx);
      vdst[d * LP_NCP] =
          (uint32_t)__builtin_bit_cast(uint16_t, hx) | ((uint32_t)__builtin_bit_cast(uint16_t, lx_) << 16);
    }
  }
  for (int i = threadIdx.x; i < 2 * 16 * 64; i += LA_THREADS) {
    const int hh = i >> 10, r = (i >> 6) & 15, ln = i & 63, q32 = ln & 31;
    const int j = (r & 3) + 8 * (r >> 2) + 4 * (ln >> 5);
    sbias[i] = (q32 < 25 && j < 25) ? P.rel_table[P.rel_index[q32 * 25 + j] * 2 + hh] : 0.0f;
  }
#endif
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const bool lvalid = l32 < 25;
  const int cy = lvalid ? l32 / 5 : 0, cx = lvalid ? l32 % 5 : 0;
  // interior mask bits for pixel parity 0 / 1: register r allowed iff query and key cell are anchors
  // (compile-time tables per lane half h, selected once: no per-lane division by 5)
  const uint32_t jbits = h ? la_jbits(1) : la_jbits(0);
  const uint32_t kbits[2] = {h ? la_kbits(1, 0) : la_kbits(0, 0), h ? la_kbits(1, 1) : la_kbits(0, 1)};
  bool qok[2];
  qok[0] = lvalid && ((cy + cx) & 1);
  qok[1] = lvalid && !((cy + cx) & 1);
  // V^T gather: key j of element e of k-step t, as a window-cell offset (-1: outside the window or
  // a padding row d >= 16 of the 32-row fragment)
  int voff[2][8];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) voff[t][e] = l32 < 16 ? (h ? la_voff(t, e, 1) : la_voff(t, e, 0)) : -1;
  const int vrow = l32 & 15;

  // ckbd: this row's pixels of one checkerboard phase only (x0 is even, so a fixed column parity)
  const int xoff = P.ckbd ? ((y0 + (P.ckbd == 1 ? 1 : 0)) & 1) : 0;
  const int nlx = P.ckbd ? LP_TW / 2 : LP_TW;
  for (int k = wave; k < nlx; k += LA_WAVES) {
    const int lx = P.ckbd ? 2 * k + xoff : k;
    const int px = x0 + lx, py = y0;
    if (px >= W) break;  // wave-uniform
    const int qcell = lvalid ? cy * LP_LW + lx + cx : LP_NCELL;
    const int par = (py + px) & 1;
    const bool interior = py >= 2 && py < H - 2 && px >= 2 && px < W - 2;  // wave-uniform
    // allowed(r): interior = parity bits; border = the in-image tests of the reference's unfold
    uint32_t allow;
    if (interior) {
      allow = qok[par] ? kbits[par] : 0u;
    } else {
      const int qgy = py + cy - 2, qgx = px + cx - 2;
      const bool qa = lvalid && qgy >= 0 && qgy < H && qgx >= 0 && qgx < W && ((par + cy + cx) & 1);
      allow = 0u;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int jy = h ? la_j(r, 1) / 5 : la_j(r, 0) / 5, jx = h ? la_j(r, 1) % 5 : la_j(r, 0) % 5;
        const int kgy = py + jy - 2, kgx = px + jx - 2;
        const bool ka = kgy >= 0 && kgy < H && kgx >= 0 && kgx < W && ((par + jy + jx) & 1);
        allow |= (qa && ka && ((jbits >> r) & 1u)) ? (1u << r) : 0u;
      }
    }
    const int64_t pos = P.ckbd ? ((int64_t)py * W + px) >> 1 : (int64_t)py * W + px;
    _Float16* dst = outp + (((int64_t)b * 25 + l32) * npos + pos) * 64;
    // one head at a time, start to store: only one S and one O accumulator live (<= 128 VGPRs, so
    // two workgroups share a CU and one's staging overlaps the other's products)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      // S^T = K Q^T over the 16 head dims (lane half h holds dims 8h .. 8h+7)
      const _Float16* kp = sm + ((1 * 2 + hh) * 2) * QKP + qcell * 16 + 8 * h;
      const _Float16* qp = sm + ((0 * 2 + hh) * 2) * QKP + qcell * 16 + 8 * h;
      const half8 kh_ = *reinterpret_cast<const half8*>(kp), kl_ = *reinterpret_cast<const half8*>(kp + QKP);
      const half8 qh_ = *reinterpret_cast<const half8*>(qp), ql_ = *reinterpret_cast<const half8*>(qp + QKP);
      floatx16 sacc, oacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) sacc[r] = 0.0f;
      sacc = mfma3(kh_, kl_, qh_, ql_, sacc);
      float mx = -3.0e38f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = sacc[r] + sbias[(hh * 16 + r) * 64 + lane] + (((allow >> r) & 1u) ? 0.0f : -100.0f);
        sacc[r] = ((jbits >> r) & 1u) ? v : -3.0e38f;
        mx = fmaxf(mx, sacc[r]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      float sum = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = ((jbits >> r) & 1u) ? softmax_exp(sacc[r] - mx) : 0.0f;
        sum += sacc[r];
      }
      sum += __shfl_xor(sum, 32);
      const float inv = 1.0f / sum;
      // O^T = V^T P^T (k = keys; P^T registers 8t .. 8t+7 are k-step t)
#pragma unroll
      for (int r = 0; r < 16; ++r) oacc[r] = 0.0f;
      const uint32_t* vp_p = reinterpret_cast<const uint32_t*>(sm + QK_H) + (hh * 16 + vrow) * LP_NCP;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float pv[8];
        half8 vh, vl;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          pv[e] = sacc[8 * t + e] * inv;
          const int c = voff[t][e] >= 0 ? voff[t][e] + lx : LP_NCELL;
          const uint32_t hl = vp_p[c];  // one read for both halves
          vh[e] = __builtin_bit_cast(_Float16, (uint16_t)(hl & 0xffffu));
          vl[e] = __builtin_bit_cast(_Float16, (uint16_t)(hl >> 16));
        }
        half8 ph, pl_;
        split8(pv, ph, pl_);
        oacc = mfma3(vh, vl, ph, pl_, oacc);
      }
      // O^T[d][i]: registers 0..3 are d = 4h .. 4h+3, registers 4..7 are d = 8 + 4h .. +3 of query i
      if (lvalid) {
        typedef _Float16 half4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          half4 hi, lo;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = oacc[4 * g + e];
            const _Float16 hv = (_Float16)v;
            hi[e] = hv;
            lo[e] = (_Float16)(v - (float)hv);
          }
          const int k = hh * 16 + 8 * g + 4 * h;
          *reinterpret_cast<half4*>(dst + k) = hi;
          *reinterpret_cast<half4*>(dst + 32 + k) = lo;
        }
      }
    }
  }
}

void local_attn_packed(const LocalAttnParams& P, _Float16* out, int npos, hipStream_t st) {
  MLIC_CHECK(P.C == 32, "packed LocalContext attention: dim 32 (2 heads x 16)");
  MLIC_CHECK(P.ckbd == 0 || (P.ckbd <= 2 && P.W % 2 == 0), "packed attention: checkerboard half needs W even");
  MLIC_CHECK(npos >= (P.ckbd ? P.H * P.W / 2 : P.H * P.W), "packed output positions");
  const int ntx = (P.W + LP_TW - 1) / LP_TW;
  hipLaunchKernelGGL(local_attn_packed_kernel, dim3(ntx * P.H, P.B), dim3(LA_THREADS), 0, st, P, out, npos);
  HIP_OK(hipGetLastError());
}

template <int HD>
static void launch_la(const LocalAttnParams& P, hipStream_t st) {
  using T = LaTile<HD>;
  const size_t lds = T::lds_floats(P.C) * sizeof(float);
  MLIC_CHECK(lds <= 160 * 1024, "local attention LDS");
  const int ntx = (P.W + T::TW - 1) / T::TW, nty = (P.H + T::TH - 1) / T::TH;
  hipLaunchKernelGGL(local_attn_mfma_kernel<HD>, dim3(ntx * nty, P.B), dim3(LA_THREADS), lds, st, P);
  HIP_OK(hipGetLastError());
}

void local_attn_mfma(const LocalAttnParams& P, hipStream_t st) {
  if (P.C == 32) launch_la<16>(P, st);
  else if (P.C == 64) launch_la<32>(P, st);
  else MLIC_CHECK(false, "LocalContext dim must be 32 or 64");
}

}  // namespace mlic
