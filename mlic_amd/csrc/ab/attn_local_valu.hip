// A/B-only kernel family (built with `make AB=1`, not part of the product libmlic_hip.so): the
// round-1 VALU form of LocalContext's 5x5 window attention (context.py:75-107), selected by
// $MLIC_LOCAL_ATTN_VALU=1; the product runs the MFMA kernels of ../attn_local.hip.
#include "../common.h"
#include "../kernels.h"

namespace mlic {

// =============================================================================================
// LocalContext windowed attention.  qkv: [B][3C][H*W] (q = ch [0,C), k = [C,2C), v = [2C,3C)),
// output T: [B][C*25][H*W] with row = (head*hd + d)*25 + query_cell, which is exactly the
// (c', ky, kx) flattening the 5x5 "fusion" conv contracts over.
constexpr int LA_T = 8;                 // 8x8 positions per workgroup
constexpr int LA_HALO = LA_T + 4;       // 12x12 staged cells

template <int HD>
__global__ __launch_bounds__(256) void local_attn_kernel(LocalAttnParams P) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int C = 2 * HD, hd = HD;
  const int H = P.H, W = P.W, HW = H * W;
  const int b = blockIdx.y;
  const int ntx = (W + LA_T - 1) / LA_T;
  const int x0 = (blockIdx.x % ntx) * LA_T, y0 = (blockIdx.x / ntx) * LA_T;
  // stage qkv halo: sm[ch][cell], ch in [0, 3C), cell in [0, 144); zero outside the image
  const float* src = P.qkv + (int64_t)b * P.qkv_bs;
  constexpr int NCELL = LA_HALO * LA_HALO;
  for (int i = threadIdx.x; i < 3 * C * NCELL; i += 256) {
    const int ch = i / NCELL, cell = i - ch * NCELL;
    const int gy = y0 - 2 + cell / LA_HALO, gx = x0 - 2 + cell % LA_HALO;
    sm[i] = (gy >= 0 && gy < H && gx >= 0 && gx < W) ? src[(int64_t)ch * HW + gy * W + gx] : 0.0f;
  }
  float* bias_s = sm + 3 * C * NCELL;  // [2][25][25]
  for (int i = threadIdx.x; i < 2 * 625; i += 256) {
    const int h = i / 625, ij = i - h * 625;
    bias_s[i] = P.rel_table[P.rel_index[ij] * 2 + h];
  }
  __syncthreads();
  const float* qs = sm;
  const float* ks = sm + C * NCELL;
  const float* vs = sm + 2 * C * NCELL;
  const float scale = P.scale;
  // work items: (query cell i, head h, local position) with position fastest
  for (int item = threadIdx.x; item < 25 * 2 * LA_T * LA_T; item += 256) {
    const int pl = item % (LA_T * LA_T);
    const int hh = (item / (LA_T * LA_T)) & 1;
    const int qi = item / (2 * LA_T * LA_T);
    const int ly = pl / LA_T, lx = pl % LA_T;
    const int py = y0 + ly, px = x0 + lx;
    if (py >= H || px >= W) continue;
    const int qky = qi / 5, qkx = qi % 5;
    const int qcell = (ly + qky) * LA_HALO + (lx + qkx);
    const int qgy = py + qky - 2, qgx = px + qkx - 2;
    const bool q_anchor = qgy >= 0 && qgy < H && qgx >= 0 && qgx < W && (((qgy + qgx) & 1) == 1);
    float qv[HD];
#pragma unroll
    for (int d = 0; d < hd; ++d) qv[d] = qs[(d * 2 + hh) * NCELL + qcell] * scale;
    float sc[25];
    float mx = -3.0e38f;
#pragma unroll
    for (int j = 0; j < 25; ++j) {
      const int kcell = (ly + j / 5) * LA_HALO + (lx + j % 5);
      float dot = 0.0f;
#pragma unroll
      for (int d = 0; d < hd; ++d) dot = fmaf(qv[d], ks[(d * 2 + hh) * NCELL + kcell], dot);
      const int kgy = py + j / 5 - 2, kgx = px + j % 5 - 2;
      const bool k_anchor = kgy >= 0 && kgy < H && kgx >= 0 && kgx < W && (((kgy + kgx) & 1) == 1);
      float s = dot + bias_s[hh * 625 + qi * 25 + j];
      s = s + ((q_anchor && k_anchor) ? 0.0f : -100.0f);
      sc[j] = s;
      mx = fmaxf(mx, s);
    }
    float sum = 0.0f;
#pragma unroll
    for (int j = 0; j < 25; ++j) { sc[j] = softmax_exp(sc[j] - mx); sum += sc[j]; }
    const float inv = 1.0f / sum;
#pragma unroll
    for (int j = 0; j < 25; ++j) sc[j] = sc[j] * inv;
    float* dst = P.out + (int64_t)b * P.out_bs + (int64_t)py * W + px;
    for (int d = 0; d < hd; ++d) {
      float o = 0.0f;
#pragma unroll
      for (int j = 0; j < 25; ++j) {
        const int kcell = (ly + j / 5) * LA_HALO + (lx + j % 5);
        o = fmaf(sc[j], vs[(d * 2 + hh) * NCELL + kcell], o);
      }
      dst[(int64_t)((hh * hd + d) * 25 + qi) * HW] = o;
    }
  }
}

void local_attn_valu(const LocalAttnParams& P, hipStream_t st) {
  MLIC_CHECK(P.C % 2 == 0 && P.C / 2 <= 32, "local attention head dim");
  const size_t lds = (size_t)(3 * P.C * LA_HALO * LA_HALO + 2 * 625) * sizeof(float);
  MLIC_CHECK(lds <= 160 * 1024, "local attention LDS");
  const int ntx = (P.W + LA_T - 1) / LA_T, nty = (P.H + LA_T - 1) / LA_T;
  if (P.C == 32) hipLaunchKernelGGL(local_attn_kernel<16>, dim3(ntx * nty, P.B), dim3(256), lds, st, P);
  else if (P.C == 64) hipLaunchKernelGGL(local_attn_kernel<32>, dim3(ntx * nty, P.B), dim3(256), lds, st, P);
  else MLIC_CHECK(false, "LocalContext dim must be 32 or 64");
  HIP_OK(hipGetLastError());
}

}  // namespace mlic
