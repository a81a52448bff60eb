// Bandwidth-bound and small-reduction kernels of the MLIC++ hot path (gfx950).
//
//  dw3x3 ............ DepthWiseConv's depthwise half (conv.py:46-63), stride 1/2, LDS halo tile,
//                     multi-segment (channel-concat) input, optional GELU
//  ln_channels ...... nn.LayerNorm over channels of an NCHW map (context.py:73, 110)
//  local_attn ....... LocalContext windowed 5x5 attention (context.py:75-107): q/k/v halo tile in
//                     LDS, Swin relative-position bias, checkerboard mask computed from parity bits
//  ctx_partial/reduce softmax_L(K).V^T over L as a split reduction with a max-rescaled fixed-order
//                     combine (F.softmax(keys, dim=L), context.py:180, 235, never materialised)
//  attn_apply ....... ctx^T . softmax_c(Q) (context.py:181, 187, 236, 239)
//  quant / likelihood / indexes / dequant: ste_round, GaussianConditional, build_indexes,
//                     checkerboard phases (mlicpp.py:112-138, ckbd.py:123-220)
//  eb_forward ....... EntropyBottleneck factorized likelihood + median rounding (compressai)
#include "common.h"
#include "kernels.h"

#include <cstdlib>

namespace mlic {

// =============================================================================================
// depthwise 3x3, pad 1.  One workgroup = one (image, channel) plane tile; the input tile with its
// halo is staged in LDS with coalesced row loads, and each thread produces a 4-wide strip of
// outputs (float4 store) from a 3 x (4*s + 2) register window, so every staged value is reused.
constexpr int DW_TW = 128;  // output tile width
constexpr int DW_TH1 = 32;  // output tile height, stride 1
constexpr int DW_TH2 = 16;  // output tile height, stride 2

template <int S>
__global__ __launch_bounds__(256) void dw3x3_kernel(DwParams P) {
  constexpr int TH = S == 1 ? DW_TH1 : DW_TH2;
  constexpr int TWI = DW_TW * S + 2, THI = TH * S + 2;
  constexpr int PITCH = TWI + 1;
  __shared__ float tile[THI * PITCH];
  const int c = blockIdx.y, b = blockIdx.z;
  const int ntx = (P.Wo + DW_TW - 1) / DW_TW;
  const int tx = blockIdx.x % ntx, ty = blockIdx.x / ntx;
  const int ox0 = tx * DW_TW, oy0 = ty * TH;
  const int ix0 = ox0 * S - 1, iy0 = oy0 * S - 1;
  int sg = 0, c0 = 0;
  while (sg + 1 < P.nseg && c >= c0 + P.seg[sg].C) { c0 += P.seg[sg].C; ++sg; }
  const float* src = P.seg[sg].p + (int64_t)b * P.seg[sg].bs + (int64_t)(c - c0) * P.H * P.W;
  {  // the patch loads in flight together, then the stores (a load -> store loop serialises them)
    constexpr int NQ = (TWI * THI + 255) / 256;
    float stg[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int yy = i / TWI, xx = i - yy * TWI;
      const int gy = iy0 + yy, gx = ix0 + xx;
      stg[q] = (i < TWI * THI && gy >= 0 && gy < P.H && gx >= 0 && gx < P.W) ? src[(int64_t)gy * P.W + gx] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int i = threadIdx.x + 256 * q;
      const int yy = i / TWI, xx = i - yy * TWI;
      if (i < TWI * THI) tile[yy * PITCH + xx] = stg[q];
    }
  }
  __syncthreads();
  float w[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) w[k] = P.w[c * 9 + k];
  const float bias = P.bias ? P.bias[c] : 0.0f;
  float* dst = P.out + (int64_t)b * P.out_bs + (int64_t)c * P.Ho * P.Wo;
  const bool vec = (P.Wo & 3) == 0;
  // 32 strips of 4 outputs per row; 256 threads cover 8 rows per pass
  const int xs = (threadIdx.x & 31) * 4;
  for (int ly = threadIdx.x >> 5; ly < TH; ly += 8) {
    const int oy = oy0 + ly;
    if (oy >= P.Ho) break;
    float win[3][4 * S + 2];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int j = 0; j < 4 * S + 2; ++j) win[ky][j] = tile[(ly * S + ky) * PITCH + xs * S + j];
    float o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float acc = 0.0f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc = fmaf(w[ky * 3 + kx], win[ky][q * S + kx], acc);
      float v = acc + bias;
      if (P.gelu) v = gelu_epi(v);
      o[q] = v;
    }
    const int ox = ox0 + xs;
    float* d = dst + (int64_t)oy * P.Wo + ox;
    if (vec && ox + 3 < P.Wo) {
      *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (ox + q < P.Wo) d[q] = o[q];
    }
  }
}

// stride-1 fast path: 32x128 output tile, the (34 x 136)-float input patch staged with aligned
// float4 loads (patch column 0 = input column ox0 - 4, so each float4 is wholly inside or outside
// the image when W % 4 == 0), and each thread computes a 4x4 output block from a sliding 3-row
// register window: 6 patch rows x (1 float4 + 2 scalars) LDS reads for 16 outputs.
// RPT rows per thread: tile height 8 * RPT (32, or 24 where it pads less, e.g. the 68-row latent)
constexpr int DWF_TW = 128, DWF_PQ = DWF_TW / 4 + 2;  // float4s per patch row
template <int RPT>
__global__ __launch_bounds__(256) void dw3x3_s1_vec_kernel(DwParams P) {
  constexpr int DWF_TH = 8 * RPT, DWF_PR = DWF_TH + 2;
  __shared__ float4 tile[DWF_PR * DWF_PQ];
  const int c = blockIdx.y, b = blockIdx.z;
  const int ntx = (P.Wo + DWF_TW - 1) / DWF_TW;
  const int ox0 = (blockIdx.x % ntx) * DWF_TW, oy0 = (blockIdx.x / ntx) * DWF_TH;
  int sg = 0, c0 = 0;
  while (sg + 1 < P.nseg && c >= c0 + P.seg[sg].C) { c0 += P.seg[sg].C; ++sg; }
  const float* src = P.seg[sg].p + (int64_t)b * P.seg[sg].bs + (int64_t)(c - c0) * P.H * P.W;
  const int W4 = P.W >> 2;
  const float4* src4 = reinterpret_cast<const float4*>(src);
  {  // the patch loads in flight together, then the stores
    constexpr int NQ = (DWF_PR * DWF_PQ + 255) / 256;
    float4 stg[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int r = i / DWF_PQ, q = i - r * DWF_PQ;
      const int gy = oy0 - 1 + r, gq = (ox0 >> 2) - 1 + q;  // float4 column
      stg[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < DWF_PR * DWF_PQ && gy >= 0 && gy < P.H && gq >= 0 && gq < W4) stg[k] = src4[(int64_t)gy * W4 + gq];
    }
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < DWF_PR * DWF_PQ) tile[i] = stg[k];
    }
  }
  __syncthreads();
  float w[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) w[k] = P.w[c * 9 + k];
  const float bias = P.bias ? P.bias[c] : 0.0f;
  const int cg = threadIdx.x & 31, rg = threadIdx.x >> 5;  // 4 columns x 4 rows per thread
  const float* tf = reinterpret_cast<const float*>(tile);
  constexpr int PITCH = DWF_PQ * 4;
  // window rows: input cols 4cg-1 .. 4cg+4  <->  patch cols 4cg+3 .. 4cg+8
  float win[3][6];
  auto load_row = [&](int pr, float* dst) {
    const float* rp = tf + pr * PITCH + 4 * cg + 3;
    const float4 m = tile[pr * DWF_PQ + cg + 1];
    dst[0] = rp[0];
    dst[1] = m.x; dst[2] = m.y; dst[3] = m.z; dst[4] = m.w;
    dst[5] = rp[5];
  };
  load_row(RPT * rg, win[0]);
  load_row(RPT * rg + 1, win[1]);
  float* dst = P.out + (int64_t)b * P.out_bs + (int64_t)c * P.Ho * P.Wo;
  const int ox = ox0 + 4 * cg;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    load_row(RPT * rg + r + 2, win[(r + 2) % 3]);
    float o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float acc = 0.0f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc = fmaf(w[ky * 3 + kx], win[(r + ky) % 3][q + kx], acc);
      float v = acc + bias;
      if (P.gelu) v = gelu_epi(v);
      o[q] = v;
    }
    const int oy = oy0 + RPT * rg + r;
    if (oy < P.Ho && ox < P.Wo)  // Wo % 4 == 0: a strip is wholly inside or outside
      *reinterpret_cast<float4*>(dst + (int64_t)oy * P.Wo + ox) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// stride-2 fast path: 16x64 output tile from a (33 x 136)-float patch (patch column 0 = input
// column 2*ox0 - 4, aligned float4 loads); each thread makes 4 horizontally adjacent outputs from
// 3 rows x 9 inputs (two float4 + one scalar LDS read per row).
constexpr int DW2_TH = 16, DW2_TW = 64, DW2_PR = 2 * DW2_TH + 1, DW2_PQ = 2 * DW2_TW / 4 + 2;
__global__ __launch_bounds__(256) void dw3x3_s2_vec_kernel(DwParams P) {
  __shared__ float4 tile[DW2_PR * DW2_PQ];
  const int c = blockIdx.y, b = blockIdx.z;
  const int ntx = (P.Wo + DW2_TW - 1) / DW2_TW;
  const int ox0 = (blockIdx.x % ntx) * DW2_TW, oy0 = (blockIdx.x / ntx) * DW2_TH;
  int sg = 0, c0 = 0;
  while (sg + 1 < P.nseg && c >= c0 + P.seg[sg].C) { c0 += P.seg[sg].C; ++sg; }
  const float* src = P.seg[sg].p + (int64_t)b * P.seg[sg].bs + (int64_t)(c - c0) * P.H * P.W;
  const int W4 = P.W >> 2;
  const float4* src4 = reinterpret_cast<const float4*>(src);
  {  // the patch loads in flight together, then the stores
    constexpr int NQ = (DW2_PR * DW2_PQ + 255) / 256;
    float4 stg[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int r = i / DW2_PQ, q = i - r * DW2_PQ;
      const int gy = 2 * oy0 - 1 + r, gq = (2 * ox0 >> 2) - 1 + q;
      stg[k] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < DW2_PR * DW2_PQ && gy >= 0 && gy < P.H && gq >= 0 && gq < W4) stg[k] = src4[(int64_t)gy * W4 + gq];
    }
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < DW2_PR * DW2_PQ) tile[i] = stg[k];
    }
  }
  __syncthreads();
  float w[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) w[k] = P.w[c * 9 + k];
  const float bias = P.bias ? P.bias[c] : 0.0f;
  const int cg = threadIdx.x & 15, ry = threadIdx.x >> 4;  // outputs (oy0 + ry, ox0 + 4cg .. +3)
  const float* tf = reinterpret_cast<const float*>(tile);
  constexpr int PITCH = DW2_PQ * 4;
  float o[4] = {bias, bias, bias, bias};
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    // input cols 8cg-1 .. 8cg+7  <->  patch cols 8cg+3 .. 8cg+11
    const int pr = 2 * ry + ky;
    const float4 m0 = tile[pr * DW2_PQ + 2 * cg + 1], m1 = tile[pr * DW2_PQ + 2 * cg + 2];
    const float in[9] = {tf[pr * PITCH + 8 * cg + 3], m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) o[q] = fmaf(w[ky * 3 + kx], in[2 * q + kx], o[q]);
  }
  if (P.gelu) {
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = gelu_epi(o[q]);
  }
  const int oy = oy0 + ry, ox = ox0 + 4 * cg;
  if (oy < P.Ho && ox < P.Wo)
    *reinterpret_cast<float4*>(P.out + (int64_t)b * P.out_bs + (int64_t)c * P.Ho * P.Wo + (int64_t)oy * P.Wo + ox) =
        make_float4(o[0], o[1], o[2], o[3]);
}

// stride-1 form for narrow planes (W / 4 <= 16 float4 columns, the Kodak-size latent): no LDS, no barrier.
// Lane = one float4 column group of one row strip (a wave holds 64 / (W / 4) strips side by side);
// each lane loads its R + 2 rows at once (dwordx4 each) and walks down them with a 3-row window; its horizontal neighbours (column 4q - 1 = lane - 1's .w, 4q + 4 = lane + 1's .x) arrive by
// DPP wave shifts, zeroed at the plane's edges.  Sum order = dw3x3_s1_vec_kernel's (acc = 0, taps
// row-major by fma, + bias [, GELU]): bit-identical.
constexpr int DWS_WAVES = 4;
__device__ __forceinline__ float dws_shr(float v) {  // lane - 1
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ float dws_shl(float v) {  // lane + 1
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130, 0xF, 0xF, true));
}
template <int R>
__global__ __launch_bounds__(64 * DWS_WAVES) void dw3x3_s1_strip_kernel(DwParams P, int nstrip) {
  const int lane = threadIdx.x & 63;
  const int W4 = P.W >> 2, spw = 64 / W4;
  const int k = lane / W4, q = lane - k * W4;
  const int64_t strip = ((int64_t)blockIdx.x * DWS_WAVES + (threadIdx.x >> 6)) * spw + k;
  const int64_t nall = (int64_t)P.B * P.C * nstrip;
  const bool live = k < spw && strip < nall;  // dead lanes still run (their DPP sources), never store
  const int64_t st = live ? strip : 0;
  const int plane = (int)(st / nstrip), si = (int)(st - (int64_t)plane * nstrip);
  const int b = plane / P.C, c = plane - b * P.C;
  int sg = 0, c0 = 0;
  while (sg + 1 < P.nseg && c >= c0 + P.seg[sg].C) { c0 += P.seg[sg].C; ++sg; }
  const float4* src = reinterpret_cast<const float4*>(P.seg[sg].p + (int64_t)b * P.seg[sg].bs +
                                                      (int64_t)(c - c0) * P.H * P.W) + q;
  const int y0 = si * R;
  auto ld = [&](int y) {
    return (live && y >= 0 && y < P.H) ? src[(int64_t)y * W4] : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  float w[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) w[t] = P.w[c * 9 + t];
  const float bias = P.bias ? P.bias[c] : 0.0f;
  float* dst = P.out + (int64_t)b * P.out_bs + (int64_t)c * P.Ho * P.Wo + 4 * q;
  // every row of the strip in flight at once (R + 2 dwordx4 per lane): the plane is small, the
  // latency is what bounds it
  float4 rows[R + 2];
#pragma unroll
  for (int i = 0; i < R + 2; ++i) rows[i] = ld(y0 - 1 + i);
  float win[3][6];
  auto unpack = [&](const float4& v, float* d) {
    const float l = dws_shr(v.w), r = dws_shl(v.x);
    d[0] = q > 0 ? l : 0.0f;
    d[1] = v.x; d[2] = v.y; d[3] = v.z; d[4] = v.w;
    d[5] = q < W4 - 1 ? r : 0.0f;
  };
  unpack(rows[0], win[0]);
  unpack(rows[1], win[1]);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    unpack(rows[r + 2], win[(r + 2) % 3]);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float acc = 0.0f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) acc = fmaf(w[ky * 3 + kx], win[(r + ky) % 3][e + kx], acc);
      float v = acc + bias;
      if (P.gelu) v = gelu_epi(v);
      o[e] = v;
    }
    const int oy = y0 + r;
    if (live && oy < P.Ho) *reinterpret_cast<float4*>(dst + (int64_t)oy * P.Wo) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

static int g_dw_strip = -1;  // -1: $MLIC_DW_STRIP (default on), else the kernel option
void dw_set_strip(int v) { g_dw_strip = v; }
static bool dw_strip_on() {
  if (g_dw_strip >= 0) return g_dw_strip != 0;
  static const bool on = [] {
    const char* e = std::getenv("MLIC_DW_STRIP");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

void dw3x3(const DwParams& P, hipStream_t st) {
  MLIC_CHECK(P.stride == 1 || P.stride == 2, "dw stride");
  MLIC_CHECK(P.Ho == (P.H - 1) / P.stride + 1 && P.Wo == (P.W - 1) / P.stride + 1, "dw output size");
  int tot = 0;
  bool aligned = (P.W % 4) == 0 && (reinterpret_cast<uintptr_t>(P.out) % 16) == 0 && (P.out_bs % 4) == 0;
  for (int i = 0; i < P.nseg; ++i) {
    tot += P.seg[i].C;
    aligned = aligned && (reinterpret_cast<uintptr_t>(P.seg[i].p) % 16) == 0 && (P.seg[i].bs % 4) == 0;
  }
  MLIC_CHECK(tot == P.C, "dw segments");
  // narrow planes (<= 64 columns: the Kodak-size latent, 32 x 48) take the strip form: 10.4 vs 14.1 us
  // for 16 x 224 x 32 x 48 (rocprof); at the 1080p latent (120 columns) both forms are within 2 %
  // (21.2 / 21.6 us for 8 x 224 x 68 x 120, against 17.0 us for a plain copy of the same bytes)
  if (P.stride == 1 && aligned && P.W / 4 <= 16 && dw_strip_on()) {
    // strip height: the fewest loaded rows per plane (R + 2 per strip of R) among 8 / 12 / 17
    const int cand[3] = {8, 12, 17};
    int best = 0;
    int64_t cost = INT64_MAX;
    for (int i = 0; i < 3; ++i) {
      const int n = (P.Ho + cand[i] - 1) / cand[i];
      const int64_t c = (int64_t)n * (cand[i] + 2);
      if (c < cost) { cost = c; best = i; }
    }
    const int R = cand[best], nstrip = (P.Ho + R - 1) / R, spw = 64 / (P.W / 4);
    const int64_t strips = (int64_t)P.B * P.C * nstrip, waves = (strips + spw - 1) / spw;
    const dim3 grid((unsigned)((waves + DWS_WAVES - 1) / DWS_WAVES));
    if (R == 8) hipLaunchKernelGGL(dw3x3_s1_strip_kernel<8>, grid, dim3(64 * DWS_WAVES), 0, st, P, nstrip);
    else if (R == 12) hipLaunchKernelGGL(dw3x3_s1_strip_kernel<12>, grid, dim3(64 * DWS_WAVES), 0, st, P, nstrip);
    else hipLaunchKernelGGL(dw3x3_s1_strip_kernel<17>, grid, dim3(64 * DWS_WAVES), 0, st, P, nstrip);
    HIP_OK(hipGetLastError());
    return;
  }
  if (P.stride == 1 && aligned) {
    const int ntx = (P.Wo + DWF_TW - 1) / DWF_TW;
    // staged rows per tile column: tiles * (TH + 2), the smaller of TH = 32 and TH = 24
    const int n32 = (P.Ho + 31) / 32, n24 = (P.Ho + 23) / 24;
    if (n24 * 26 < n32 * 34) {
      hipLaunchKernelGGL(dw3x3_s1_vec_kernel<3>, dim3(ntx * n24, P.C, P.B), dim3(256), 0, st, P);
    } else {
      hipLaunchKernelGGL(dw3x3_s1_vec_kernel<4>, dim3(ntx * n32, P.C, P.B), dim3(256), 0, st, P);
    }
    HIP_OK(hipGetLastError());
    return;
  }
  if (P.stride == 2 && aligned && (P.Wo % 4) == 0) {
    const int ntx = (P.Wo + DW2_TW - 1) / DW2_TW, nty = (P.Ho + DW2_TH - 1) / DW2_TH;
    hipLaunchKernelGGL(dw3x3_s2_vec_kernel, dim3(ntx * nty, P.C, P.B), dim3(256), 0, st, P);
    HIP_OK(hipGetLastError());
    return;
  }
  const int TH = P.stride == 1 ? DW_TH1 : DW_TH2;
  const int ntx = (P.Wo + DW_TW - 1) / DW_TW, nty = (P.Ho + TH - 1) / TH;
  if (P.stride == 1) hipLaunchKernelGGL(dw3x3_kernel<1>, dim3(ntx * nty, P.C, P.B), dim3(256), 0, st, P);
  else hipLaunchKernelGGL(dw3x3_kernel<2>, dim3(ntx * nty, P.C, P.B), dim3(256), 0, st, P);
  HIP_OK(hipGetLastError());
}

// =============================================================================================
// LayerNorm over C channels of each pixel (C <= 128), NCHW
template <int C>
__global__ void ln_channels_kernel(const float* __restrict__ x, int64_t x_bs, float* __restrict__ y, int64_t y_bs,
                                   const float* __restrict__ g, const float* __restrict__ bta, int HW, float eps) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= HW) return;
  const float* xp = x + (int64_t)b * x_bs + p;
  float v[C];
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < C; ++c) { v[c] = xp[(int64_t)c * HW]; s += v[c]; }
  const float mean = s / (float)C;
  float q = 0.0f;
#pragma unroll
  for (int c = 0; c < C; ++c) { const float d = v[c] - mean; q = fmaf(d, d, q); }
  const float rstd = 1.0f / sqrtf(q / (float)C + eps);
  float* yp = y + (int64_t)b * y_bs + p;
#pragma unroll
  for (int c = 0; c < C; ++c) yp[(int64_t)c * HW] = (v[c] - mean) * rstd * g[c] + bta[c];
}

void ln_channels(const float* x, int64_t x_bs, float* y, int64_t y_bs, const float* g, const float* b, int C,
                 int HW, int B, hipStream_t st) {
  const dim3 grid((HW + 127) / 128, B);
  if (C == 32) hipLaunchKernelGGL(ln_channels_kernel<32>, grid, dim3(128), 0, st, x, x_bs, y, y_bs, g, b, HW, 1e-5f);
  else if (C == 64) hipLaunchKernelGGL(ln_channels_kernel<64>, grid, dim3(128), 0, st, x, x_bs, y, y_bs, g, b, HW, 1e-5f);
  else if (C == 128) hipLaunchKernelGGL(ln_channels_kernel<128>, grid, dim3(128), 0, st, x, x_bs, y, y_bs, g, b, HW, 1e-5f);
  else MLIC_CHECK(false, "LayerNorm channels must be 32, 64 or 128");
  HIP_OK(hipGetLastError());
}

// LocalContext windowed attention: the MFMA kernels (attn_local.hip); the round-1 VALU kernel is an
// A/B baseline in ab/attn_local_valu.hip (make AB=1, $MLIC_LOCAL_ATTN_VALU=1).
void local_attn(const LocalAttnParams& P, hipStream_t st) {
  static const bool valu = [] {
    const char* e = std::getenv("MLIC_LOCAL_ATTN_VALU");
    return e && std::atoi(e) != 0;
  }();
  if (valu) local_attn_valu(P, st);
  else local_attn_mfma(P, st);
}


// =============================================================================================
// Linear attention (context.py:180-187, 235-239): out = ctx^T . softmax_c(Q) with
// ctx = softmax_L(K) . V^T, without materialising either softmax:
//  * ctx_partial: per (image, head, split of L) the per-channel max m_s of the split's active keys,
//    sum_p exp(k - m_s) v (a register-tiled K.V^T) and sum_p exp(k - m_s);
//  * ctx_reduce: the splits combined in a fixed order with the max-rescaling exp(m_s - M), then the
//    division by the total exp-sum (bitwise reproducible, no atomics);
//  * attn_apply: the channel softmax of each pixel's query in registers, then ctx^T . q.
// kmask = 1: only anchor positions are keys (the intra-slice squeezed anchor half); qmask = 1: only
// non-anchor positions have queries (outputs 0 at anchors).
constexpr int CTX_CHUNK = 64;
#ifndef MLIC_LINATT_ABL  // diagnostics build: 1 = no K.V^T accumulation, 2 = no ctx^T.q contraction
#define MLIC_LINATT_ABL 0
#endif

// record per (image, head, split): [HD] key maxima m_s, [HD][HD] sum_p exp(k_c - m_s) v_d,
// [HD] sum_p exp(k_c - m_s).  256 threads; the K.V^T tile of thread t is a TC x TC block
// (TC = HD / 16) read from pixel-major LDS copies as float2 pairs.
// the fixed-order combine of one output's nsplit records (ctx_reduce_kernel).  Measured and rejected
// (round 4): the combine inside the partial launch by each (image, head)'s last-arriving block
// (agent-scope release fence + ticket per block, acquire in the last): 0.126 ms per inter-context call
// at 8 x 68 x 120 against 0.105 for partial + this separate reduce + the old apply launch -- the release
// fence of every one of the ~2200 blocks costs more than the launch it saves
__device__ __forceinline__ void ctx_combine(const float* __restrict__ src, float* __restrict__ dst, int hd, int nsplit,
                                            int o) {
  const int nout = hd * hd, rec = hd * (hd + 2), c = o / hd;
  float M = -3.0e38f;
  for (int k = 0; k < nsplit; ++k) M = fmaxf(M, src[(int64_t)k * rec + c]);
  float num = 0.0f, den = 0.0f;
  for (int k = 0; k < nsplit; ++k) {
    const float* r = src + (int64_t)k * rec;
    const float w = softmax_exp(r[c] - M);
    num = fmaf(w, r[hd + o], num);
    den = fmaf(w, r[hd + nout + c], den);
  }
  dst[o] = num / den;
}

template <int HD>
__global__ __launch_bounds__(256) void ctx_partial_kernel(const float* __restrict__ K, int64_t k_bs,
                                                          const float* __restrict__ V, int64_t v_bs,
                                                          float* __restrict__ part, int heads, int H, int W,
                                                          int nsplit, int kmask) {
  constexpr int KP = HD + 2;                  // row pitch (floats): float2-aligned, 2-way write conflicts
  constexpr int NE = HD * CTX_CHUNK / 256;    // staged elements per thread per chunk: c = wave + 4 j, pixel = lane
  constexpr int TC = HD / 16;
  __shared__ __attribute__((aligned(16))) float kt[CTX_CHUNK][KP];
  __shared__ __attribute__((aligned(16))) float vt[CTX_CHUNK][KP];
  __shared__ float mxs[HD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x, h = blockIdx.y % heads, b = blockIdx.y / heads;
  const int HW = H * W;
  const int per = (HW + nsplit - 1) / nsplit;
  const int pbeg = split * per, pend = min(HW, pbeg + per);
  const float* kb = K + (int64_t)b * k_bs + (int64_t)h * HD * HW;
  const float* vb = V + (int64_t)b * v_bs + (int64_t)h * HD * HW;
  auto active = [&](int p) { return kmask == 0 || is_anchor(p / W, p % W); };
  // pass 1: the split's per-channel key maximum, one wave per channel
  for (int c = wave; c < HD; c += 4) {
    float m = -3.0e38f;
    for (int p = pbeg + lane; p < pend; p += 64)
      if (active(p)) m = fmaxf(m, kb[(int64_t)c * HW + p]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) mxs[c] = m;
  }
  __syncthreads();
  float mloc[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) mloc[j] = mxs[wave + 4 * j];
  float ssum[NE];
#pragma unroll
  for (int j = 0; j < NE; ++j) ssum[j] = 0.0f;
  const int c0 = (tid >> 4) * TC, d0 = (tid & 15) * TC;
  float acc[TC][TC];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int k = 0; k < TC; ++k) acc[i][k] = 0.0f;
  for (int p0 = pbeg; p0 < pend; p0 += CTX_CHUNK) {
    const int p = p0 + lane;
    const bool in = p < pend, on = in && active(p);
    float kv[NE], vv[NE];
#pragma unroll
    for (int j = 0; j < NE; ++j) {  // loads first, one latency per chunk
      const int64_t off = (int64_t)(wave + 4 * j) * HW + p;
      kv[j] = on ? kb[off] : 0.0f;
      vv[j] = in ? vb[off] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < NE; ++j) {
      const float e = on ? softmax_exp(kv[j] - mloc[j]) : 0.0f;
      ssum[j] += e;
      kt[lane][wave + 4 * j] = e;
      vt[lane][wave + 4 * j] = vv[j];
    }
    __syncthreads();
#pragma unroll 8
    for (int pp = 0; pp < ((MLIC_LINATT_ABL & 1) ? 1 : CTX_CHUNK); ++pp) {  // (diagnostics: no K.V^T FLOPs)
      if constexpr (TC == 2) {
        const float2 a = *reinterpret_cast<const float2*>(&kt[pp][c0]);
        const float2 v = *reinterpret_cast<const float2*>(&vt[pp][d0]);
        acc[0][0] = fmaf(a.x, v.x, acc[0][0]);
        acc[0][1] = fmaf(a.x, v.y, acc[0][1]);
        acc[1][0] = fmaf(a.y, v.x, acc[1][0]);
        acc[1][1] = fmaf(a.y, v.y, acc[1][1]);
      } else {
        acc[0][0] = fmaf(kt[pp][c0], vt[pp][d0], acc[0][0]);
      }
    }
    __syncthreads();
  }
  float* dst = part + (((int64_t)b * heads + h) * nsplit + split) * (HD * (HD + 2));
  if (tid < HD) dst[tid] = mxs[tid];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int k = 0; k < TC; ++k) dst[HD + (c0 + i) * HD + d0 + k] = acc[i][k];
#pragma unroll
  for (int j = 0; j < NE; ++j) {  // fixed butterfly; lane 0's value is the record
    float t = ssum[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) dst[HD + HD * HD + wave + 4 * j] = t;
  }
}

__global__ void ctx_reduce_kernel(const float* __restrict__ part, float* __restrict__ ctx, int hd, int nsplit,
                                  int total) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // over (b*heads) * hd * hd
  if (i >= total) return;
  const int nout = hd * hd, rec = hd * (hd + 2);
  const int bh = i / nout;
  ctx_combine(part + (int64_t)bh * nsplit * rec, ctx + (int64_t)bh * nout, hd, nsplit, i % nout);
}

// out[b][h*hd+d][p] = sum_c ctx[b][h][c][d] * softmax_c(Q[b][h*hd+c][p]); ctx rows read as float4
template <int HD>
__global__ __launch_bounds__(256) void attn_apply_kernel(const float* __restrict__ ctx, const float* __restrict__ Q,
                                                         int64_t q_bs, float* __restrict__ out, int64_t o_bs,
                                                         int heads, int H, int W, int qmask) {
  constexpr int hd = HD;
  __shared__ __attribute__((aligned(16))) float cs[HD * HD];
  const int HW = H * W;
  const int h = blockIdx.y % heads, b = blockIdx.y / heads;
  const float* cb = ctx + ((int64_t)b * heads + h) * hd * hd;
  for (int i = threadIdx.x; i < hd * hd; i += 256) cs[i] = cb[i];
  __syncthreads();
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= HW) return;
  float* op = out + (int64_t)b * o_bs + (int64_t)h * hd * HW + p;
  if (qmask && is_anchor(p / W, p % W)) {
    for (int d = 0; d < hd; ++d) op[(int64_t)d * HW] = 0.0f;
    return;
  }
  const float* qp = Q + (int64_t)b * q_bs + (int64_t)h * hd * HW + p;
  float q[HD];
  query_softmax<HD>(qp, HW, q);
  float a[HD];
#pragma unroll
  for (int d = 0; d < hd; ++d) a[d] = 0.0f;
#pragma unroll
  for (int c = 0; c < ((MLIC_LINATT_ABL & 2) ? 1 : hd); ++c) {  // (diagnostics: no ctx^T.q FLOPs)
#pragma unroll
    for (int d4 = 0; d4 < hd / 4; ++d4) {
      const float4 w = *reinterpret_cast<const float4*>(&cs[c * hd + 4 * d4]);  // broadcast
      a[4 * d4] = fmaf(w.x, q[c], a[4 * d4]);
      a[4 * d4 + 1] = fmaf(w.y, q[c], a[4 * d4 + 1]);
      a[4 * d4 + 2] = fmaf(w.z, q[c], a[4 * d4 + 2]);
      a[4 * d4 + 3] = fmaf(w.w, q[c], a[4 * d4 + 3]);
    }
  }
#pragma unroll
  for (int d = 0; d < hd; ++d) op[(int64_t)d * HW] = a[d];
}

int64_t linear_attention_part_floats(int heads, int hd, int B, int nsplit) {
  return (int64_t)B * heads * nsplit * (hd * (hd + 2));
}

void linear_attention_ctx(const float* K, int64_t k_bs, const float* V, int64_t v_bs, float* part, float* ctx,
                          int heads, int hd, int H, int W, int B, int nsplit, int kmask, hipStream_t st) {
  MLIC_CHECK(hd == 16 || hd == 32, "head dim");
  if (hd == 16)
    hipLaunchKernelGGL(ctx_partial_kernel<16>, dim3(nsplit, heads * B), dim3(256), 0, st, K, k_bs, V, v_bs, part, heads,
                       H, W, nsplit, kmask);
  else
    hipLaunchKernelGGL(ctx_partial_kernel<32>, dim3(nsplit, heads * B), dim3(256), 0, st, K, k_bs, V, v_bs, part, heads,
                       H, W, nsplit, kmask);
  HIP_OK(hipGetLastError());
  const int total = B * heads * hd * hd;
  hipLaunchKernelGGL(ctx_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, part, ctx, hd, nsplit, total);
  HIP_OK(hipGetLastError());
}

void linear_attention(const float* K, int64_t k_bs, const float* V, int64_t v_bs, const float* Q, int64_t q_bs,
                      float* out, int64_t o_bs, float* part, float* ctx, int heads, int hd, int H, int W, int B,
                      int nsplit, int kmask, int qmask, hipStream_t st) {
  MLIC_CHECK(hd == 16 || hd == 32, "head dim");
  const int HW = H * W;
  if (hd == 16)
    hipLaunchKernelGGL(ctx_partial_kernel<16>, dim3(nsplit, heads * B), dim3(256), 0, st, K, k_bs, V, v_bs, part, heads,
                       H, W, nsplit, kmask);
  else
    hipLaunchKernelGGL(ctx_partial_kernel<32>, dim3(nsplit, heads * B), dim3(256), 0, st, K, k_bs, V, v_bs, part, heads,
                       H, W, nsplit, kmask);
  HIP_OK(hipGetLastError());
  const int total = B * heads * hd * hd;
  hipLaunchKernelGGL(ctx_reduce_kernel, dim3((total + 255) / 256), dim3(256), 0, st, part, ctx, hd, nsplit, total);
  HIP_OK(hipGetLastError());
  if (hd == 16)
    hipLaunchKernelGGL(attn_apply_kernel<16>, dim3((HW + 255) / 256, heads * B), dim3(256), 0, st, ctx, Q, q_bs, out,
                       o_bs, heads, H, W, qmask);
  else
    hipLaunchKernelGGL(attn_apply_kernel<32>, dim3((HW + 255) / 256, heads * B), dim3(256), 0, st, ctx, Q, q_bs, out,
                       o_bs, heads, H, W, qmask);
  HIP_OK(hipGetLastError());
}

// =============================================================================================
// checkerboard mask copy (ckbd_anchor / ckbd_nonanchor as a materialised map)
__global__ void ckbd_mask_kernel(const float* __restrict__ x, int64_t x_bs, float* __restrict__ y, int64_t y_bs, int C,
                                 int H, int W, int keep_anchor) {
  const int64_t HW = (int64_t)H * W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= C * HW) return;
  const int p = (int)(i % HW);
  const bool a = is_anchor(p / W, p % W);
  y[(int64_t)b * y_bs + i] = (a == (keep_anchor != 0)) ? x[(int64_t)b * x_bs + i] : 0.0f;
}

void ckbd_mask(const float* x, int64_t x_bs, float* y, int64_t y_bs, int C, int H, int W, int B, int keep_anchor,
               hipStream_t st) {
  const int64_t n = (int64_t)C * H * W;
  hipLaunchKernelGGL(ckbd_mask_kernel, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, st, x, x_bs, y, y_bs, C, H,
                     W, keep_anchor);
  HIP_OK(hipGetLastError());
}

// =============================================================================================
// slice-loop quantisation.  params: EP output [2C] (scales = [0,C), means = [C,2C)).
//  phase 0 (anchor):     yh[c,p] = anchor(p) ? q(y, m) : 0
//  phase 1 (non-anchor): yh[c,p] = anchor(p) ? yh[c,p] : q(y, m_na);  and, when lik != null,
//                        lik[c,p] = GC(y, s_sel, m_sel) with (s,m) taken from pa at anchor pixels
//                        and from pn at non-anchor pixels (ckbd_merge).
//  q(y, m) = round((y - m) * sc) * rs + m  (sc = rs = 1 => exactly torch.round(y - m) + m)
//  sym/idx (optional): int32 squeezed [C][H][W/2] phase streams for the rANS coder.
__device__ __forceinline__ float std_cum(float x) { return 0.5f * erfcf(-0.70710678118654752440f * x); }

__device__ __forceinline__ float gauss_lik(float y, float s, float m) {
  // compressai GaussianConditional.forward (eval): dequantize, _likelihood, lower bounds
  const float outv = rintf(y - m) + m;
  const float v = fabsf(outv - m);
  const float sb = fmaxf(s, 0.11f);
  const float lik = std_cum((0.5f - v) / sb) - std_cum((-0.5f - v) / sb);
  return fmaxf(lik, 1e-9f);
}

__device__ __forceinline__ int scale_index(float s, const float* __restrict__ table, int n) {
  // compressai build_indexes: (n - 1) - #{t in table[:-1] : max(s, 0.11) <= t}
  const float sb = fmaxf(s, 0.11f);
  int idx = n - 1;
  for (int k = 0; k < n - 1; ++k) idx -= (sb <= table[k]) ? 1 : 0;
  return idx;
}

__global__ void quant_phase_kernel(QuantParams P) {
  const int HW = P.H * P.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= (int64_t)P.C * HW) return;
  const int c = (int)(i / HW), p = (int)(i % HW);
  const int h = p / P.W, w = p % P.W;
  const bool anc = is_anchor(h, w);
  const bool mine = (P.phase == 0) == anc;
  const float y = P.y[(int64_t)b * P.y_bs + i];
  const float* pp = P.params + (int64_t)b * P.params_bs;
  const float sc = P.vbr ? P.sc[b] : 1.0f, rs = P.vbr ? P.rs[b] : 1.0f;
  float* yh = P.yh + (int64_t)b * P.yh_bs + i;
  if (P.lik) {
    const float* pa = P.params_a + (int64_t)b * P.params_a_bs;
    const float s = anc ? pa[(int64_t)c * HW + p] : pp[(int64_t)c * HW + p];
    const float m = anc ? pa[(int64_t)(c + P.C) * HW + p] : pp[(int64_t)(c + P.C) * HW + p];
    float lk;
    if (P.vbr) lk = gauss_lik(y * sc, s * sc, m * sc);
    else lk = gauss_lik(y, s, m);
    P.lik[(int64_t)b * P.lik_bs + i] = lk;
  }
  if (!mine) {
    if (P.phase == 0) *yh = 0.0f;
    return;
  }
  const float s = pp[(int64_t)c * HW + p];
  const float m = pp[(int64_t)(c + P.C) * HW + p];
  float q;
  if (P.vbr) q = rintf((y - m) * sc);
  else q = rintf(y - m);
  *yh = P.vbr ? q * rs + m : q + m;
  if (P.sym || P.sym16) {
    const int64_t sq = (int64_t)b * P.C * HW / 2 + ((int64_t)c * P.H + h) * (P.W / 2) + (w >> 1);
    const int ix = scale_index(P.vbr ? s * sc : s, P.table, P.ntable);
    if (P.sym) P.sym[sq] = (int32_t)q;
    if (P.idx) P.idx[sq] = ix;
    if (P.sym16) {
      const float lim = (float)P.nlim;  // 32767 unless a test lowers it (narrow_limit)
      const bool fits = q >= -lim - 1.0f && q <= lim;
      P.sym16[sq] = (int16_t)(fits ? q : (q < 0.0f ? -lim - 1.0f : lim));
      P.idx8[sq] = (uint8_t)ix;
      if (!fits) *P.ovf = 1;  // a vector store from the lanes that overflow (benign race: all store 1)
    }
  }
}

void quant_phase(const QuantParams& P, hipStream_t st) {
  MLIC_CHECK(P.W % 2 == 0, "even latent width");
  const int64_t n = (int64_t)P.C * P.H * P.W;
  hipLaunchKernelGGL(quant_phase_kernel, dim3((unsigned)((n + 255) / 256), P.B), dim3(256), 0, st, P);
  HIP_OK(hipGetLastError());
}

// decoder: indexes of one phase (squeezed order), from the EP scales
__global__ void phase_indexes_kernel(QuantParams P) {
  const int HW = P.H * P.W, W2 = P.W / 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // squeezed index within image
  const int b = blockIdx.y;
  if (i >= (int64_t)P.C * P.H * W2) return;
  const int c = (int)(i / (P.H * W2));
  const int r = (int)(i % (P.H * W2));
  const int h = r / W2, j = r % W2;
  const int w = 2 * j + ((P.phase == 0) ? (1 - (h & 1)) : (h & 1));
  const float s = P.params[(int64_t)b * P.params_bs + (int64_t)c * HW + h * P.W + w];
  const int ix = scale_index(P.vbr ? s * P.sc[b] : s, P.table, P.ntable);
  const int64_t o = (int64_t)b * P.C * P.H * W2 + i;
  if (P.idx8) P.idx8[o] = (uint8_t)ix;
  else P.idx[o] = ix;
}

void phase_indexes(const QuantParams& P, hipStream_t st) {
  const int64_t n = (int64_t)P.C * P.H * (P.W / 2);
  hipLaunchKernelGGL(phase_indexes_kernel, dim3((unsigned)((n + 255) / 256), P.B), dim3(256), 0, st, P);
  HIP_OK(hipGetLastError());
}

// decoder: yh at the phase's pixels = sym * rs + m (anchor phase also zeroes the others)
__global__ void phase_dequant_kernel(QuantParams P) {
  const int HW = P.H * P.W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= (int64_t)P.C * HW) return;
  const int c = (int)(i / HW), p = (int)(i % HW);
  const int h = p / P.W, w = p % P.W;
  const bool mine = (P.phase == 0) == is_anchor(h, w);
  float* yh = P.yh + (int64_t)b * P.yh_bs + i;
  if (!mine) {
    if (P.phase == 0) *yh = 0.0f;
    return;
  }
  const int64_t sq = (int64_t)b * P.C * HW / 2 + ((int64_t)c * P.H + h) * (P.W / 2) + (w >> 1);
  const float q = P.sym16 ? (float)P.sym16[sq] : (float)P.sym[sq];
  const float m = P.params[(int64_t)b * P.params_bs + (int64_t)(c + P.C) * HW + p];
  *yh = P.vbr ? q * P.rs[b] + m : q + m;
}

void phase_dequant(const QuantParams& P, hipStream_t st) {
  const int64_t n = (int64_t)P.C * P.H * P.W;
  hipLaunchKernelGGL(phase_dequant_kernel, dim3((unsigned)((n + 255) / 256), P.B), dim3(256), 0, st, P);
  HIP_OK(hipGetLastError());
}

// =============================================================================================
// EntropyBottleneck: z_hat = round(z - med) + med, likelihood via the factorized logistic
// cumulative (filters 3,3,3,3), symbols = round(z - med) for the coder
__device__ __forceinline__ float softplus_t(float x) {
  // F.softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(expf(x));
}

__device__ void eb_logits(const EbParams& P, int c, float x, float* out1) {
  float v[3];
  float u[3];
  // layer 0: [3x1]
  for (int o = 0; o < 3; ++o) {
    float a = softplus_t(P.m0[c * 3 + o]) * x;
    a = a + P.b0[c * 3 + o];
    a = a + tanhf(P.f0[c * 3 + o]) * tanhf(a);
    v[o] = a;
  }
  const float* ms[3] = {P.m1, P.m2, P.m3};
  const float* bs[3] = {P.b1, P.b2, P.b3};
  const float* fs[3] = {P.f1, P.f2, P.f3};
  for (int l = 0; l < 3; ++l) {
    for (int o = 0; o < 3; ++o) {
      float a = 0.0f;
      for (int k = 0; k < 3; ++k) a = fmaf(softplus_t(ms[l][(c * 3 + o) * 3 + k]), v[k], a);
      a = a + bs[l][c * 3 + o];
      a = a + tanhf(fs[l][c * 3 + o]) * tanhf(a);
      u[o] = a;
    }
    for (int o = 0; o < 3; ++o) v[o] = u[o];
  }
  float a = 0.0f;
  for (int k = 0; k < 3; ++k) a = fmaf(softplus_t(P.m4[c * 3 + k]), v[k], a);
  *out1 = a + P.b4[c];
}

__global__ void eb_forward_kernel(EbParams P) {
  const int HW = P.H * P.W;
  const int64_t n = (int64_t)P.B * P.C * HW;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)((i / HW) % P.C);
  const float med = P.quantiles[c * 3 + 1];
  const float z = P.z[i];
  const float r = rintf(z - med);
  const float zh = r + med;
  if (P.z_hat) P.z_hat[i] = zh;
  if (P.sym) P.sym[i] = (int32_t)r;
  if (P.lik) {
    float lo, up;
    eb_logits(P, c, zh - 0.5f, &lo);
    eb_logits(P, c, zh + 0.5f, &up);
    const float sl = 1.0f / (1.0f + expf(-lo));
    const float su = 1.0f / (1.0f + expf(-up));
    P.lik[i] = fmaxf(su - sl, 1e-9f);
  }
}

void eb_forward(const EbParams& P, hipStream_t st) {
  const int64_t n = (int64_t)P.B * P.C * P.H * P.W;
  hipLaunchKernelGGL(eb_forward_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P);
  HIP_OK(hipGetLastError());
}

// z_hat from decoded symbols (decoder side)
__global__ void eb_dequant_kernel(const int32_t* __restrict__ sym, const float* __restrict__ quantiles,
                                  float* __restrict__ z_hat, int C, int HW, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int c = (int)((i / HW) % C);
  z_hat[i] = (float)sym[i] + quantiles[c * 3 + 1];
}

void eb_dequant(const int32_t* sym, const float* quantiles, float* z_hat, int C, int HW, int B, hipStream_t st) {
  const int64_t n = (int64_t)B * C * HW;
  hipLaunchKernelGGL(eb_dequant_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, sym, quantiles, z_hat, C,
                     HW, n);
  HIP_OK(hipGetLastError());
}

// =============================================================================================
// weight preparation (model create time)
// conv weight [Cout][Cin][K][K] (or linear [Cout][Cin]) -> packed [K*K][Cin][Cout]
__global__ void pack_conv_kernel(const float* __restrict__ w, float* __restrict__ out, int Cout, int Cin, int KK) {
  const int64_t n = (int64_t)Cout * Cin * KK;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int co = (int)(i / ((int64_t)Cin * KK));
  const int rem = (int)(i % ((int64_t)Cin * KK));
  const int ci = rem / KK, tap = rem % KK;
  out[((int64_t)tap * Cin + ci) * Cout + co] = w[i];
}

__global__ void copy_many_kernel(const CopyDesc* __restrict__ d) {
  const CopyDesc c = d[blockIdx.x];
  const int64_t t0 = (int64_t)blockIdx.y * blockDim.x + threadIdx.x, nt = (int64_t)gridDim.y * blockDim.x;
  if (((reinterpret_cast<uintptr_t>(c.dst) | reinterpret_cast<uintptr_t>(c.src)) & 15) == 0) {
    const int64_t n4 = c.n >> 2;  // 16-byte pieces, then the tail
    for (int64_t i = t0; i < n4; i += nt)
      reinterpret_cast<float4*>(c.dst)[i] = reinterpret_cast<const float4*>(c.src)[i];
    for (int64_t i = 4 * n4 + t0; i < c.n; i += nt) c.dst[i] = c.src[i];
  } else {
    for (int64_t i = t0; i < c.n; i += nt) c.dst[i] = c.src[i];
  }
}

void copy_many(const CopyDesc* descs, int n, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(copy_many_kernel, dim3((unsigned)n, 128), dim3(256), 0, st, descs);
  HIP_OK(hipGetLastError());
}

void pack_conv(const float* w, float* out, int Cout, int Cin, int KK, hipStream_t st) {
  const int64_t n = (int64_t)Cout * Cin * KK;
  hipLaunchKernelGGL(pack_conv_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, w, out, Cout, Cin, KK);
  HIP_OK(hipGetLastError());
}

// GDN reparametrisation: eff = max(p, bound)^2 - pedestal; gamma [C][C] is packed as a 1x1 conv
__global__ void gdn_prep_kernel(const float* __restrict__ beta, const float* __restrict__ gamma,
                                const float* __restrict__ bb, const float* __restrict__ bped,
                                const float* __restrict__ gb, const float* __restrict__ gped,
                                float* __restrict__ beta_eff, float* __restrict__ gamma_pk,
                                float* __restrict__ gamma_eff, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < C) {
    const float v = fmaxf(beta[i], bb[0]);
    beta_eff[i] = v * v - bped[0];
  }
  if (i < C * C) {
    const int co = i / C, ci = i % C;
    const float v = fmaxf(gamma[i], gb[0]);
    const float e = v * v - gped[0];
    gamma_pk[ci * C + co] = e;
    gamma_eff[i] = e;  // [co][ci], conv-weight layout
  }
}

void gdn_prep(const float* beta, const float* gamma, const float* bb, const float* bped, const float* gb,
              const float* gped, float* beta_eff, float* gamma_pk, float* gamma_eff, int C, hipStream_t st) {
  hipLaunchKernelGGL(gdn_prep_kernel, dim3((C * C + 255) / 256), dim3(256), 0, st, beta, gamma, bb, bped, gb, gped,
                     beta_eff, gamma_pk, gamma_eff, C);
  HIP_OK(hipGetLastError());
}

// LocalContext attention mask as the reference materialises it (for the bit-exact test only;
// the attention kernel derives it from parity bits)
__global__ void local_mask_kernel(float* __restrict__ out, int H, int W) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)H * W * 625;
  if (i >= n) return;
  const int p = (int)(i / 625), ij = (int)(i % 625);
  const int qi = ij / 25, kj = ij % 25;
  const int py = p / W, px = p % W;
  auto va = [&](int cell) {
    const int y = py + cell / 5 - 2, x = px + cell % 5 - 2;
    return y >= 0 && y < H && x >= 0 && x < W && (((y + x) & 1) == 1);
  };
  out[i] = (va(qi) && va(kj)) ? 0.0f : -100.0f;
}

void local_mask(float* out, int H, int W, hipStream_t st) {
  const int64_t n = (int64_t)H * W * 625;
  hipLaunchKernelGGL(local_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, H, W);
  HIP_OK(hipGetLastError());
}

// image metrics support: uint8 truncation as torchvision ToPILImage (clamp, *255, .byte())
__global__ void sq_err_u8_kernel(const float* __restrict__ a, const float* __restrict__ b, double* __restrict__ out,
                                 int64_t n_per, int64_t a_bs, int64_t b_bs) {
  __shared__ double red[256];
  const int img = blockIdx.y;
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_per; i += (int64_t)gridDim.x * 256) {
    const float va = floorf(fminf(fmaxf(a[img * a_bs + i], 0.0f), 1.0f) * 255.0f);
    const float vb = floorf(fminf(fmaxf(b[img * b_bs + i], 0.0f), 1.0f) * 255.0f);
    const double d = (double)va - (double)vb;
    s += d * d;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(out + img, red[0]);
}

void sq_err_u8(const float* a, int64_t a_bs, const float* b, int64_t b_bs, double* out, int64_t n_per, int B,
               hipStream_t st) {
  HIP_OK(hipMemsetAsync(out, 0, sizeof(double) * B, st));
  const int nb = (int)std::min<int64_t>(1024, (n_per + 255) / 256);
  hipLaunchKernelGGL(sq_err_u8_kernel, dim3(nb, B), dim3(256), 0, st, a, b, out, n_per, a_bs, b_bs);
  HIP_OK(hipGetLastError());
}

// sum of -log2 likelihoods per image (the bpp numerator of loss/rd_loss.py:42-45): per-block partial
// sums, then one fixed-order pass per image, so the result does not depend on block scheduling
constexpr int NEGLOG2_BLOCKS = 256;

__global__ void neglog2_partial_kernel(const float* __restrict__ lik, int64_t n_per, double* __restrict__ part) {
  __shared__ double red[256];
  const int img = blockIdx.y;
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_per; i += (int64_t)gridDim.x * 256)
    s += -(double)log2f(lik[img * n_per + i]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(int64_t)img * NEGLOG2_BLOCKS + blockIdx.x] = red[0];
}

__global__ void neglog2_final_kernel(const double* __restrict__ part, int nb, double* __restrict__ out, int B) {
  const int img = blockIdx.x * blockDim.x + threadIdx.x;
  if (img >= B) return;
  double s = 0.0;
  for (int k = 0; k < nb; ++k) s += part[(int64_t)img * NEGLOG2_BLOCKS + k];
  out[img] = s;
}

int64_t neglog2_partial_doubles(int B) { return (int64_t)B * NEGLOG2_BLOCKS; }

void neglog2_sum(const float* lik, int64_t n_per, int B, double* out, double* part, hipStream_t st) {
  const int nb = (int)std::min<int64_t>(NEGLOG2_BLOCKS, (n_per + 255) / 256);
  hipLaunchKernelGGL(neglog2_partial_kernel, dim3(nb, B), dim3(256), 0, st, lik, n_per, part);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(neglog2_final_kernel, dim3((B + 63) / 64), dim3(64), 0, st, part, nb, out, B);
  HIP_OK(hipGetLastError());
}

// element-wise entry points of the slice loop's device functions (tests: A16 / A17 bit-exactness)
__global__ void gauss_lik_kernel(const float* __restrict__ y, const float* __restrict__ s, const float* __restrict__ m,
                                 int64_t n, float sc, int vbr, float* __restrict__ lik) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  lik[i] = vbr ? gauss_lik(y[i] * sc, s[i] * sc, m[i] * sc) : gauss_lik(y[i], s[i], m[i]);
}

void gauss_likelihood(const float* y, const float* s, const float* m, int64_t n, float vbr_scale, float* lik,
                      hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(gauss_lik_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, s, m, n, vbr_scale,
                     vbr_scale != 1.0f ? 1 : 0, lik);
  HIP_OK(hipGetLastError());
}

__global__ void scale_index_kernel(const float* __restrict__ s, int64_t n, const float* __restrict__ table, int nt,
                                   int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  idx[i] = scale_index(s[i], table, nt);
}

void scale_indexes(const float* s, int64_t n, const float* table, int ntable, int32_t* idx, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scale_index_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s, n, table, ntable,
                     idx);
  HIP_OK(hipGetLastError());
}

}  // namespace mlic
