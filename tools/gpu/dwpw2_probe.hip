// Phase timing probe of the producer / consumer fused depthwise + pointwise kernel
// (mlic_amd/csrc/conv_dwpw2.hip) with -DMLIC_D2_TRACE: s_memtime cycles per phase, summed over the
// waves of each role, per step and wave.  Build (CPU container):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DMLIC_D2_TRACE -I mlic_amd/csrc \
//         tools/gpu/dwpw2_probe.hip -o tools/gpu/dwpw2_probe
// Run on the GPU box: tools/gpu/dwpw2_probe B C H W iters epi.  Random values: timing only.
#include "../../mlic_amd/csrc/conv_dwpw2.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace mlic;

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8;
  const int Cn = argc > 2 ? atoi(argv[2]) : 192;
  const int H = argc > 3 ? atoi(argv[3]) : 544;
  const int W = argc > 4 ? atoi(argv[4]) : 960;
  const int iters = argc > 5 ? atoi(argv[5]) : 10;
  const int epi = argc > 6 ? atoi(argv[6]) : EPI_GELU;
  const size_t n = (size_t)B * Cn * H * W;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-0.5f, 0.5f);
  std::vector<float> hx(n);
  for (auto& v : hx) v = U(rng);
  std::vector<_Float16> hw((size_t)Cn * Cn);
  for (auto& v : hw) v = (_Float16)(U(rng) * 0.1f);
  std::vector<float> hdw((size_t)Cn * 9), hb(Cn);
  for (auto& v : hdw) v = U(rng);
  for (auto& v : hb) v = U(rng);
  float *x, *y, *r, *dw, *db, *bias;
  _Float16 *wh, *wl;
  int* flag;
  unsigned long long* tr;
  HIP_OK(hipMalloc(&x, n * 4));
  HIP_OK(hipMalloc(&y, n * 4));
  HIP_OK(hipMalloc(&r, n * 4));
  HIP_OK(hipMalloc(&dw, hdw.size() * 4));
  HIP_OK(hipMalloc(&db, Cn * 4));
  HIP_OK(hipMalloc(&bias, Cn * 4));
  HIP_OK(hipMalloc(&wh, hw.size() * 2));
  HIP_OK(hipMalloc(&wl, hw.size() * 2));
  HIP_OK(hipMalloc(&flag, 4));
  HIP_OK(hipMalloc(&tr, 16 * 8));
  HIP_OK(hipMemcpy(x, hx.data(), n * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(r, hx.data(), n * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(dw, hdw.data(), hdw.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(db, hb.data(), Cn * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(bias, hb.data(), Cn * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(wh, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(wl, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  HIP_OK(hipMemset(flag, 0, 4));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(d2_trace), &tr, sizeof(tr)));
  ConvParams P{};
  P.nseg = 1;
  P.seg[0] = Seg{x, Cn, (int64_t)Cn * H * W};
  P.Cin = Cn; P.H = H; P.W = W; P.Cout = Cn; P.Ho = H; P.Wo = W; P.K = 1; P.stride = 1; P.pad = 0;
  P.bias = bias; P.out = y; P.out_cs = (int64_t)H * W; P.out_bs = (int64_t)Cn * H * W; P.B = B;
  P.epi = epi; P.rflag = flag; P.res = r; P.res_bs = P.out_bs;
  dwpw2_set(1);
  MLIC_CHECK(dwpw2_ok(P, Cn), "probe shape");
  dwpw2_forward(P, wh, wl, Cn, dw, db, nullptr);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemset(tr, 0, 16 * 8));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  HIP_OK(hipEventRecord(e0, nullptr));
  for (int i = 0; i < iters; ++i) dwpw2_forward(P, wh, wl, Cn, dw, db, nullptr);
  HIP_OK(hipEventRecord(e1, nullptr));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[16];
  HIP_OK(hipMemcpy(h, tr, sizeof h, hipMemcpyDeviceToHost));
  int ncu = 0;
  HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int Rr = d2_rows(H); const long long tiles = (long long)((W + 31) / 32) * ((H + Rr - 1) / Rr) * B;
  const long long steps = (long long)((W + 31) / 32) * B * ((H + Rr - 1) / Rr) * Rr * iters;  // output rows x segments
  const int nc = Cn / 32, np = 2;
  printf("dwpw2 B=%d C=%d %dx%d epi=%d: %.3f ms per launch; tiles %lld, %.1f per CU\n", B, Cn, H, W, epi, ms / iters,
         tiles, (double)tiles / ncu);
  const char* cn[3] = {"mfma", "epilogue", "barrier"};
  const char* pn[4] = {"dma-issue", "dma-wait", "depthwise", "barrier"};  // (row pipeline: per output row)
  printf("consumer cycles per step per wave:");
  for (int k = 0; k < 3; ++k) printf("  %s %.0f", cn[k], (double)h[k] / (steps * nc));
  printf("\nproducer cycles per step per wave:");
  for (int k = 0; k < 4; ++k) printf("  %s %.0f", pn[k], (double)h[8 + k] / (steps * np));
  printf("\n");
  return 0;
}
