// Timing probe of the fused depthwise+pointwise kernel (mlic_amd/csrc/conv_dwpw.hip) at the g_a
// stage-1 shape; variants are compile-time macros of conv_dwpw.hip.  Build (CPU container):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I mlic_amd/csrc \
//         tools/gpu/dwpw_probe.hip -o tools/gpu/dwpw_probe [-DDP_DN=4 ...]
// Run on the GPU box: tools/gpu/dwpw_probe B C H W iters.  Values are random: timing only
// (correctness: tests/test_gpu_conv.py::test_dwpw_fused).
#include "../../mlic_amd/csrc/conv_dwpw.hip"

#include <cstdio>
#include <random>
#include <string>
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
  float *x, *y, *dw, *db, *bias;
  _Float16 *wh, *wl;
  int* flag;
  HIP_OK(hipMalloc(&x, n * 4));
  HIP_OK(hipMalloc(&y, n * 4));
  HIP_OK(hipMalloc(&dw, hdw.size() * 4));
  HIP_OK(hipMalloc(&db, Cn * 4));
  HIP_OK(hipMalloc(&bias, Cn * 4));
  HIP_OK(hipMalloc(&wh, hw.size() * 2));
  HIP_OK(hipMalloc(&wl, hw.size() * 2));
  HIP_OK(hipMalloc(&flag, 4));
  HIP_OK(hipMemcpy(x, hx.data(), n * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(dw, hdw.data(), hdw.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(db, hb.data(), Cn * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(bias, hb.data(), Cn * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(wh, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(wl, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
  HIP_OK(hipMemset(flag, 0, 4));
  ConvParams P{};
  P.nseg = 1;
  P.seg[0] = Seg{x, Cn, (int64_t)Cn * H * W};
  P.Cin = Cn; P.H = H; P.W = W; P.Cout = Cn; P.Ho = H; P.Wo = W; P.K = 1; P.stride = 1; P.pad = 0;
  P.bias = bias; P.out = y; P.out_cs = (int64_t)H * W; P.out_bs = (int64_t)Cn * H * W; P.B = B;
  P.epi = epi; P.rflag = flag;
#ifdef MLIC_DP_TRACE
  unsigned long long* dtr;
  HIP_OK(hipMalloc(&dtr, 8 * 512 * 8));
  HIP_OK(hipMemset(dtr, 0, 8 * 512 * 8));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_dp_trace), &dtr, sizeof(dtr)));
#endif
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  dwpw_forward(P, wh, wl, Cn, dw, db, 0);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) dwpw_forward(P, wh, wl, Cn, dw, db, 0);
  HIP_OK(hipEventRecord(e1, 0));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  printf("dwpw B=%d C=%d %dx%d: %.3f ms  %.0f GB/s algorithmic\n", B, Cn, H, W, ms, 8.0 * n / (ms * 1e-3) / 1e9);
#ifdef MLIC_DP_TRACE
  std::vector<unsigned long long> tr(8 * 512);
  HIP_OK(hipMemcpy(tr.data(), dtr, tr.size() * 8, hipMemcpyDeviceToHost));
  // per k-step of wave 0: wait+barrier, lstore, gload, compute (+ epilogue at block ends)
  const unsigned long long t0 = tr[0];
  printf(" g   barrier  lstore  gload  compute   (wave 0, cycles)\n");
  for (int g = 0; g + 1 < 60; ++g) {
    const unsigned long long* a = &tr[8 * g];
    const unsigned long long nx = tr[8 * (g + 1)];
    if (!nx) break;
    const unsigned long long ep = a[4];
    printf("%3d %8lld %7lld %6lld %8lld %s\n", g, (long long)(a[1] - a[0]), (long long)(a[2] - a[1]),
           (long long)(a[3] - a[2]), (long long)((ep ? ep : nx) - a[3]),
           ep ? ("epi " + std::to_string((long long)(nx - ep))).c_str() : "");
  }
  (void)t0;
#endif
  return 0;
}
