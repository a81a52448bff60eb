// Timing probe of the fused 1x1 chain kernel (mlic_amd/csrc/chain.hip) at the bench's EntropyParameters
// shapes, with per-step shader-clock timestamps of two workgroups.  Build (CPU container):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -DMLIC_CHAIN_TRACE \
//         -I mlic_amd/csrc tools/gpu/chain_probe.hip -o tools/gpu/chain_probe
// Run on the GPU box: tools/gpu/chain_probe B HW cin0 aux cout3 iters
// Values are random; only the timing is of interest (correctness: tests/test_gpu_parity.py).
#include "../../mlic_amd/csrc/chain.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace mlic;

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 8;
  const int HW = argc > 2 ? atoi(argv[2]) : 8160;
  const int cin0 = argc > 3 ? atoi(argv[3]) : 320;
  const int aux = argc > 4 ? atoi(argv[4]) : 1;
  const int c3 = argc > 5 ? atoi(argv[5]) : 64;
  const int iters = argc > 6 ? atoi(argv[6]) : 20;
  const int cout[4] = {320, 256, 128, c3};
  const int cin[4] = {cin0, 320, 256, 128};
  int64_t wh = 0;
  for (int l = 0; l < 4; ++l) wh += chain_layer_halves(cout[l], cin[l]);

  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-0.05f, 0.05f);
  std::vector<_Float16> hw(wh);
  for (auto& v : hw) v = (_Float16)U(rng);
  std::vector<float> hx((size_t)B * (cin0 > 0 ? cin0 : 1) * HW);
  for (auto& v : hx) v = U(rng);

  _Float16* dw;
  float *dx, *daux = nullptr, *dout, *dbias;
  int* dflag;
  HIP_OK(hipMalloc(&dw, wh * 2));
  HIP_OK(hipMemcpy(dw, hw.data(), wh * 2, hipMemcpyHostToDevice));
  HIP_OK(hipMalloc(&dx, hx.size() * 4));
  HIP_OK(hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  if (aux) {
    HIP_OK(hipMalloc(&daux, (size_t)B * 320 * HW * 4));
    HIP_OK(hipMemset(daux, 0, (size_t)B * 320 * HW * 4));
  }
  HIP_OK(hipMalloc(&dout, (size_t)B * c3 * HW * 4));
  HIP_OK(hipMalloc(&dbias, 1024 * 4));
  HIP_OK(hipMemset(dbias, 0, 1024 * 4));
  HIP_OK(hipMalloc(&dflag, 4));
  HIP_OK(hipMemset(dflag, 0, 4));
  unsigned long long* dtr;
  const size_t ntr = 2 * 4 * CH_TR_STEPS * 3;
  HIP_OK(hipMalloc(&dtr, ntr * 8));
  HIP_OK(hipMemset(dtr, 0, ntr * 8));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_trace), &dtr, sizeof(dtr)));

  ChainParams P{};
  P.nseg = cin0 > 0 ? 1 : 0;
  P.seg[0] = Seg{dx, cin0, (int64_t)cin0 * HW};
  P.cin0 = cin0;
  P.HW = HW;
  P.B = B;
  for (int l = 0; l < 4; ++l) P.bias[l] = dbias + 256 * l;
  P.wimg = dw;
  P.out = dout;
  P.out_bs = (int64_t)c3 * HW;
  P.rflag = dflag;
  P.aux = daux;
  P.aux_bs = (int64_t)320 * HW;

  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  chain_forward(P, 4, cout, 0);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) chain_forward(P, 4, cout, 0);
  HIP_OK(hipEventRecord(e1, 0));
  HIP_OK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  double macs = 0;
  for (int l = 0; l < 4; ++l) macs += (double)cout[l] * cin[l];
  const double flop = 2.0 * macs * B * HW;
  printf("chain B=%d HW=%d cin0=%d aux=%d c3=%d: %.4f ms  %.1f TF/s fp32-equiv\n", B, HW, cin0, aux, c3, ms,
         flop / (ms * 1e-3) / 1e12);

  // the trace of the last launch
  std::vector<unsigned long long> tr(ntr);
  HIP_OK(hipMemcpy(tr.data(), dtr, ntr * 8, hipMemcpyDeviceToHost));
  const int T = cin0 / 32 + 10 + 8 + 4;
  for (int g = 0; g < 2; ++g) {
    const unsigned long long* w0 = &tr[(size_t)g * 4 * CH_TR_STEPS * 3];
    const unsigned long long t0 = w0[0];
    printf("wg %d: total %llu clk\n", g, w0[(T < CH_TR_STEPS ? T : CH_TR_STEPS - 1) * 3] - t0);
    printf(" step  wait(w0)  barrier(w0)  work(w0)  | wait w1 w2 w3\n");
    for (int t = 0; t < T && t < CH_TR_STEPS; ++t) {
      auto at = [&](int w, int t_, int k) { return tr[(((size_t)g * 4 + w) * CH_TR_STEPS + t_) * 3 + k]; };
      const unsigned long long nxt = (t + 1 < T) ? at(0, t + 1, 0) : at(0, T < CH_TR_STEPS ? T : CH_TR_STEPS - 1, 0);
      printf(" %3d %8lld %8lld %8lld | %8lld %8lld %8lld\n", t, (long long)(at(0, t, 1) - at(0, t, 0)),
             (long long)(at(0, t, 2) - at(0, t, 1)), (long long)(nxt - at(0, t, 2)),
             (long long)(at(1, t, 1) - at(1, t, 0)), (long long)(at(2, t, 1) - at(2, t, 0)),
             (long long)(at(3, t, 1) - at(3, t, 0)));
    }
  }
  int flag = 0;
  HIP_OK(hipMemcpy(&flag, dflag, 4, hipMemcpyDeviceToHost));
  printf("range flag %d\n", flag);
  return 0;
}
