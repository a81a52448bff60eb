// Vector-memory issue-rate probe: wave64 buffer loads of 4 / 8 / 16 bytes per lane from an
// L2-resident buffer, every CU busy; reports wave-instructions per CU-cycle and bytes per CU-cycle.
// build: hipcc -O3 --offload-arch=gfx950 tools/gpu/ta_probe.hip -o tools/gpu/ta_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int W>  // dwords per lane
__global__ __launch_bounds__(512) void probe(const float* __restrict__ src, int bytes, int iters, int stride_lane, float* out,
                                             int oob_mask) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0, bytes, 0x00020000);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t vo = (uint32_t)((blockIdx.x * 8 + wave) * 4096 + lane * stride_lane) % (uint32_t)(bytes - 64 * 64);
  const bool oob = (oob_mask & 64) ? true : (lane & oob_mask) != 0;  // these lanes read past the buffer (0, no memory access)
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const uint32_t o = oob ? 0x80000000u : vo + (uint32_t)u * 4096u;
      if (W == 1) acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0));
      if (W == 2) { auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, o, 0, 0); acc += __builtin_bit_cast(float, v[0]) + __builtin_bit_cast(float, v[1]); }
      if (W == 4) { auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0); acc += __builtin_bit_cast(float, v[0]) + __builtin_bit_cast(float, v[3]); }
    }
    vo = (vo + 65536u) % (uint32_t)(bytes - 64 * 64 - 16 * 4096);
  }
  if (acc == 12345.f) out[0] = acc;
}

template <int W>
int run(const float* buf, int bytes, int stride_lane, const char* tag, int oob_mask = 0) {
  int dev, ncu;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  float* out;
  CK(hipMalloc(&out, 4));
  const int iters = 200;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(probe<W>, dim3(ncu), dim3(512), 0, 0, buf, bytes, 10, stride_lane, out, oob_mask);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(probe<W>, dim3(ncu), dim3(512), 0, 0, buf, bytes, iters, stride_lane, out, oob_mask);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double insts_per_cu = 8.0 * 16 * iters;
  const double cyc = ms * 1e-3 * 2.1e9;
  printf("%-28s %6.3f ms  %.2f cyc per wave-load per CU  %.1f B/clk/CU (lane bytes)\n", tag, ms, cyc / insts_per_cu,
         insts_per_cu * 64 * 4 * W / cyc);
  CK(hipFree(out));
  return 0;
}

int main() {
  const int bytes = 8 << 20;  // L2/MALL-resident working set
  float* buf;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 0, bytes));
  run<1>(buf, bytes, 4, "dword, contiguous lanes");
  run<2>(buf, bytes, 8, "dwordx2, contiguous lanes");
  run<4>(buf, bytes, 16, "dwordx4, contiguous lanes");
  run<1>(buf, bytes, 0, "dword, all lanes one addr");
  run<1>(buf, bytes, 64, "dword, 64B apart per lane");
  run<1>(buf, bytes, 4, "dword, 8 lanes live, 56 OOB", 7);
  run<4>(buf, bytes, 16, "dwordx4, 8 lanes live, 56 OOB", 7);
  run<1>(buf, bytes, 4, "dword, all lanes OOB", 63 | 64);
  return 0;
}
