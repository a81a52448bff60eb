// Probe: does a register written right after an MFMA that reads it as SrcA / SrcB change what the MFMA
// computes?  (The dwpw2 bring-up failure, DESIGN §5: in the masked-residual builds hipcc placed
// `v_mov_b32 v18, 0` and the residual loads into v[18:21] one instruction after the MFMA that reads
// v[18:21] as its B operand, and the wrong outputs were whole 16-column halves of the MFMA's B.)
//
// One wave, v_mfma_f32_32x32x16_f16 with A = [I16 | 0] (row r < 16 selects k = r) so D[r][c] = B[r][c]:
// every (k, column) element of B that the MFMA saw is visible in D.  B[k][c] = 1 + k + 16 c (exact in
// fp16).  Right after the MFMA the first B register (lane holds k = 8h, 8h + 1) is overwritten with
// -1000 by: a VALU v_mov (VALU), a second MFMA-independent VALU op after N s_nops, or a VMEM load.
// Everything is one asm statement on fixed registers (hipcc pads nothing inside asm), so the gap is
// exactly what the string says.  Output per case: which columns of k = 0/1 (lanes h = 0) and
// k = 8/9 (h = 1) read the overwritten value.
//
// build: hipcc -O2 --offload-arch=gfx950 tools/gpu/mfma_war_probe.hip -o tools/gpu/mfma_war_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

#define NOP0 ""
#define NOP1 "s_nop 0\n\t"
#define NOP2 "s_nop 1\n\t"
#define NOP4 "s_nop 3\n\t"
#define NOP8 "s_nop 7\n\t"
#define NOP16 "s_nop 7\n\ts_nop 7\n\t"
#define NOP32 "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"

#define LOADIN                                                                                         \
  "v_mov_b32 v100, %[b0]\n\tv_mov_b32 v101, %[b1]\n\tv_mov_b32 v102, %[b2]\n\tv_mov_b32 v103, %[b3]\n\t" \
  "v_mov_b32 v104, %[a0]\n\tv_mov_b32 v105, %[a1]\n\tv_mov_b32 v106, %[a2]\n\tv_mov_b32 v107, %[a3]\n\t" \
  "s_nop 7\n\ts_nop 7\n\t"
#define MF32 "v_mfma_f32_32x32x16_f16 v[108:123], v[104:107], v[100:103], 0\n\t"
#define MF16 "v_mfma_f32_16x16x32_f16 v[108:111], v[104:107], v[100:103], 0\n\t"
#define DRAIN "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\t"
#define OUT16                                                                                              \
  "v_mov_b32 %[o0], v108\n\tv_mov_b32 %[o1], v109\n\tv_mov_b32 %[o2], v110\n\tv_mov_b32 %[o3], v111\n\t"     \
  "v_mov_b32 %[o4], v112\n\tv_mov_b32 %[o5], v113\n\tv_mov_b32 %[o6], v114\n\tv_mov_b32 %[o7], v115\n\t"     \
  "v_mov_b32 %[o8], v116\n\tv_mov_b32 %[o9], v117\n\tv_mov_b32 %[o10], v118\n\tv_mov_b32 %[o11], v119\n\t"  \
  "v_mov_b32 %[o12], v120\n\tv_mov_b32 %[o13], v121\n\tv_mov_b32 %[o14], v122\n\tv_mov_b32 %[o15], v123\n\t" \
  "s_waitcnt vmcnt(0)"
#define OPS                                                                                                  \
  : [o0] "=&v"(o[0]), [o1] "=&v"(o[1]), [o2] "=&v"(o[2]), [o3] "=&v"(o[3]), [o4] "=&v"(o[4]),                \
    [o5] "=&v"(o[5]), [o6] "=&v"(o[6]), [o7] "=&v"(o[7]), [o8] "=&v"(o[8]), [o9] "=&v"(o[9]),                \
    [o10] "=&v"(o[10]), [o11] "=&v"(o[11]), [o12] "=&v"(o[12]), [o13] "=&v"(o[13]), [o14] "=&v"(o[14]),      \
    [o15] "=&v"(o[15])                                                                                       \
  : [b0] "v"(bw[0]), [b1] "v"(bw[1]), [b2] "v"(bw[2]), [b3] "v"(bw[3]), [a0] "v"(aw[0]), [a1] "v"(aw[1]),    \
    [a2] "v"(aw[2]), [a3] "v"(aw[3]), [junk] "v"(junk), [jp] "v"(jptr)                                       \
  : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112",   \
    "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "memory"

// case: 0..6 VALU overwrite of SrcB v100 after 0,1,2,4,8,16,32 wait states; 7 VMEM load into v100 right
// after; 8 VALU overwrite of SrcA v104 right after; 9 no overwrite (control); 10..12 16x16x32 VALU SrcB
// after 0, 4, 16 (16x16x32 output: 4 registers)
#define CASE32(id, PRE, WR)                                     \
  case id:                                                      \
    asm volatile(LOADIN MF32 PRE WR DRAIN OUT16 OPS);           \
    break;
#define CASE16(id, PRE)                                                                                         \
  case id:                                                                                                      \
    asm volatile(LOADIN MF16 PRE "v_mov_b32 v100, %[junk]\n\t" DRAIN                                           \
                 "v_mov_b32 %[o0], v108\n\tv_mov_b32 %[o1], v109\n\tv_mov_b32 %[o2], v110\n\tv_mov_b32 %[o3], " \
                 "v111\n\tv_mov_b32 %[o4], v108\n\tv_mov_b32 %[o5], v108\n\tv_mov_b32 %[o6], v108\n\tv_mov_b32 "   \
                 "%[o7], v108\n\tv_mov_b32 %[o8], v108\n\tv_mov_b32 %[o9], v108\n\tv_mov_b32 %[o10], v108\n\t"    \
                 "v_mov_b32 %[o11], v108\n\tv_mov_b32 %[o12], v108\n\tv_mov_b32 %[o13], v108\n\tv_mov_b32 "       \
                 "%[o14], v108\n\tv_mov_b32 %[o15], v108\n\ts_waitcnt vmcnt(0)" OPS);                              \
    break;

#define WRB "v_mov_b32 v100, %[junk]\n\t"
#define WRA "v_mov_b32 v104, %[junk]\n\t"
#define LDB "global_load_dword v100, %[jp], off\n\t"

__global__ void probe(int which, const unsigned* jsrc, float* out) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  const int r16 = l & 15, q16 = l >> 4;
  half8 a, b;
  for (int j = 0; j < 8; ++j) {
    if (which < 10) {
      a[j] = (_Float16)((r == 8 * h + j) ? 1.0f : 0.0f);       // 32x32x16: A[r][8h + j]
      b[j] = (_Float16)(1.0f + (8 * h + j) + 16.0f * r);      // B[8h + j][r]
    } else {
      a[j] = (_Float16)((r16 == 8 * q16 + j) ? 1.0f : 0.0f);   // 16x16x32: A[l & 15][8 (l >> 4) + j]
      b[j] = (_Float16)(1.0f + (8 * q16 + j) + 32.0f * r16);  // B[8 (l >> 4) + j][l & 15]
    }
  }
  unsigned aw[4], bw[4];
  __builtin_memcpy(aw, &a, 16);
  __builtin_memcpy(bw, &b, 16);
  const unsigned junk = 0xE3D0E3D0u;  // (-1000, -1000) in fp16
  const unsigned* jptr = jsrc + l;
  float o[16];
  switch (which) {
    CASE32(0, NOP0, WRB)
    CASE32(1, NOP1, WRB)
    CASE32(2, NOP2, WRB)
    CASE32(3, NOP4, WRB)
    CASE32(4, NOP8, WRB)
    CASE32(5, NOP16, WRB)
    CASE32(6, NOP32, WRB)
    CASE32(7, NOP0, LDB)
    CASE32(8, NOP0, WRA)
    CASE32(9, NOP0, "")
    CASE16(10, NOP0)
    CASE16(11, NOP4)
    CASE16(12, NOP16)
    default: break;
  }
  for (int k = 0; k < 16; ++k) out[l * 16 + k] = o[k];
}

int main() {
  unsigned* dj;
  float* dout;
  CK(hipMalloc(&dj, 64 * 4));
  CK(hipMalloc(&dout, 64 * 16 * 4));
  unsigned hj[64];
  for (int i = 0; i < 64; ++i) hj[i] = 0xE3D0E3D0u;
  CK(hipMemcpy(dj, hj, sizeof hj, hipMemcpyHostToDevice));
  const char* names[] = {"VALU SrcB +0", "VALU SrcB +1", "VALU SrcB +2", "VALU SrcB +4", "VALU SrcB +8",
                         "VALU SrcB +16", "VALU SrcB +32", "VMEM SrcB +0", "VALU SrcA +0", "control",
                         "16x16 VALU SrcB +0", "16x16 VALU SrcB +4", "16x16 VALU SrcB +16"};
  for (int which = 0; which < 13; ++which) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(dout, 0, 64 * 16 * 4));
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, which, dj, dout);
      CK(hipDeviceSynchronize());
      float h[64 * 16];
      CK(hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost));
      // D[row][col]: 32x32 map col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5);
      // 16x16 map col = lane & 15, row = 4 (lane >> 4) + reg
      int seen_junk = 0, wrong = 0;
      char cols[2][33] = {};
      for (int hh = 0; hh < 2; ++hh)
        for (int c = 0; c < 32; ++c) cols[hh][c] = '.';
      for (int lane = 0; lane < 64; ++lane)
        for (int reg = 0; reg < (which < 10 ? 16 : 4); ++reg) {
          int row, col;
          if (which < 10) {
            col = lane & 31;
            row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
          } else {
            col = lane & 15;
            row = 4 * (lane >> 4) + reg;
          }
          const float v = h[lane * 16 + reg];
          float want;
          if (which < 10) want = row < 16 ? 1.0f + row + 16.0f * col : 0.0f;
          else want = 1.0f + row + 32.0f * col;
          if (v == want) continue;
          if (v == -1000.0f) {
            ++seen_junk;
            const int hh = (which < 10) ? row / 8 : row / 8;
            cols[hh & 1][col] = '#';
          } else {
            ++wrong;
          }
        }
      printf("%-22s rep %d: junk seen %3d, other wrong %3d | k0/1 cols %s | k8/9 cols %s\n", names[which], rep,
             seen_junk, wrong, cols[0], cols[1]);
    }
  }
  return 0;
}
