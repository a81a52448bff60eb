// Host-side launchers of the MLIC++ HIP kernels (see conv_mfma.hip, kernels.hip).
#pragma once
#include "common.h"

#include <algorithm>

namespace mlic {

// implicit-GEMM conv on MFMA (conv_mfma.hip)
// tile instantiation chosen for P: 0 = <64,64>, 1 = <64,128>, 2 = <128,64>, 3 = <128,128>
int conv_variant(const ConvParams& P);
void conv_forward(const ConvParams& P, hipStream_t st);

// split-fp16 ("f16x3") MFMA conv (conv_f16x3.hip): same contract, weights pre-split to
// hi/lo fp16 [Cout][K*K][cin_pad] (cin_pad = Cin rounded up to 32)
int conv_f16x3_variant(const ConvParams& P);
void conv_f16x3_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st);
int conv_x3v2_variant(const ConvParams& P);
void conv_x3v2_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st);
// prescale: split w * 2^e with the layer's max |w| * 2^e in [2^14, 2^15); returns e (0 without
// prescale).  Synchronises st.
int split_weights(const float* w, _Float16* wh, _Float16* wl, int Cout, int Cin, int KK, int cin_pad, bool prescale,
                  hipStream_t st);

// specialised convs (conv_pw.hip)
bool pw_resident_ok(const ConvParams& P, int cin_pad);
void pw_resident_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st);
bool conv_narrow_ok(const ConvParams& P);
void conv_narrow_forward(const ConvParams& P, hipStream_t st);
// A/B-only families (ab/*.hip, make AB=1): v1 tiles, halo tiles, VALU local attention; the product
// build links ab/ab_stubs.cpp instead (they throw; conv_halo_ok is false)
bool ab_families_built();
bool conv_halo_ok(const ConvParams& P, int cin_pad);
void conv_halo_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st);
// g_s's N -> 12 3x3 output conv as 1x1 per-tap partials [B][108][H][W] + this gather (conv_pw.hip):
// out [B][3][2H][2W] = PixelShuffle(2)(bias + sum over taps of the shifted partials)
void taps_gather(const float* part, int64_t part_bs, const float* bias, float* out, int64_t out_bs, int H, int W,
                 int B, hipStream_t st);
bool conv_smallcin_ok(const ConvParams& P);
void conv_smallcin_forward(const ConvParams& P, hipStream_t st);

// fused depthwise 3x3 (stride 1, pad 1) + pointwise 1x1 (conv_dwpw.hip): P describes the pointwise
// conv with the DEPTHWISE input as its input; dww [Cin][9], dwb [Cin]; needs W even (dwpw_ok)
bool dwpw_ok(const ConvParams& P, int cin_pad);
// the model's choice on top of dwpw_ok: grids where the fused kernel measured faster (per image only)
bool dwpw_grid_ok(const ConvParams& P);
// producer / consumer forms for Cin = Cout in {96, 128, 160, 192}, bias / GELU (+ residual): dwpw_forward
// takes the chosen one (dwpw2_set) where it applies
bool dwpw2_ok(const ConvParams& P, int cin_pad);
// mlic_set_kernel_option("dwpw2"): -1 = $MLIC_DWPW2 (default 2), 0 = dwpw_kernel, 1 = the row-pipelined
// LDS form (ab/conv_dwpw2.hip: A/B-only family, make AB=1), 2 = the register-row form (conv_dwpw3.hip)
void dwpw2_set(int on);
// the A/B-only row-pipelined LDS form (ab/conv_dwpw2.hip; the product build's stub reports false / throws)
bool dwpw2_lds_ok(const ConvParams& P, int cin_pad);
void dwpw2_lds_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                       const float* dwb, hipStream_t st);
bool dwpw3_shape_ok(const ConvParams& P, int cin_pad);
// the same kernel's pointwise-only form for the full-resolution 1x1 convs (pw_resident MODE 0 - 3, Cin = Cout
// in {96, 128, 160, 192}): pw_resident_forward takes it where pw3_ok; mlic_set_kernel_option("pw3"):
// -1 = $MLIC_PW3 (default 1), 0 off, 1 from 256 K px per image, 2 every grid
bool pw3_ok(const ConvParams& P, int cin_pad);
void pw3_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, hipStream_t st);
void pw3_set(int on);
void dwpw3_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                   const float* dwb, hipStream_t st);
void dwpw2_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                   const float* dwb, hipStream_t st);
void dwpw_forward(const ConvParams& P, const _Float16* wh, const _Float16* wl, int cin_pad, const float* dww,
                  const float* dwb, hipStream_t st);

// LDS-DMA split-fp16 conv (conv_x4.hip): activations packed per call into a zero-bordered split
// layout (x4_pack_act, workspace of x4_act_halves halves), weights packed once (x4_pack_weights)
int x4_bm(int Cout);
// hi = the reduced-precision form (single fp16 term, 64-channel chunks; g_s only)
int x4_nchunk(int cin_pad, bool hi);
int64_t x4_weight_halves(int Cout, int KK, int cin_pad, bool hi = false);
void x4_pack_weights(const _Float16* wh, const _Float16* wl, int Cout, int KK, int cin_pad, _Float16* dst,
                     hipStream_t st, bool hi = false);
int64_t x4_act_halves(const ConvParams& P, int cin_pad, bool hi = false);
bool conv_x4_ok(const ConvParams& P, int cin_pad);
void x4_pack_act(const ConvParams& P, int cin_pad, _Float16* dst, hipStream_t st, bool hi = false);
// 1x1 layers: x4 builds its B rows from the fp32 input itself (no packed copy; act = nullptr)
bool x4_direct_ok(const ConvParams& P, bool hi);
// A/B switch of the halo-staged B operand (tests): 1 on, 0 off, -1 the default ($MLIC_X4_HALO)
void x4_set_halo(int on);
// A/B switch of the fused linear attention (model.cpp linatt_reproject): 1 on, 0 off, -1 default
void linatt_set_fused(int on);
// part: the split-K partial planes (x4_part_bytes bytes; nullptr = no split)
int x4_splitk(const ConvParams& P, int cin_pad, bool hi = false);
int64_t x4_part_bytes(const ConvParams& P, int cin_pad, bool hi = false);
void conv_x4_forward(const ConvParams& P, const _Float16* act, const _Float16* wx, int cin_pad, hipStream_t st,
                     float* part = nullptr, bool hi = false);

// kernel-family selection (conv_dispatch.cpp)
enum ConvImpl : int {
  CONV_F32 = 0, CONV_X3 = 1, CONV_X3V2 = 2, CONV_PW = 3, CONV_NARROW = 4, CONV_SMALLCIN = 5, CONV_HALO = 6,
  CONV_X4 = 7,
  CONV_X4H = 8  // x4 in the reduced-precision form (fp16 operands, fp32 accumulation): g_s on request only
};
struct ConvWeights {
  const float* wpk;  // fp32 packed [K*K][Cin][Cout] (in ConvParams too)
  const _Float16* wh;
  const _Float16* wl;
  int cin_pad;
  const _Float16* wx4 = nullptr;  // x4_pack_weights image (null: CONV_X4 not available)
  int wexp = 0;                   // wh/wl hold w * 2^wexp (split_weights)
  const _Float16* wx4h = nullptr; // the reduced-precision image (x4_pack_weights hi; null: no CONV_X4H)
};
int conv_select(const ConvParams& P, const ConvWeights& w, int precision);
// device workspace conv_run needs for impl (bytes; 0 = none)
int64_t conv_ws_bytes(int impl, const ConvParams& P, const ConvWeights& w);
void conv_run(int impl, const ConvParams& P, const ConvWeights& w, hipStream_t st, void* ws = nullptr);

// live-profiling categories (one per kernel family / tile instantiation)
enum ProfCat : int {
  PCAT_CONV_F32 = 0,     // 0..3  conv_mfma_kernel tiles (conv_variant)
  PCAT_CONV_X3 = 4,      // 4..7  conv_f16x3_kernel tiles (conv_f16x3_variant)
  PCAT_CONV_X3V2 = 8,    // 8..10 conv_x3v2_kernel tiles <64,128>, <128,256>, <128,128>
  PCAT_CONV_X3V2_WIDE = 11,  // conv_x3v2_kernel<256,256> (8 waves)
  PCAT_CONV_PW = 12,
  PCAT_CONV_NARROW = 13,
  PCAT_CONV_SMALLCIN = 14,
  PCAT_CONV_HALO = 15,
  PCAT_DW = 16,
  PCAT_LOCAL = 17,
  PCAT_LINATT = 18,
  PCAT_ELEM = 19,
  PCAT_CONV_X4 = 20,
  PCAT_CHAIN = 21,
  PCAT_DWPW = 22,
  PCAT_COUNT = 23
};
int conv_prof_cat(int impl, const ConvParams& P);
const char* prof_cat_name(int cat);

struct DwParams {
  Seg seg[MAXSEG];
  int nseg;
  int C, H, W, Ho, Wo, stride;
  const float* w;     // [C][9]
  const float* bias;  // [C]
  float* out;
  int64_t out_bs;
  int gelu;
  int B;
};
void dw3x3(const DwParams& P, hipStream_t st);
void dw_set_strip(int v);
void x4_set_splitk(int v);  // -1 default ($MLIC_X4_SPLITK, off), 0 off, 1 on  // A/B: 0 = the LDS-tile kernel for narrow stride-1 planes too

void ln_channels(const float* x, int64_t x_bs, float* y, int64_t y_bs, const float* g, const float* b, int C,
                 int HW, int B, hipStream_t st);

struct LocalAttnParams {
  const float* qkv;
  int64_t qkv_bs;
  float* out;  // [C*25][HW]
  int64_t out_bs;
  const float* rel_table;  // [81][2]
  const int* rel_index;    // [625] int32
  float scale;
  int C, H, W, B;
  // local_attn_packed only: 0 = every query pixel; 1 / 2 = the anchor / non-anchor pixels only, written
  // at their squeezed position y * W / 2 + x / 2 (W even)
  int ckbd;
};
void local_attn(const LocalAttnParams& P, hipStream_t st);       // MFMA (attn_local.hip) unless MLIC_LOCAL_ATTN_VALU=1
void local_attn_mfma(const LocalAttnParams& P, hipStream_t st);
void local_attn_valu(const LocalAttnParams& P, hipStream_t st);
// dim 32 only: output in conv_x4's packed split layout [B][25 query cells][npos][64 halves]
// (channel head*16 + d), the B operand of the fusion conv with its K permuted to cell*32 + channel
void local_attn_packed(const LocalAttnParams& P, _Float16* out, int npos, hipStream_t st);

// context.py:180-187 / 235-239 in three launches (no materialised softmax); kmask: anchor-only keys,
// qmask: non-anchor-only queries; part: linear_attention_part_floats() floats
int64_t linear_attention_part_floats(int heads, int hd, int B, int nsplit);
void linear_attention(const float* K, int64_t k_bs, const float* V, int64_t v_bs, const float* Q, int64_t q_bs,
                      float* out, int64_t o_bs, float* part, float* ctx, int heads, int hd, int H, int W, int B,
                      int nsplit, int kmask, int qmask, hipStream_t st);
// the fused form: ctx = softmax_L(K) . V^T (partials + the fixed-order combine), then linatt_pack
// (conv_x4.hip) computes ctx^T . softmax_c(Q) straight into the packed operand of the conv that
// consumes the attention (P: that conv's params; dst: x4_act_halves(P, P.Cin) halves)
void linear_attention_ctx(const float* K, int64_t k_bs, const float* V, int64_t v_bs, float* part, float* ctx,
                          int heads, int hd, int H, int W, int B, int nsplit, int kmask, hipStream_t st);
void linatt_pack(const float* Q, int64_t q_bs, const float* ctx, int heads, int hd, int qmask, const ConvParams& P,
                 _Float16* dst, hipStream_t st);
void ckbd_mask(const float* x, int64_t x_bs, float* y, int64_t y_bs, int C, int H, int W, int B, int keep_anchor,
               hipStream_t st);

struct QuantParams {
  const float* y;  // latent slice [C][HW] (encoder side)
  int64_t y_bs;
  const float* params;  // EP output of this phase [2C][HW]
  int64_t params_bs;
  const float* params_a;  // anchor-phase EP output (likelihood merge), phase 1 only
  int64_t params_a_bs;
  float* yh;  // y_hat slice [C][HW]
  int64_t yh_bs;
  float* lik;  // likelihood slice or null
  int64_t lik_bs;
  int32_t* sym;  // squeezed symbols or null
  int32_t* idx;  // squeezed indexes or null
  // the narrow coder streams that cross PCIe (a scale index is < 64; a symbol almost always fits 16
  // bits): encoder: written beside sym, a symbol beyond int16 saturates sym16 and sets *ovf (the host
  // then takes the int32 sym); decoder: phase_indexes writes idx8, phase_dequant reads sym16 when set
  int16_t* sym16;
  uint8_t* idx8;
  int* ovf;
  int nlim;  // the narrow range [-nlim - 1, nlim]: 32767 (int16); smaller only under the test knob below
  const float* table;
  int ntable;
  int phase;  // 0 anchor, 1 non-anchor
  int vbr;
  const float* sc;  // [B] per-image VBR gain (mlicpp_vbr.py:137, Gain[s] or inputscale), when vbr
  const float* rs;  // [B] 1 / sc, computed once on the host in fp32 (the reference's 1 / scale)
  int C, H, W, B;
};
void quant_phase(const QuantParams& P, hipStream_t st);
void phase_indexes(const QuantParams& P, hipStream_t st);
void phase_dequant(const QuantParams& P, hipStream_t st);

struct EbParams {
  const float* z;
  float* z_hat;
  float* lik;
  int32_t* sym;
  const float* quantiles;  // [C][1][3]
  const float *m0, *m1, *m2, *m3, *m4;
  const float *b0, *b1, *b2, *b3, *b4;
  const float *f0, *f1, *f2, *f3;
  int C, H, W, B;
};
void eb_forward(const EbParams& P, hipStream_t st);
void eb_dequant(const int32_t* sym, const float* quantiles, float* z_hat, int C, int HW, int B, hipStream_t st);

void pack_conv(const float* w, float* out, int Cout, int Cin, int KK, hipStream_t st);
// many device-to-device float copies in one launch (the weight load's per-parameter copies: one kernel
// instead of a blit per tensor); `descs` is a device array of n {dst, src, count}
struct CopyDesc {
  float* dst;
  const float* src;
  int64_t n;
};
void copy_many(const CopyDesc* descs, int n, hipStream_t st);
void gdn_prep(const float* beta, const float* gamma, const float* bb, const float* bped, const float* gb,
              const float* gped, float* beta_eff, float* gamma_pk, float* gamma_eff, int C, hipStream_t st);
void local_mask(float* out, int H, int W, hipStream_t st);
void sq_err_u8(const float* a, int64_t a_bs, const float* b, int64_t b_bs, double* out, int64_t n_per, int B,
               hipStream_t st);
// per-image sum of -log2(lik) (fixed order); part = neglog2_partial_doubles(B) doubles of scratch
int64_t neglog2_partial_doubles(int B);
void neglog2_sum(const float* lik, int64_t n_per, int B, double* out, double* part, hipStream_t st);
// GaussianConditional likelihood (vbr_scale != 1: of y*sc, s*sc, m*sc) and build_indexes, element-wise
void gauss_likelihood(const float* y, const float* s, const float* m, int64_t n, float vbr_scale, float* lik,
                      hipStream_t st);
void scale_indexes(const float* s, int64_t n, const float* table, int ntable, int32_t* idx, hipStream_t st);

// fused 1x1 chain (chain.hip): layer widths cout[0..nl-1] in {320,256,128,64|128} (EntropyParameters)
// or {128,64} (LocalContext MLP), GELU between layers; weights pre-packed by chain_pack per layer,
// concatenated
struct ChainParams {
  Seg seg[MAXSEG];
  int nseg, cin0;  // layer-0 input: channel concat, cin0 % 32 == 0
  int HW, B;       // pixels per image (HW % 4 == 0)
  const float* bias[4];
  int wexp[4];       // each layer's split weights are w * 2^wexp (split_weights)
  const _Float16* wimg;
  float* out;      // [B][cout[nl-1]][HW] (batch stride out_bs)
  int64_t out_bs;
  const float* res;  // optional residual added to the output (same layout, batch stride res_bs)
  int64_t res_bs;
  int* rflag;        // fp16 range guard (common.h range_check)
  const float* aux;  // optional [B][C1][HW] added to layer 0's pre-activation (hoisted part of layer 0)
  int64_t aux_bs;
  // checkerboard half: 0 = every pixel; 1 = the anchor pixels only ((y + x) odd), 2 = the non-anchor
  // pixels only (W even): the other half of every output plane is not written.  EntropyParameters'
  // outputs are read at their own phase's pixels only (ckbd_anchor / ckbd_nonanchor masks,
  // mlicpp.py:226-228, 239-241; quant_phase / phase_indexes / phase_dequant read `mine` pixels)
  int ckbd, W;
  int sq_in;  // with ckbd: the inputs and the residual are squeezed planes of HW / 2 pixels (pixel q at q)
};
bool chain_supported(int nl, const int* cout);
int64_t chain_layer_halves(int Cout, int Cin);
void chain_pack(const _Float16* wh, const _Float16* wl, int Cout, int Cin, int cin_pad, int permute, _Float16* dst,
                hipStream_t st);
void chain_forward(const ChainParams& P, int nl, const int* cout, hipStream_t st);
// mlic_set_kernel_option("chain_nj"): 16-pixel column blocks per wave (-1 = $MLIC_CHAIN_NJ or 1; 2 = the
// rounds 2-5 four-wave form); the same bits either way
void chain_set_nj(int nj);
// mlic_set_kernel_option("ep_half"): EntropyParameters on its phase's half of the grid (-1 = $MLIC_EP_HALF
// or on; 0 = the whole grid)
void chain_set_ep_half(int on);
bool chain_ep_half();

}  // namespace mlic
