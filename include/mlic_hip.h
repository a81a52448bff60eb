/* mlic_hip — MI355X-native (gfx950) MLIC++ encode/decode: C ABI.
 *
 * Drop-in boundary for the reference's CompressionModel API (MLIC++/models/mlicpp.py):
 *   mlic_create / mlic_destroy ........ MLICPlusPlus.__init__ + load_state_dict (mlicpp.py:14-77, 461-468);
 *                                       weights are the reference state_dict tensors, by name
 *   mlic_forward ...................... MLICPlusPlus.forward (mlicpp.py:79-185); VBR: mlicpp_vbr.py:137-519
 *   mlic_set_entropy_tables ........... GaussianConditional/EntropyBottleneck CDF buffers after update()
 *                                       (mlicpp.py:470-475; compressai _quantized_cdf/_cdf_length/_offset)
 *   mlic_compress / mlic_encoded_* .... MLICPlusPlus.compress (mlicpp.py:199-290) incl. the rANS coder
 *   mlic_decompress ................... MLICPlusPlus.decompress (mlicpp.py:292-378)
 *   mlic_pmf_to_quantized_cdf ......... compressai._CXX.pmf_to_quantized_cdf (used by update())
 *   mlic_rans_encode / mlic_rans_decode  compressai.ans.RansEncoder.encode_with_indexes /
 *                                       RansDecoder.decode_with_indexes (byte-compatible)
 *
 * Conventions: every function returns 0 on success, nonzero on error (message via mlic_last_error(),
 * thread-local); no C++ exception crosses the ABI.  Tensors are caller-owned device buffers, NCHW
 * fp32, contiguous.  `stream` is a hipStream_t (NULL = default stream); calls on one handle are
 * serialised on that stream.  The library owns its packed weights and a per-handle workspace.
 */
#ifndef MLIC_HIP_H
#define MLIC_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mlic_model mlic_model;

const char* mlic_last_error(void);
const char* mlic_version(void);

/* names/ptrs: n float32 device tensors (state_dict entries, plus "__scale_table" [64]);
 * shapes: n*4 int64 (unused dims 1), ndims: n */
int mlic_create(const char* model_name, int n, const char* const* names, const float* const* ptrs,
                const int64_t* shapes, const int* ndims, void* stream, mlic_model** out);
int mlic_destroy(mlic_model* m);

/* x [B,3,H,W] (H, W multiples of 64) -> x_hat [B,3,H,W], y_lik [B,M,H/16,W/16], z_lik [B,N,H/64,W/64];
 * outputs may be NULL.  vbr_scale = Gain[s] for *_VBR models (ignored otherwise, pass 1). */
int mlic_forward(mlic_model* m, void* stream, const float* x, int B, int H, int W, float* x_hat, float* y_lik,
                 float* z_lik, float vbr_scale);
/* *_v: one VBR gain per image (host array of B floats; NULL = 1), so one batch mixes levels
 * (BASELINE config 5); equal to B calls with the scalar form, bit for bit */
int mlic_forward_v(mlic_model* m, void* stream, const float* x, int B, int H, int W, float* x_hat, float* y_lik,
                   float* z_lik, const float* vbr_scales);

int mlic_set_entropy_tables(mlic_model* m, const int32_t* gc_cdf, const int32_t* gc_len, const int32_t* gc_off,
                            int gc_n, int gc_stride, const int32_t* eb_cdf, const int32_t* eb_len,
                            const int32_t* eb_off, int eb_n, int eb_stride);

/* compress/decompress split a batch over `lanes` host threads, each with its own HIP stream and
 * workspace, so the host rANS coding of one lane overlaps the kernels of another (default 4, or
 * $MLIC_LANES).  Results are identical for any lane count. */
int mlic_set_lanes(mlic_model* m, int lanes);
/* the lanes' HIP stream priorities are staggered (lane 0 highest, $MLIC_LANE_PRIORITY=0 disables); `base`
 * offsets this model's lanes (lane i at greatest + base + i, clamped to the device's range), so request
 * streams served by separate models drift apart as well.  Applies to lanes created afterwards (a model
 * creates its lanes on first use).  Scheduling only: results do not depend on it. */
int mlic_set_priority_base(mlic_model* m, int base);
int mlic_compress(mlic_model* m, void* stream, const float* x, int B, int H, int W, float vbr_scale);
int mlic_compress_v(mlic_model* m, void* stream, const float* x, int B, int H, int W, const float* vbr_scales);
int mlic_encoded_size(mlic_model* m, int b, size_t* y_len, size_t* z_len);
int mlic_encoded_copy(mlic_model* m, int b, uint8_t* y, uint8_t* z);
/* the coder inputs of image b from the last compress(): y symbols/indexes (all phases, coder order)
 * and z symbols; pass NULL buffers to query the counts */
int mlic_encoded_streams(mlic_model* m, int b, int64_t* n_y, int64_t* n_z, int32_t* y_sym, int32_t* y_idx,
                         int32_t* z_sym);
/* sum of -log2 of image b's y / z likelihoods in the last compress(): bpp_lik = (y + z) / (H * W) of the
 * unpadded image (loss/rd_loss.py:42-45) */
int mlic_encoded_bits(mlic_model* m, int b, double* y_bits, double* z_bits);
/* the reference's batched layout (models/mlicpp.py:215, 279-281: one y stream for a B > 1 batch,
 * phase-major and image-minor; strings = [[y], [z_0 .. z_B-1]]): images [first, first + count) of the
 * last compress coded into one stream (out = NULL queries the length; the coding runs on every call) */
int mlic_batch_stream(mlic_model* m, int first, int count, uint8_t* out, size_t cap, size_t* len);
/* decode such a stream (mlicpp.py:306-307 decodes strings[0][0] for the whole batch): one lane, the
 * images of each phase in order */
int mlic_decompress_batch_stream(mlic_model* m, void* stream, const uint8_t* y, size_t y_len, const uint8_t* const* z,
                                 const size_t* z_len, int B, int hz, int wz, float* x_hat, const float* vbr_scales);
/* y[b], z[b]: host byte strings of image b; hz, wz = latent z grid (shape returned by compress) */
int mlic_decompress(mlic_model* m, void* stream, const uint8_t* const* y, const size_t* y_len,
                    const uint8_t* const* z, const size_t* z_len, int B, int hz, int wz, float* x_hat,
                    float vbr_scale);
int mlic_decompress_v(mlic_model* m, void* stream, const uint8_t* const* y, const size_t* y_len,
                      const uint8_t* const* z, const size_t* z_len, int B, int hz, int wz, float* x_hat,
                      const float* vbr_scales);

/* module-level entry points (tests / profiling): which = local|chan|inter|intra|epa|epn|lrpn|g_a|h_a|h_s|g_s|rbu|rbws */
int mlic_run_module(mlic_model* m, void* stream, const char* which, int idx, const float* in0, const float* in1,
                    int B, int Cin, int H, int W, float* out);
int mlic_workspace_bytes(mlic_model* m, size_t* arena, size_t* weights);

/* dense-conv arithmetic: 2 = split-fp16 MFMA "f16x3" v2 tiles + specialised kernels (default; error
 * below fp32 summation-order noise), 1 = f16x3 v1 tiles, 0 = fp32 MFMA.  Also $MLIC_PRECISION. */
int mlic_set_precision(mlic_model* m, int precision);
/* g_s only (synthesis.py:56-73): 0 = the model precision above (default), 1 = its dense
 * subpel convs on fp16 operands with fp32 accumulation (one MFMA term instead of three).  Changes
 * x_hat only (forward / decompress); bitstreams and likelihoods are unaffected.  Gate: |dPSNR| <= 0.01 dB.
 * Also $MLIC_SYNTH_FP16=1. */
int mlic_set_synthesis_precision(mlic_model* m, int mode);
/* test switch: fill every workspace block with NaN (0xFF bytes) when it is handed out, so a kernel
 * reading memory its producer never wrote fails visibly (also $MLIC_POISON=1).  Off by default. */
int mlic_set_poison(mlic_model* m, int on);
/* process-wide kernel A/B switches (tests, micro-benchmarks): "x4_halo" = the conv_x4 kernel's
 * halo-staged B operand for K x K stride-1 convs (1 on, 0 off, -1 default = $MLIC_X4_HALO or on);
 * "linatt_fused" = the linear attention's output written straight into the
 * reprojection conv's packed operand ($MLIC_LINATT_FUSED); "dw_strip" = the register-strip depthwise
 * 3x3 for stride-1 planes up to 64 columns ($MLIC_DW_STRIP); "x4_splitk" = split-K for few-tile
 * 3x3 / 5x5 convs (default off, $MLIC_X4_SPLITK=1) -- set it before a handle's first call (the
 * workspace is sized for the setting in force then); "dwpw2" = the form of the fused depthwise +
 * pointwise for Cin = Cout in {96, 128, 160, 192} (-1 default = $MLIC_DWPW2 or 2: the register-row
 * dwpw3_kernel; 1 the row-pipelined LDS form, A/B-only library since round 6; 0 the round-4 dwpw_kernel) --
 * every form gives the same bits; "pw3" = the full-resolution 1x1 convs with Cin = Cout (GDN / IGDN at
 * 544 x 960) on that kernel's pointwise form (-1 default = $MLIC_PW3 or 1: from 256 K px per image; 2: every
 * grid; 0 = pw_resident, the same bits); "narrow_limit" = L: coder symbols outside [-L - 1, L] cross PCIe
 * as int32 (the encoder's overflow copy, the decoder's int32 re-decode) -- a test knob for those fallback
 * paths, bitstreams unchanged (L <= 0: the int16 range, the default); "chain_nj" = 16-pixel column blocks
 * per wave of the fused 1x1 chain (-1 default = $MLIC_CHAIN_NJ or 1; 2 = four waves of 32 pixels, the same
 * bits); "ep_half" = the slice loop's EntropyParameters chains (and its LocalContext, read by the non-anchor
 * EntropyParameters only) over their own phase's checkerboard half
 * (-1 default = $MLIC_EP_HALF or on; 0 = the whole grid: the same bits at every pixel that is read) */
int mlic_set_kernel_option(const char* name, int value);
/* 1 when this library holds the A/B-only kernel families (v1 split-fp16 tiles = precision 1, the halo
 * tiles = conv impl 6, the VALU local attention = local-attention impl 0; `make AB=1`), else 0: the
 * product build fails those requests loudly */
int mlic_ab_families(int* built);
/* fp16 range-guard fallbacks taken since the last reset (each changes the arithmetic of one call):
 * forward re-run whole in exact fp32 (the entropy model left fp16's range; compress refuses such an
 * input), forward's g_s alone, decompress's g_s alone (the same policy on both sides, so
 * decompress(compress(x)) == forward(x) bit for bit whenever compress succeeds) */
int mlic_range_fallbacks(mlic_model* m, int64_t* forward_full, int64_t* forward_gs, int64_t* decompress_gs,
                         int reset);
/* live kernel timing (HIP events on the executor stream), one category per kernel family / tile
 * instantiation: mlic_profile_categories gives the count, mlic_profile_category_name the kernel
 * name of each.  read() sums and clears. */
int mlic_set_profiling(mlic_model* m, int on);
int mlic_profile_read(mlic_model* m, int cat, int64_t* launches, double* ms, double* flops, double* bytes);
/* tab-separated per-layer table (layer, category, launches, ms, GFLOP, TFLOP/s) of the recorded
 * conv events, sorted by time; call before mlic_profile_read (which clears) */
int mlic_profile_layers(mlic_model* m, char* buf, size_t cap, size_t* written);

int mlic_profile_categories(int* n);
/* host time summed over threads since the last reset: rANS encode, rANS decode, waits on the GPU */
int mlic_host_stats(mlic_model* m, double* enc_ms, double* dec_ms, double* wait_ms, int reset);
int mlic_profile_category_name(int cat, char* buf, size_t cap);

/* kernel-level entry points (bit-exact tests, micro-benchmarks) */
/* one conv layer with a given kernel family: impl -1 = the model's choice (precision 2), 0 fp32 MFMA,
 * 1 f16x3, 2 f16x3 v2, 3 resident-weight 1x1, 4 narrow 3x3, 5 small-Cin 1x1, 6 halo-tiled 3x3,
 * 7 x4 (split-fp16, both operands staged by LDS-DMA; K in 1, 3, 5, stride 1), 8 x4 with fp16 operands
 * (single term, fp32 accumulation: the reduced-precision synthesis form).  w is torch layout
 * [Cout][Cin][K][K]; pad = K/2; epi = Epi flags of common.h (aux for GDN, res for residual).
 * Synchronous on `stream`. */
int mlic_conv_run(void* stream, int impl, const float* x, const float* w, const float* bias, float* y, int B, int Cin,
                  int Cout, int H, int W, int K, int stride, int epi, const float* aux, const float* res);
/* the kernel family the model runs a conv layer of this shape with (precision 2; no GPU needed:
 * host logic only) -> *impl.  Depends on the layer and one image's grid, never on B: the decoder must
 * reproduce the encoder's entropy parameters bit for bit whatever batch either side uses. */
int mlic_conv_choice(int B, int Cin, int Cout, int H, int W, int K, int stride, int epi, int* impl);
/* depthwise 3x3 (pad 1, stride 1|2, optional GELU); w [C][9]; synchronous on `stream` */
int mlic_dw_run(void* stream, const float* x, const float* w, const float* bias, float* y, int B, int C, int H, int W,
                int stride, int gelu);
/* fused depthwise 3x3 (stride 1, pad 1; dww [C][9], dwb [C]) + pointwise 1x1 (w [Cout][C]) with
 * epi in {0, GELU} | RES (res: [B][Cout][H][W]); C, Cout in {128, 192}; synchronous on `stream` */
int mlic_dwpw_run(void* stream, const float* x, const float* dww, const float* dwb, const float* w, const float* bias,
                  float* y, int B, int C, int Cout, int H, int W, int epi, const float* res);
/* impl as mlic_conv_run (CONV_* ids), < 0 = the model's choice; epi = Epi flags (RES in place,
   GDN/IGDN with the input as operand) */
int mlic_bench_conv(int impl, int B, int Cin, int Cout, int H, int W, int K, int stride, int epi, int iters,
                    double* ms_per, double* tflops);
int mlic_local_attn_mask(void* stream, float* out, int H, int W); /* [H*W, 25, 25] of {0, -100} */
/* LocalContext window attention: qkv [B][3C][H*W] -> out [B][25C][H*W]; impl 0 = VALU, 1 = MFMA */
int mlic_local_attn_run(void* stream, int impl, const float* qkv, const float* rel_table, const int32_t* rel_index,
                        float* out, int C, int H, int W, int B, float scale);
/* LocalContext attention (dim 32) in conv_x4's packed split layout: out = uint16 (fp16 bits)
   [B][25][npos][64], npos = ceil(H*W / 32) * 32; channel k = head*16 + d, hi at k, lo at 32 + k */
int mlic_local_attn_packed_run(void* stream, const float* qkv, const float* rel_table, const int32_t* rel_index,
                               uint16_t* out, int H, int W, int B, float scale);
/* the same for one checkerboard phase's query pixels only (ckbd 1: anchors, (y + x) odd; 2: non-anchors;
   W even), written at the squeezed position y * W / 2 + x / 2: npos = ceil(H*W/2 / 32) * 32 (round 6: the
   slice loop's LocalContext, whose only consumer reads the non-anchor pixels) */
int mlic_local_attn_packed_half_run(void* stream, const float* qkv, const float* rel_table, const int32_t* rel_index,
                                    uint16_t* out, int H, int W, int B, float scale, int ckbd);
int mlic_image_sq_err_u8(void* stream, const float* a, const float* b, int B, int64_t n_per, double* out);
/* per-image sum of -log2(lik) over n_per elements (fixed reduction order); synchronous */
int mlic_neglog2_sum(void* stream, const float* lik, int B, int64_t n_per, double* out);
/* GaussianConditional likelihood (compressai, eval; mlicpp.py:132,168) element-wise: lik = max(Phi((0.5-|v|)/s')
 * - Phi((-0.5-|v|)/s'), 1e-9), v = round(y - m), s' = max(s, 0.11); vbr_scale != 1 evaluates it at (y, s, m) *
 * vbr_scale (mlicpp_vbr.py:292).  The kernel's device function is the one the slice loop runs. */
int mlic_gaussian_likelihood(void* stream, const float* y, const float* scales, const float* means, int64_t n,
                             float vbr_scale, float* lik);
/* build_indexes (utils/ckbd.py:128-129): idx = (ntable-1) - #{t in table[:-1] : max(s, 0.11) <= t} */
int mlic_scale_indexes(void* stream, const float* scales, int64_t n, const float* table, int ntable, int32_t* out);

/* host entropy coder (compressai-compatible) */
int mlic_pmf_to_quantized_cdf(const float* pmf, int n, int precision, int32_t* cdf_out /* n + 1 */);
int mlic_rans_encode(const int32_t* symbols, const int32_t* indexes, int64_t n, const int32_t* cdf,
                     const int32_t* cdf_len, const int32_t* offset, int n_tables, int stride, uint8_t* out,
                     size_t cap, size_t* written);
int mlic_rans_decode(const uint8_t* data, size_t nbytes, const int32_t* indexes, int64_t n, const int32_t* cdf,
                     const int32_t* cdf_len, const int32_t* offset, int n_tables, int stride, int32_t* out);
/* The decompress path's narrow decode, on the host alone (tests): the stream is decoded in `nparts`
 * consecutive pieces of n / nparts symbols (the 20 phases of one image) with uint8 table indexes, each
 * piece first into int16 and, when a value falls outside the narrow range (int16, or
 * mlic_set_kernel_option("narrow_limit", L)), reset to the piece's start and decoded again into int32 --
 * exactly PhaseDecoder::run's per-image step.  out: all n symbols as int32; *widened: pieces that
 * took the int32 fallback. */
int mlic_rans_decode_narrow(const uint8_t* data, size_t nbytes, const uint8_t* indexes, int64_t n, int nparts,
                            const int32_t* cdf, const int32_t* cdf_len, const int32_t* offset, int n_tables,
                            int stride, int32_t* out, int* widened);

#ifdef __cplusplus
}
#endif
#endif
