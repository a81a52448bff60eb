// Conv kernel selection: one place decides which kernel family runs a conv layer, so the model,
// the per-kernel C-ABI test entry (mlic_conv_run) and the micro-benchmark all run the same choice.
#include "kernels.h"

#include <cstdlib>

namespace mlic {

// $MLIC_X4=0 disables the LDS-DMA x4 kernel (A/B switch)
static bool x4_on() {
  static const bool on = [] {
    const char* e = std::getenv("MLIC_X4");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

// kernel sizes x4 takes (digits of $MLIC_X4_K, default "135"): the A/B switch for 1x1 / 5x5 layers
// (5x5: the context reprojections, 8 x 68 x 120, 64..320 channels: x4 1.1-1.9x the halo kernel)
static bool x4_k_on(int K) {
  static const int mask = [] {
    const char* e = std::getenv("MLIC_X4_K");
    int m = 0;
    for (const char* c = e ? e : "135"; *c; ++c)
      if (*c >= '0' && *c <= '9') m |= 1 << (*c - '0');
    return m;
  }();
  return (mask >> K) & 1;
}

// The choice depends on the layer's shape and ONE image's grid, never on the batch: kernel families
// round differently, and the decoder must rebuild the encoder's entropy parameters bit for bit
// whatever batch either side runs (a stream coded in a batch of 8 decodes alone).  The grid-fill
// thresholds are per image, sized for the bench's batches (8 per lane).
int conv_select(const ConvParams& P, const ConvWeights& w, int precision) {
  if (conv_smallcin_ok(P)) return CONV_SMALLCIN;  // exact fp32 VALU, all precisions
  if (conv_narrow_ok(P)) return CONV_NARROW;      // exact fp32 VALU, all precisions
  if (precision == 0 || !w.wh) return CONV_F32;
  if (precision == 1) return CONV_X3;
  // resident weights: from >= 1 K pixels per image (Kodak-size latent 32 x 48, 16 images: 2-3x x3v2
  // on every latent 1x1 it serves; the 1080p latent and the full-resolution layers are far above)
  if ((int64_t)P.Ho * P.Wo >= 1024 && pw_resident_ok(P, w.cin_pad)) return CONV_PW;
  // x4: the dense 3x3 convs with wide Cout (g_s / h_s subpel convs), the 5x5 reprojections, the big
  // 1x1 GEMMs (the hoisted EntropyParameters hyper columns, h_s's last layer: Cin x Cout >= 2^18) and
  // the mid-size 1x1s with Cin, Cout >= 192 that the resident kernel does not serve (context q/k/v
  // 224..288, the LRP's 352..640 -> 224, the small-decoder EntropyParameters: 1.07-2.1x x3v2 on the
  // 1080p and Kodak-size latents, the activation pack included).  Any grid: the split-K path
  // (x4_splitk) fills the chip for few-tile 3x3 / 5x5 shapes (h_s at the z grid, 8 x 12 .. 17 x 30:
  // 1.5-2.5x x3v2)
  // Round 3: 3x3 convs from Cout 64 too (the small-decoder model's dense channel-context convs
  // 96..288 -> 96 / 128 at the latent grid: 1.26-1.75x x3v2)
  const bool big1 = (int64_t)P.Cin * P.Cout >= (1 << 18), mid1 = P.Cin >= 192 && P.Cout >= 192;
  const bool x4_shape = P.K == 1 ? (big1 || mid1) : P.Cout >= 64;
  if (w.wx4 && x4_on() && x4_k_on(P.K) && x4_shape && conv_x4_ok(P, w.cin_pad)) return CONV_X4;
  // halo: the 5x5 reprojection (145 vs 126 TF/s); for 3x3 the 8-wave 256x256 x3v2 tile is faster
  // (243 vs 232 TF/s on the g_s subpel conv), for 1x1 the halo staging does not pay
  if (P.K == 5 && conv_halo_ok(P, w.cin_pad) &&
      (int64_t)((P.Cout + 127) / 128) * ((P.Wo + 31) / 32) * ((P.Ho + 3) / 4) >= 8)
    return CONV_HALO;
  return CONV_X3V2;
}

int conv_prof_cat(int impl, const ConvParams& P) {
  switch (impl) {
    case CONV_F32: return PCAT_CONV_F32 + conv_variant(P);
    case CONV_X3: return PCAT_CONV_X3 + conv_f16x3_variant(P);
    case CONV_X3V2: {
      const int v = conv_x3v2_variant(P);
      return v == 3 ? PCAT_CONV_X3V2_WIDE : PCAT_CONV_X3V2 + v;
    }
    case CONV_PW: return PCAT_CONV_PW;
    case CONV_NARROW: return PCAT_CONV_NARROW;
    case CONV_HALO: return PCAT_CONV_HALO;
    case CONV_X4:
    case CONV_X4H: return PCAT_CONV_X4;
    default: return PCAT_CONV_SMALLCIN;
  }
}

int64_t conv_ws_bytes(int impl, const ConvParams& P, const ConvWeights& w) {
  // x4: the packed activations, then (256-byte aligned) the split-K partial planes
  if (impl != CONV_X4 && impl != CONV_X4H) return 0;
  const bool hi = impl == CONV_X4H;
  const int64_t act = x4_direct_ok(P, hi) ? 0 : (2 * x4_act_halves(P, w.cin_pad, hi) + 255) / 256 * 256;
  return act + x4_part_bytes(P, w.cin_pad, hi);
}

void conv_run(int impl, const ConvParams& P0, const ConvWeights& w, hipStream_t st, void* ws) {
  // the split-fp16 families read the prescaled hi/lo weights: their epilogues undo the row scale;
  // the fp32 families read the unscaled fp32 weights
  ConvParams P = P0;
  const bool split = impl == CONV_X3 || impl == CONV_X3V2 || impl == CONV_PW || impl == CONV_HALO || impl == CONV_X4 ||
                     impl == CONV_X4H;
  P.wexp = split ? w.wexp : 0;
  switch (impl) {
    case CONV_F32: conv_forward(P, st); break;
    case CONV_X3: conv_f16x3_forward(P, w.wh, w.wl, w.cin_pad, st); break;
    case CONV_X3V2: conv_x3v2_forward(P, w.wh, w.wl, w.cin_pad, st); break;
    case CONV_PW: pw_resident_forward(P, w.wh, w.wl, w.cin_pad, st); break;
    case CONV_NARROW: conv_narrow_forward(P, st); break;
    case CONV_SMALLCIN: conv_smallcin_forward(P, st); break;
    case CONV_HALO: conv_halo_forward(P, w.wh, w.wl, w.cin_pad, st); break;
    case CONV_X4:
    case CONV_X4H: {
      const bool hi = impl == CONV_X4H;
      const _Float16* wx = hi ? w.wx4h : w.wx4;
      const bool direct = x4_direct_ok(P, hi);  // 1x1: B rows built from the fp32 input in the kernel
      MLIC_CHECK((ws || direct) && wx, "conv_x4: workspace and packed weights required");
      _Float16* act = direct ? nullptr : static_cast<_Float16*>(ws);
      const int64_t abytes = direct ? 0 : (2 * x4_act_halves(P, w.cin_pad, hi) + 255) / 256 * 256;
      float* part = x4_part_bytes(P, w.cin_pad, hi) > 0 ? reinterpret_cast<float*>(static_cast<char*>(ws) + abytes)
                                                         : nullptr;
      if (!direct) x4_pack_act(P, w.cin_pad, act, st, hi);
      conv_x4_forward(P, act, wx, w.cin_pad, st, part, hi);
      break;
    }
    default: throw Error("mlic: unknown conv implementation " + std::to_string(impl));
  }
}

const char* prof_cat_name(int cat) {
  static const char* names[PCAT_COUNT] = {
      "conv_mfma_kernel<64,64>",     "conv_mfma_kernel<64,128>",  "conv_mfma_kernel<128,64>",
      "conv_mfma_kernel<128,128>",   "conv_f16x3_kernel<32,256>", "conv_f16x3_kernel<64,128>",
      "conv_f16x3_kernel<128,64>",   "conv_f16x3_kernel<128,128>", "conv_x3v2_kernel<64,128>",
      "conv_x3v2_kernel<128,256>",   "conv_x3v2_kernel<128,128>", "conv_x3v2_kernel<256,256>",
      "pw_resident_kernel",
      "conv3x3_narrow_kernel",       "conv1x1_smallcin_kernel",   "conv_halo_kernel",
      "dw3x3_kernel",
      "local_attn_kernel",           "linear_attention",          "elementwise",
      "conv_x4_kernel",              "chain_kernel",              "dwpw_kernel"};
  return (cat >= 0 && cat < PCAT_COUNT) ? names[cat] : "";
}

}  // namespace mlic
