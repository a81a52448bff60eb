// Stand-ins for the A/B-only kernel families (ab/*.hip) in the product build (make AB=0, the
// default): the product never selects them; an explicit request (mlic_set_precision(1), $MLIC_X4=0 with a
// 5x5 conv, $MLIC_LOCAL_ATTN_VALU=1, mlic_conv_run impl 1 / 6, mlic_local_attn_run impl 0, dwpw2 form 1) fails
// loudly.
#include "../kernels.h"

namespace mlic {

static void ab_missing(const char* what) {
  throw Error(std::string("mlic: ") + what + " is an A/B-only kernel family, not in this build (make AB=1)");
}
bool ab_families_built() { return false; }
int conv_f16x3_variant(const ConvParams&) { return 0; }
void conv_f16x3_forward(const ConvParams&, const _Float16*, const _Float16*, int, hipStream_t) {
  ab_missing("conv_f16x3 (v1 tiles, precision 1)");
}
bool conv_halo_ok(const ConvParams&, int) { return false; }
void conv_halo_forward(const ConvParams&, const _Float16*, const _Float16*, int, hipStream_t) {
  ab_missing("conv_halo");
}
void local_attn_valu(const LocalAttnParams&, hipStream_t) { ab_missing("the VALU local attention"); }
bool dwpw2_lds_ok(const ConvParams&, int) { return false; }
void dwpw2_lds_forward(const ConvParams&, const _Float16*, const _Float16*, int, const float*, const float*,
                       hipStream_t) {
  ab_missing("dwpw2 (the row-pipelined LDS form, mlic_set_kernel_option(\"dwpw2\", 1))");
}

}  // namespace mlic
