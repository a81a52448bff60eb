// make AB=1: the A/B-only kernel families (ab/*.hip) are in this library
#include "../kernels.h"

namespace mlic {
bool ab_families_built() { return true; }
}  // namespace mlic
