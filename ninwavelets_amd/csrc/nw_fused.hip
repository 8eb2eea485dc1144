// nw_fused.hip — placeholder until the fused engine lands.
#include "nw_internal.h"
namespace nw {
bool fused_supported(int64_t, int) { return false; }
hipError_t fused_prepare(int64_t, int) { return hipSuccess; }
hipError_t launch_fused(const WDesc&, int, int, const void*, void*, int64_t, hipStream_t) {
    return hipErrorNotSupported;
}
}  // namespace nw
