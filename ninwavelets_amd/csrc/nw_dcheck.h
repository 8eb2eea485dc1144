// nw_dcheck.h — debug-kernel bounds checks (SURVEY.md §5 "Race detection / sanitizers").
//
// Built only into the debug library (`make -C ninwavelets_amd/csrc debug` ->
// libninwave_debug.so, -DNW_DEBUG_BOUNDS; load it with NINWAVE_LIB).  NW_DCHECK(cond) in a
// kernel counts a failing check in a device word of its source file and records the first
// failing site; nothing traps, so a broken index shows up as a status, not as a GPU fault.
// The API synchronises after every call in that build, reads and clears every file's words
// and fails with NW_E_BOUNDS naming file:line.  The product library compiles the checks out.
#pragma once
#include <hip/hip_runtime.h>

namespace nw {
// (fails, first failing site, source file of the kernels) of one translation unit, cleared
using DcheckTake = hipError_t (*)(unsigned* fails, unsigned* site, const char** file);
int dcheck_register(DcheckTake fn);   // nw_api.cpp; called at static initialisation
constexpr unsigned kDcheckHeaderSite = 100000;   // sites in nw_fft_dev.h: line + this
}  // namespace nw

#ifdef NW_DEBUG_BOUNDS
namespace {
__device__ unsigned g_nw_dcheck[2];   // failing checks, first failing site
__device__ __noinline__ void nw_dcheck_fail(unsigned site) {
    atomicAdd(&g_nw_dcheck[0], 1u);
    atomicCAS(&g_nw_dcheck[1], 0u, site);
}
hipError_t nw_dcheck_take(unsigned* fails, unsigned* site, const char** file) {
    unsigned h[2] = {0u, 0u};
    hipError_t e = hipMemcpyFromSymbol(h, HIP_SYMBOL(g_nw_dcheck), sizeof h);
    if (e != hipSuccess) return e;
    *fails = h[0];
    *site = h[1];
    *file = __BASE_FILE__;
    if (h[0]) {
        const unsigned z[2] = {0u, 0u};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_nw_dcheck), z, sizeof z);
    }
    return e;
}
const int g_nw_dcheck_registered = nw::dcheck_register(&nw_dcheck_take);
}  // namespace
// (variadic: template argument lists in the condition carry commas)
#define NW_DCHECK(...)                                          \
    do {                                                        \
        if (!(__VA_ARGS__)) nw_dcheck_fail((unsigned)__LINE__);  \
    } while (0)
#define NW_DCHECK_H(...)                                                                \
    do {                                                                                \
        if (!(__VA_ARGS__)) nw_dcheck_fail(nw::kDcheckHeaderSite + (unsigned)__LINE__);  \
    } while (0)
#else
#define NW_DCHECK(...) \
    do {               \
    } while (0)
#define NW_DCHECK_H(...) \
    do {                 \
    } while (0)
#endif
