// solve4_launch.hip -- separate translation unit for solve4_kernel (four boards per
// wave, two per 16-bit half of every word), built like solve2_launch.hip with
// -mllvm -simplifycfg-sink-common=false (see Makefile).
#define SDK_NO_SOLVE_KERNEL
#define SDK_DEFINE_SOLVE4_KERNEL
#include "solve4_kernel.h"
#include "expand4_kernel.h"

namespace sdk {

hipError_t launch_solve4(const SolveArgs& a, unsigned grid, hipStream_t stream) {
    if (a.donate)
        solve4_kernel<true><<<grid, 64, 0, stream>>>(a);
    else if (a.save)   // the split phase of a phased solve: saves the stacks it stops
        solve4_kernel<false, true><<<grid, 64, 0, stream>>>(a);
    else if (a.found)  // a first-solution scan of a lex frontier: cancels boards above the lowest hit
        solve4_kernel<false, false, true><<<grid, 64, 0, stream>>>(a);
    else
        solve4_kernel<false><<<grid, 64, 0, stream>>>(a);
    return hipGetLastError();
}

hipError_t launch_expand4(const ExpandArgs& a, unsigned grid, hipStream_t stream) {
    expand4_kernel<<<grid, 64, 0, stream>>>(a);
    return hipGetLastError();
}

int solve4_dn_blocks_per_cu() {
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, solve4_kernel<true>, 64, 0) != hipSuccess) return -1;
    return blocks;
}

}  // namespace sdk

#if SDK_SOLVE4_PROFILE
// profiling build only: the g_prof4 counters (see solve4_kernel.h), optionally zeroed
extern "C" int sdk_debug_prof4(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sdk::g_prof4), sizeof(sdk::g_prof4)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long zero[10] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(sdk::g_prof4), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

#if SDK_SOLVE4_TIMELINE
// timeline build only: the per-workgroup stamps of the last launch (see solve4_kernel.h), zeroed after
extern "C" int sdk_debug_tl4(unsigned long long* out, int n) {
    if (n > sdk::kTl4Max) n = sdk::kTl4Max;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sdk::g_tl4), (size_t)n * 4 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    static unsigned long long zero[sdk::kTl4Max][4];
    if (hipMemcpyToSymbol(HIP_SYMBOL(sdk::g_tl4), zero, sizeof(zero)) != hipSuccess) return -1;
    return 0;
}
#endif
