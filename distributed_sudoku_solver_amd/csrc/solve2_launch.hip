// solve2_launch.hip -- separate translation unit for solve2_kernel (two boards per
// wave), compiled with -mllvm -simplifycfg-sink-common=false (see Makefile): with
// common-store sinking the three per-lane cell states are stored through a phi
// of their addresses and demoted to scratch memory.
#define SDK_NO_SOLVE_KERNEL
#define SDK_DEFINE_SOLVE2_KERNEL
#include "solve2_kernel.h"

namespace sdk {

hipError_t launch_solve2(const SolveArgs& a, unsigned grid, hipStream_t stream) {
    solve2_kernel<<<grid, 64, 0, stream>>>(a);
    return hipGetLastError();
}

}  // namespace sdk
