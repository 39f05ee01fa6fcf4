// solve4_launch.hip -- separate translation unit for solve4_kernel (four boards per
// wave, two per 16-bit half of every word), built like solve2_launch.hip with
// -mllvm -simplifycfg-sink-common=false (see Makefile).
#define SDK_NO_SOLVE_KERNEL
#define SDK_DEFINE_SOLVE4_KERNEL
#include "solve4_kernel.h"

namespace sdk {

hipError_t launch_solve4(const SolveArgs& a, unsigned grid, hipStream_t stream) {
    solve4_kernel<<<grid, 64, 0, stream>>>(a);
    return hipGetLastError();
}

}  // namespace sdk
