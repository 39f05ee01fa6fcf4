// prop32_launch.hip -- translation unit of prop32_kernel (bit-sliced root propagation, 32 boards
// per half-wave; see prop32_kernel.h)
#define SDK_NO_SOLVE_KERNEL
#define SDK_DEFINE_PROP32_KERNEL
#include "prop32_kernel.h"

namespace sdk {

hipError_t launch_prop32(const Prop32Args& a, unsigned grid, hipStream_t stream) {
    prop32_kernel<<<grid, 64, 0, stream>>>(a);
    return hipGetLastError();
}

}  // namespace sdk
