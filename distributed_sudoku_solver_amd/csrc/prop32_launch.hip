// prop32_launch.hip -- translation unit of prop32_kernel (bit-sliced root propagation, 32 boards
// per half-wave; see prop32_kernel.h)
#define SDK_NO_SOLVE_KERNEL
#define SDK_DEFINE_PROP32_KERNEL
#include "prop32_kernel.h"

namespace sdk {

// stamps non-null: the diagnostic twin that records the in-kernel clock (prop32_body)
hipError_t launch_prop32(const Prop32Args& a, unsigned grid, hipStream_t stream, uint64_t* stamps) {
    if (stamps)
        prop32_clock_kernel<<<grid, 64, 0, stream>>>(a, stamps);
    else
        prop32_kernel<<<grid, 64, 0, stream>>>(a);
    return hipGetLastError();
}

hipError_t launch_p32_scatter(const uint32_t* list, const uint8_t* sub_out, const int8_t* sub_st, const uint8_t* in,
                              uint8_t* out, int8_t* status, unsigned grid, hipStream_t stream) {
    p32_scatter_kernel<<<grid, 256, 0, stream>>>(list, sub_out, sub_st, in, out, status);
    return hipGetLastError();
}

}  // namespace sdk

#if SDK_PROP32_STATS
// profiling build only: the g_p32_stats histograms (see prop32_kernel.h), zeroed after the read
extern "C" int sdk_debug_p32_stats(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sdk::g_p32_stats), sizeof(sdk::g_p32_stats)) != hipSuccess) return -1;
    static const unsigned long long zero[4][128] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(sdk::g_p32_stats), zero, sizeof(zero)) != hipSuccess) return -1;
    return 0;
}
#endif
