// fetch_calib.hip -- dev tool: what rocprofv3 FETCH_SIZE / WRITE_SIZE report for the solve
// kernels' global access pattern, to correct their per-launch HBM traffic.
//
// Moves n records exactly like solve4_kernel / solve2_kernel move a board: each 32-lane
// half takes one record, lane j < 27 loads the 3 bytes j, j+27, j+54 (byte loads) and
// stores 3 output bytes at the same offsets, lane 0 stores 1 status byte.  Algorithmic
// traffic: 81 n read + 82 n written.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(64) void fetch_kernel(const unsigned char* __restrict__ in, unsigned char* __restrict__ out,
                                                   unsigned char* __restrict__ status, unsigned n) {
    const int hl = threadIdx.x & 31, half = threadIdx.x >> 5;
    for (unsigned r = blockIdx.x * 2 + half; r < n; r += gridDim.x * 2) {
        const unsigned char* src = in + (size_t)r * 81;
        unsigned char* dst = out + (size_t)r * 81;
        unsigned v = 0;
        if (hl < 27) {
            const unsigned a = src[hl], b = src[hl + 27], c = src[hl + 54];
            dst[hl] = (unsigned char)(a + 1);
            dst[hl + 27] = (unsigned char)(b + 1);
            dst[hl + 54] = (unsigned char)(c + 1);
            v = a + b + c;
        }
        for (int m = 16; m >= 1; m >>= 1) v += __shfl_xor(v, m);
        if (hl == 0) status[r] = (unsigned char)v;
    }
}

// The same records and bytes, output written 16 records per wave with 16-B stores: a
// group's 1296 B start 16-B aligned and are covered by 81 dwordx4 stores (lanes 0..63, then
// 0..16), so every output line is written whole, at once.  Mode 1 of main: what WRITE_SIZE
// reports when the 81-B records are not written one by one.
__global__ __launch_bounds__(64) void fetch_kernel_wide(const unsigned char* __restrict__ in,
                                                        unsigned char* __restrict__ out,
                                                        unsigned char* __restrict__ status, unsigned n) {
    const unsigned groups = n / 16;
    for (unsigned g = blockIdx.x; g < groups; g += gridDim.x) {
        const uint4* src = reinterpret_cast<const uint4*>(in + (size_t)g * 1296);
        uint4* dst = reinterpret_cast<uint4*>(out + (size_t)g * 1296);
        for (unsigned k = threadIdx.x; k < 81; k += 64) {
            uint4 v = src[k];
            v.x += 0x01010101u; v.y += 0x01010101u; v.z += 0x01010101u; v.w += 0x01010101u;
            dst[k] = v;
        }
        if (threadIdx.x < 4)
            reinterpret_cast<unsigned*>(status + (size_t)g * 16)[threadIdx.x] = 0x01010101u;
    }
}

int main(int argc, char** argv) {
    const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : 10000000u;
    const int mode = argc > 2 ? atoi(argv[2]) : 0;   // 0: the solvers' byte pattern, 1: wide stores
    unsigned char *in, *out, *status;
    CK(hipMalloc(&in, (size_t)n * 81));
    CK(hipMalloc(&out, (size_t)n * 81));
    CK(hipMalloc(&status, n));
    CK(hipMemset(in, 3, (size_t)n * 81));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const unsigned grid = prop.multiProcessorCount * 32;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(a));
        if (mode == 1)
            fetch_kernel_wide<<<grid, 64>>>(in, out, status, n);
        else
            fetch_kernel<<<grid, 64>>>(in, out, status, n);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("fetch_kernel mode %d n=%u records: %.3f ms, algorithmic %.1f MB read + %.1f MB written\n", mode, n, ms,
               n * 81 / 1e6, n * 82 / 1e6);
    }
    return 0;
}
