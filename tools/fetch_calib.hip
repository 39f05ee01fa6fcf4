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

int main(int argc, char** argv) {
    const unsigned n = argc > 1 ? (unsigned)atoi(argv[1]) : 10000000u;
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
        fetch_kernel<<<grid, 64>>>(in, out, status, n);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("fetch_kernel n=%u records: %.3f ms, algorithmic %.1f MB read + %.1f MB written\n", n, ms,
               n * 81 / 1e6, n * 82 / 1e6);
    }
    return 0;
}
