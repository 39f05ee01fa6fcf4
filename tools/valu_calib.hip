// valu_calib.hip -- dev tool: VALU and LDS issue-rate ceilings on this GPU, the
// denominators of the solve kernel's compute roofline.
//
//   int-valu : 32-bit integer/logic VALU ops (v_xor/v_add/v_and), 8 independent
//              chains per lane, every CU full (32 waves/CU)
//   lds-read : ds_read_b32, conflict-free, 8 reads in flight per wave
//
// Reports wave-instructions per second chip-wide.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_calib tools/valu_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void valu_kernel(unsigned* out, unsigned seed) {
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < kIters; ++i) {
        // exactly 32 VALU per iteration: 8 independent chains x (xor, add, and, or)
        asm volatile(
            "v_xor_b32 %0, 0x55, %0\n v_xor_b32 %1, 0x55, %1\n v_xor_b32 %2, 0x55, %2\n v_xor_b32 %3, 0x55, %3\n"
            "v_xor_b32 %4, 0x55, %4\n v_xor_b32 %5, 0x55, %5\n v_xor_b32 %6, 0x55, %6\n v_xor_b32 %7, 0x55, %7\n"
            "v_add_u32 %0, 7, %0\n v_add_u32 %1, 7, %1\n v_add_u32 %2, 7, %2\n v_add_u32 %3, 7, %3\n"
            "v_add_u32 %4, 7, %4\n v_add_u32 %5, 7, %5\n v_add_u32 %6, 7, %6\n v_add_u32 %7, 7, %7\n"
            "v_and_b32 %0, 0x7fff, %0\n v_and_b32 %1, 0x7fff, %1\n v_and_b32 %2, 0x7fff, %2\n v_and_b32 %3, 0x7fff, %3\n"
            "v_and_b32 %4, 0x7fff, %4\n v_and_b32 %5, 0x7fff, %5\n v_and_b32 %6, 0x7fff, %6\n v_and_b32 %7, 0x7fff, %7\n"
            "v_or_b32 %0, 0x100, %0\n v_or_b32 %1, 0x100, %1\n v_or_b32 %2, 0x100, %2\n v_or_b32 %3, 0x100, %3\n"
            "v_or_b32 %4, 0x100, %4\n v_or_b32 %5, 0x100, %5\n v_or_b32 %6, 0x100, %6\n v_or_b32 %7, 0x100, %7\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    }
    const unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) out[blockIdx.x] = r;   // keep the chains live
}

__global__ __launch_bounds__(256) void lds_kernel(unsigned* out, unsigned seed) {
    __shared__ unsigned s[2048];
    for (int i = threadIdx.x; i < 2048; i += 256) s[i] = i * seed;
    __syncthreads();
    const unsigned addr = (unsigned)(threadIdx.x & 63) * 4u;   // lane-linear: conflict-free
    unsigned r0, r1, r2, r3, r4, r5, r6, r7, acc = 0;
    for (int i = 0; i < kIters / 8; ++i) {
        // exactly 8 ds_read_b32 per iteration, all in flight before one wait
        asm volatile(
            "ds_read_b32 %0, %8\n ds_read_b32 %1, %8 offset:256\n ds_read_b32 %2, %8 offset:512\n"
            "ds_read_b32 %3, %8 offset:768\n ds_read_b32 %4, %8 offset:1024\n ds_read_b32 %5, %8 offset:1280\n"
            "ds_read_b32 %6, %8 offset:1536\n ds_read_b32 %7, %8 offset:1792\n s_waitcnt lgkmcnt(0)\n"
            : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
            : "v"(addr) : "memory");
        acc += r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
    int cus = 0;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    cus = prop.multiProcessorCount;
    unsigned* d;
    CK(hipMalloc(&d, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int blocks = cus * 8;   // 8 x 4 waves = 32 waves per CU
    float ms;
    double waves = (double)blocks * 4;

    for (int rep = 0; rep < 2; ++rep) {
        valu_kernel<<<blocks, 256>>>(d, 7);
        CK(hipEventRecord(e0));
        for (int k = 0; k < 5; ++k) valu_kernel<<<blocks, 256>>>(d, 7 + k);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        double instr = waves * kIters * 32.0 * 5;
        printf("int-valu: %.3f ms/launch  %.3e wave-instr/s  = %.3f wave-instr/cycle/SIMD at 2.4 GHz\n",
               ms / 5, instr / (ms * 1e-3), instr / (ms * 1e-3) / (cus * 4 * 2.4e9));

        lds_kernel<<<blocks, 256>>>(d, 7);
        CK(hipEventRecord(e0));
        for (int k = 0; k < 5; ++k) lds_kernel<<<blocks, 256>>>(d, 7 + k);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        instr = waves * (kIters / 8) * 8.0 * 5;
        printf("lds-read: %.3f ms/launch  %.3e wave-instr/s  = %.3f wave-instr/cycle/CU at 2.4 GHz\n",
               ms / 5, instr / (ms * 1e-3), instr / (ms * 1e-3) / (cus * 2.4e9));
    }
    CK(hipFree(d));
    return 0;
}
