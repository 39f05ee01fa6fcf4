// Probe (dev tool): where does global_load_lds_ubyte put lane L's byte in LDS?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/glds_probe tools/glds_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(const unsigned char* src, unsigned char* out) {
    __shared__ __attribute__((aligned(16))) unsigned char s[512];
    for (int i = threadIdx.x; i < 512; i += 64) s[i] = 0xEE;
    __syncthreads();
    if (threadIdx.x < 27 || (threadIdx.x >= 32 && threadIdx.x < 59))
        __builtin_amdgcn_global_load_lds((const void*)(src + threadIdx.x), (__attribute__((address_space(3))) void*)(s + 64), 1, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // unaligned dword source: lane L loads bytes 1 + 4L .. 4 + 4L
    if (threadIdx.x < 21)
        __builtin_amdgcn_global_load_lds((const void*)(src + 1 + 4 * threadIdx.x), (__attribute__((address_space(3))) void*)(s + 384), 4, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) out[i] = s[i];
}
int main() {
    unsigned char h[256], o[512];
    for (int i = 0; i < 256; ++i) h[i] = (unsigned char)(i + 1);
    unsigned char *d, *dout;
    hipMalloc(&d, 256); hipMalloc(&dout, 512);
    hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(d, dout);
    hipMemcpy(o, dout, 512, hipMemcpyDeviceToHost);
    for (int i = 0; i < 512; ++i) { printf("%02x%s", o[i], (i % 32 == 31) ? "\n" : " "); }
    return 0;
}
