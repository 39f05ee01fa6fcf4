// read_ceiling.hip -- HBM read ceiling of this GPU for the checker's access pattern (dev tool).
//
// The checker (check_kernel.h) streams 81 B per board and writes 1 B: it is a READ stream.  The
// guide's 6.29 TB/s is a float4 COPY (half of it writes).  This measures what a pure read stream
// reaches -- dwordx4 loads, grid-stride, U loads in flight per thread, an XOR fold and one dword
// store per thread -- over the checker's 8.1 GB, with and without the non-temporal hint, at the
// checker's grid (blocks of 256 threads, B blocks per CU), so the checker's fraction of 8 TB/s can
// be read against the fraction a plain read reaches.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/read_ceiling tools/read_ceiling.hip
// run:   tools/read_ceiling [bytes=8100000000]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ src, size_t n4, unsigned* __restrict__ out) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(&src[i + u * stride]) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
    }
    for (; i < n4; i += stride) acc ^= src[i];
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// the checker's access pattern without its arithmetic: a 256-board tile (20,736 B) per workgroup,
// grid-stride over tiles, the next tile's six dwordx4 per thread in flight while the current one
// goes through LDS (stores, barrier, one dword read per thread, barrier) -- check_kernel minus
// check_board_lds.  SPIN adds ~SPIN dependent VALU per tile and thread, standing in for the check.
template <int SPIN, int READS = 0, int STORE = 0>
__global__ __launch_bounds__(256) void tile_kernel(const u32x4* __restrict__ src, size_t ntiles, unsigned* __restrict__ out,
                                                   unsigned char* __restrict__ bytes = nullptr) {
    __shared__ u32x4 tile[1296 + 1];
    __shared__ u32x4 vst[16];          // STORE 2: the tile's 256 verdict bytes
    const int t = threadIdx.x;
    u32x4 pre[6];
    unsigned acc = 0;
    size_t tix = blockIdx.x;
    unsigned char pend[STORE >= 16 ? STORE : 1];
    size_t ptix[STORE >= 16 ? STORE : 1];
    unsigned npend = 0;
    auto load = [&](size_t ti) {
        const u32x4* s4 = src + ti * 1296;
#pragma unroll
        for (int j = 0; j < 5; ++j) pre[j] = __builtin_nontemporal_load(&s4[j * 256 + t]);
        if (t < 16) pre[5] = __builtin_nontemporal_load(&s4[5 * 256 + t]);
    };
    if (tix < ntiles) load(tix);
    for (; tix < ntiles; tix += gridDim.x) {
#pragma unroll
        for (int j = 0; j < 5; ++j) tile[j * 256 + t] = pre[j];
        if (t < 16) tile[5 * 256 + t] = pre[5];
        __syncthreads();
        if (tix + gridDim.x < ntiles) load(tix + gridDim.x);
        unsigned v = reinterpret_cast<const unsigned*>(tile)[(t * 81) >> 2];
#pragma unroll
        for (int k = 1; k < READS; ++k) v ^= reinterpret_cast<const unsigned*>(tile)[((t * 81) >> 2) + k];
#pragma unroll 1
        for (int k = 0; k < SPIN; ++k) v = v * 2654435761u + (unsigned)k;
        acc ^= v;
        if (STORE == 1) bytes[tix * 256 + t] = (unsigned char)v;
        if (STORE == 3) __builtin_nontemporal_store((unsigned char)v, &bytes[tix * 256 + t]);
        if (STORE >= 16) {              // deferred: the last STORE tiles' bytes kept, then written in a burst
            pend[npend % STORE] = (unsigned char)v;
            ptix[npend % STORE] = tix;
            if (++npend % STORE == 0) {
#pragma unroll
                for (int q = 0; q < STORE; ++q) __builtin_nontemporal_store(pend[q], &bytes[ptix[q] * 256 + t]);
            }
        }
        if (STORE == 2) {               // through LDS: one 16-B store per lane of the first 16 lanes
            reinterpret_cast<unsigned char*>(vst)[t] = (unsigned char)v;
            __syncthreads();
            if (t < 16) reinterpret_cast<u32x4*>(bytes + tix * 256)[t] = vst[t];
        }
        __syncthreads();
    }
    out[blockIdx.x * 256 + t] = acc;
}

template <int SPIN, int READS = 0, int STORE = 0>
int run_tile(const u32x4* src, size_t n4, unsigned* out, int cus, int bpc, unsigned char* bytes = nullptr);

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

template <int U, bool NT>
int run(const char* name, const u32x4* src, size_t n4, unsigned* out, int cus, int bpc) {
    const unsigned grid = (unsigned)(cus * bpc);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 10; ++w) read_kernel<U, NT><<<grid, 256>>>(src, n4, out);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) read_kernel<U, NT><<<grid, 256>>>(src, n4, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double tbs = (double)n4 * 16 / (ms * 1e-3) / 1e12;
    std::printf("%-8s U=%d blocks/CU=%2d  %.3f ms  %.3f TB/s  %.1f %% of 8 TB/s\n", name, U, bpc, ms, tbs, tbs / 8.0 * 100);
    return 0;
}

template <int SPIN, int READS, int STORE>
int run_tile(const u32x4* src, size_t n4, unsigned* out, int cus, int bpc, unsigned char* bytes) {
    const unsigned grid = (unsigned)(cus * bpc);
    const size_t ntiles = n4 / 1296;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 10; ++w) tile_kernel<SPIN, READS, STORE><<<grid, 256>>>(src, ntiles, out, bytes);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) tile_kernel<SPIN, READS, STORE><<<grid, 256>>>(src, ntiles, out, bytes);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double tbs = (double)ntiles * 1296 * 16 / (ms * 1e-3) / 1e12;
    std::printf("tile     spin=%3d reads=%2d store=%d blocks/CU=%2d  %.3f ms  %.3f TB/s  %.1f %% of 8 TB/s\n", SPIN,
                READS, (int)STORE, bpc, ms, tbs, tbs / 8.0 * 100);
    return 0;
}

int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8100000000ull;
    const size_t n4 = bytes / 16;
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    u32x4* src;
    unsigned* out;
    CK(hipMalloc(&src, n4 * 16));
    CK(hipMemset(src, 0x5a, n4 * 16));
    CK(hipMalloc(&out, (size_t)cus * 16 * 256 * 4));
    std::printf("read ceiling: %.2f GB, %d CUs\n", n4 * 16 / 1e9, cus);
    unsigned char* vbytes;
    CK(hipMalloc(&vbytes, n4 * 16 / 81 + 4096));
    for (int bpc : {3, 4}) {
        if (run_tile<0>(src, n4, out, cus, bpc) || run_tile<0, 22>(src, n4, out, cus, bpc) ||
            run_tile<0, 22, 1>(src, n4, out, cus, bpc, vbytes) || run_tile<0, 22, 2>(src, n4, out, cus, bpc, vbytes) ||
            run_tile<0, 22, 3>(src, n4, out, cus, bpc, vbytes) || run_tile<0, 22, 16>(src, n4, out, cus, bpc, vbytes) ||
            run_tile<0, 22, 32>(src, n4, out, cus, bpc, vbytes) || run_tile<100>(src, n4, out, cus, bpc))
            return 1;
    }
    CK(hipFree(vbytes));
    for (int bpc : {3, 4, 8}) {
        if (run<4, true>("nt", src, n4, out, cus, bpc) || run<4, false>("plain", src, n4, out, cus, bpc) ||
            run<8, true>("nt", src, n4, out, cus, bpc))
            return 1;
    }
    CK(hipFree(src));
    CK(hipFree(out));
    return 0;
}
