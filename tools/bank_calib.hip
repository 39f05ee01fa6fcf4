// bank_calib.hip -- dev tool: does the VALU issue rate of 2- and 3-VGPR-source ops depend on the
// source registers' banks (register index mod 4)?  tools/issue_calib.hip measured 3-source VOP3
// (v_or3 / v_bitop3) at ~1.0 wave-instruction per SIMD quad-cycle and 1-source VOP2 at ~1.7 with
// whatever registers the compiler picked; prop32's step is 3-source ops throughout.  Each kernel
// here is a raw asm loop over fixed physical registers: 8 independent chains whose destinations
// sit in bank 0 (v8, v12, ... v36), the other sources in chosen banks.  Each wave stamps
// s_memtime around its loop; the rate per SIMD quad-cycle is waves-per-SIMD x instructions over
// the waves' mean elapsed quad-cycles.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/bank_calib tools/bank_calib.hip
// run:   tools/bank_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

// 8 chains x the op with srcs (S1, S2): "OP v8, v8, S1, S2" ... "OP v36, v36, S1, S2"
#define C8_3(OP, S1, S2, SUF)                                                                     \
    OP " v8, v8, " S1 ", " S2 SUF "\n" OP " v12, v12, " S1 ", " S2 SUF "\n" OP " v16, v16, " S1 ", " S2 SUF \
    "\n" OP " v20, v20, " S1 ", " S2 SUF "\n" OP " v24, v24, " S1 ", " S2 SUF "\n" OP " v28, v28, " S1    \
    ", " S2 SUF "\n" OP " v32, v32, " S1 ", " S2 SUF "\n" OP " v36, v36, " S1 ", " S2 SUF "\n"
#define C8_2(OP, S1)                                                                               \
    OP " v8, " S1 ", v8\n" OP " v12, " S1 ", v12\n" OP " v16, " S1 ", v16\n" OP " v20, " S1 ", v20\n" OP \
    " v24, " S1 ", v24\n" OP " v28, " S1 ", v28\n" OP " v32, " S1 ", v32\n" OP " v36, " S1 ", v36\n"
// 3-source chains with the chains' own registers spread over banks 0..3 (v8..v15) and srcs fixed
#define C8_3S(OP, S1, S2, SUF)                                                                    \
    OP " v8, v8, " S1 ", " S2 SUF "\n" OP " v9, v9, " S1 ", " S2 SUF "\n" OP " v10, v10, " S1 ", " S2 SUF \
    "\n" OP " v11, v11, " S1 ", " S2 SUF "\n" OP " v12, v12, " S1 ", " S2 SUF "\n" OP " v13, v13, " S1    \
    ", " S2 SUF "\n" OP " v14, v14, " S1 ", " S2 SUF "\n" OP " v15, v15, " S1 ", " S2 SUF "\n"

#define INIT                                                                                       \
    "s_mov_b64 s[0:1], exec\n s_mov_b64 vcc, exec\n v_mov_b32 v1, %[a]\n v_mov_b32 v2, %[b]\n v_mov_b32 v3, %[a]\n v_mov_b32 v5, %[b]\n"           \
    "v_mov_b32 v6, %[a]\n v_mov_b32 v40, %[a]\n v_mov_b32 v44, %[b]\n"                            \
    "v_mov_b32 v8, %[a]\n v_mov_b32 v9, %[b]\n v_mov_b32 v10, %[a]\n v_mov_b32 v11, %[b]\n"         \
    "v_mov_b32 v12, %[a]\n v_mov_b32 v13, %[b]\n v_mov_b32 v14, %[a]\n v_mov_b32 v15, %[b]\n"       \
    "v_mov_b32 v16, %[a]\n v_mov_b32 v20, %[b]\n v_mov_b32 v24, %[a]\n v_mov_b32 v28, %[b]\n"       \
    "v_mov_b32 v32, %[a]\n v_mov_b32 v36, %[b]\n"
#define CLOB "v1", "v2", "v3", "v5", "v6", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", \
             "v20", "v24", "v28", "v32", "v36", "v40", "v44"

template <int K>
__device__ __forceinline__ void body(unsigned a, unsigned b, int iters) {
    // 4 x 8 = 32 instructions per iteration
#define LOOP(X) asm volatile(INIT "1:\n" X X X X "s_sub_u32 %[n], %[n], 1\n s_cmp_lg_u32 %[n], 0\n s_cbranch_scc1 1b\n" \
                             : [n] "+s"(iters) : [a] "v"(a), [b] "v"(b) : CLOB, "scc", "s0", "s1", "vcc")
    if (K == 0) LOOP(C8_3("v_or3_b32", "v1", "v2", ""));                 // banks 0 | 1 | 2
    if (K == 1) LOOP(C8_3("v_or3_b32", "v40", "v44", ""));               // banks 0 | 0 | 0
    if (K == 2) LOOP(C8_3("v_bitop3_b32", "v1", "v2", " bitop3:0xe8"));  // banks 0 | 1 | 2
    if (K == 3) LOOP(C8_3("v_bitop3_b32", "v40", "v44", " bitop3:0xe8")); // 0 | 0 | 0
    if (K == 4) LOOP(C8_3("v_bitop3_b32", "v1", "v5", " bitop3:0xe8"));  // 0 | 1 | 1
    if (K == 5) LOOP(C8_3("v_bitop3_b32", "v40", "v1", " bitop3:0xe8")); // 0 | 0 | 1
    if (K == 6) LOOP(C8_3("v_bitop3_b32", "v1", "v1", " bitop3:0xe8"));  // 0 | 1 | 1 (one register)
    if (K == 7) LOOP(C8_3("v_bitop3_b32", "v1", "v3", " bitop3:0xe8"));  // 0 | 1 | 3
    if (K == 8) LOOP(C8_3("v_and_or_b32", "v1", "v2", ""));              // 0 | 1 | 2
    if (K == 9) LOOP(C8_3("v_add3_u32", "v1", "v2", ""));                // 0 | 1 | 2
    if (K == 10) LOOP(C8_2("v_and_b32", "v1"));                         // VOP2 1 | 0
    if (K == 11) LOOP(C8_2("v_and_b32", "v40"));                        // VOP2 0 | 0
    if (K == 12) LOOP(C8_2("v_and_b32", "0x7f"));                       // VOP2 const | 0
    if (K == 13) LOOP(C8_2("v_and_b32_e64", "v1"));                     // VOP3-encoded 2 source 1 | 0
    if (K == 14) LOOP(C8_3S("v_bitop3_b32", "v1", "v2", " bitop3:0xe8")); // chains over banks 0..3
    if (K == 15) LOOP(C8_3("v_bitop3_b32", "v1", "v2", " bitop3:0xfe"));  // OR3 as bitop3, 0 | 1 | 2
    if (K == 16) LOOP(C8_3("v_cndmask_b32_e64", "v1", "s[0:1]", ""));     // 2 VGPRs + SGPR mask
    if (K == 17) LOOP(C8_2("v_cndmask_b32_e32", "v1"));                  // VOP2 with vcc
    if (K == 18) LOOP(C8_2("v_pk_add_u16", "v1"));                       // VOP3P 2 source 1 | 0
    if (K == 19) LOOP(C8_3("v_lshl_or_b32", "v1", "v2", ""));            // 0 | 1 | 2
    if (K == 20) LOOP(C8_3("v_perm_b32", "v1", "v2", ""));               // 0 | 1 | 2
    if (K == 21) LOOP(C8_3("v_mad_u32_u24", "v1", "v2", ""));            // 0 | 1 | 2
    if (K == 22) LOOP(C8_3("v_bfi_b32", "v1", "v2", ""));                // 0 | 1 | 2
    if (K == 23) LOOP(C8_2("v_lshrrev_b32", "v1"));                      // VOP2 1 | 0
    if (K == 24) LOOP(C8_3("v_xad_u32", "v1", "v2", ""));                // 0 | 1 | 2
#undef LOOP
}
constexpr int kKinds = 25;

template <int K>
__global__ __launch_bounds__(64) void kern(unsigned long long* stamps, unsigned a, unsigned b, int iters) {
    extern __shared__ unsigned pad[];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    body<K>(a, b, iters);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t1 - t0 + (pad[0] & 0u);
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static const char* kName[] = {"or3 0|1|2", "or3 0|0|0", "bitop3 0|1|2", "bitop3 0|0|0", "bitop3 0|1|1",
                              "bitop3 0|0|1", "bitop3 0|1|1 (one reg)", "bitop3 0|1|3", "and_or 0|1|2",
                              "add3 0|1|2", "and vop2 1|0", "and vop2 0|0", "and vop2 const|0", "and e64 1|0",
                              "bitop3 chains 0-3|1|2", "bitop3:fe (or3) 0|1|2",
                              "cndmask e64 0|1|sgpr", "cndmask e32 1|0|vcc", "pk_add_u16 1|0", "lshl_or 0|1|2",
                              "perm 0|1|2", "mad_u32_u24 0|1|2", "bfi 0|1|2", "lshrrev vop2 1|0", "xad 0|1|2"};

template <int K>
int run(int cus, int w, unsigned long long* d, int lds) {
    const int blocks = cus * 4 * w, iters = 4000;
    hipEvent_t ea, eb;
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    kern<K><<<blocks, 64, lds>>>(d, 1u, 2u, 100);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(ea));
    kern<K><<<blocks, 64, lds>>>(d, 1u, 2u, iters);
    CK(hipEventRecord(eb));
    CK(hipEventSynchronize(eb));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, ea, eb));
    std::vector<unsigned long long> h(2 * blocks);
    CK(hipMemcpy(h.data(), d, blocks * 16, hipMemcpyDeviceToHost));
    double mean = 0, cyc = 0, rt = 0;
    for (int i = 0; i < blocks; ++i) {
        cyc += (double)h[2 * i];
        rt += (double)h[2 * i + 1];
    }
    mean = cyc / blocks;
    const double ghz = cyc / rt / 10.0;          // s_memrealtime: 100 MHz
    const double per_wave = 32.0 * iters;
    // per wave: w waves share the SIMD for the wave's whole elapsed time;  whole kernel: all
    // wave-instructions over the SIMDs' quad-cycles of the event-timed launch at the waves' clock
    const double rate_wave = w * per_wave / (mean / 4.0);
    const double rate_wall = blocks * per_wave / (ms * 1e-3 * ghz * 1e9 * cus * 4 / 4.0);
    std::printf("%-24s waves/SIMD %d: %.3f VALU/SIMD quad-cycle (per wave), %.3f (wall %.3f ms at %.3f GHz)\n",
                kName[K], w, rate_wave, rate_wall, ms, ghz);
    CK(hipEventDestroy(ea));
    CK(hipEventDestroy(eb));
    return 0;
}

template <int K>
int run_all(int cus, int w, unsigned long long* d, int lds) {
    if (run<K>(cus, w, d, lds)) return 1;
    if constexpr (K + 1 < kKinds) return run_all<K + 1>(cus, w, d, lds);
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    unsigned long long* d;
    CK(hipMalloc(&d, (size_t)cus * 4 * 8 * 16));
    for (int w : {1, 2, 4, 8}) {
        const int lds = 160 * 1024 / (4 * w) - 256;   // at most 4 w workgroups (waves) per CU
        if (run_all<0>(cus, w, d, lds)) return 1;
    }
    CK(hipFree(d));
    return 0;
}
