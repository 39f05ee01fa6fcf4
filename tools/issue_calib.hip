// issue_calib.hip -- dev tool: VALU issue ceilings of solve4_kernel's own instruction mix on
// this GPU.  Every kernel is one 64-lane wave per workgroup, with LDS
// padding so that exactly W waves share each SIMD (W = 7: solve4_kernel's occupancy; 8: the
// CU's limit).  Each is run under rocprofv3 --pmc (SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU2,
// SQ_CYCLES, GRBM_GUI_ACTIVE, ...) so that VALU per SIMD quad-cycle comes from the counters,
// not from an instruction count by hand.
//
//   int2    8 independent chains of 2-operand 32-bit ops with inline constants (xor/add/and/or)
//   b3      the or3 chains as v_bitop3_b32 only (round 6)
//   or3     8 independent chains of 3-VGPR-source ops (v_or3_b32, v_bitop3_b32, v_and_or_b32):
//           the unit summary's and the cell update's shape
//   pk      8 independent chains of packed 16-bit ops (v_pk_add_u16, v_pk_ashrrev_i16,
//           v_pk_sub_u16, v_pk_min_u16)
//   mix     unit4x + three upd4x of solve4_kernel.h (the exact-wave round's VALU, the same asm
//           blocks and dependency chains) on registers only: no LDS between them
//   mix2    two independent copies of `mix` interleaved in one wave (twice the ILP)
//   round   round4<true> of solve4_kernel.h (LDS stores, the nine unit reads, the summary, the
//           unit store, the seven unit reads, three cell updates) plus the loop's four ballots:
//           the round alone, no search step, no dequeue -- the ceiling of a round-bound kernel
//   roundf  the same with round4<false> (the non-exact round: taken-twice and empty-cell tests)
//
// Output: one line per kernel and occupancy: ms per launch, wave-iterations/s, and (for the
// register kernels) VALU wave-instructions/s from the known count per iteration.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/issue_calib tools/issue_calib.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define SDK_NO_SOLVE_KERNEL
#include "../distributed_sudoku_solver_amd/csrc/solve4_kernel.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int kLdsPerCu = 163840;

__global__ __launch_bounds__(64) void k_int2(unsigned* out, unsigned seed, int iters) {
    extern __shared__ unsigned pad[];
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < iters; ++i) {
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
    if (r == 0x12345678u) out[blockIdx.x] = r + pad[0];
}

__global__ __launch_bounds__(64) void k_or3(unsigned* out, unsigned seed, int iters) {
    extern __shared__ unsigned pad[];
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned k0 = seed * 3u + threadIdx.x, k1 = seed ^ 0x5a5a5a5au;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_or3_b32 %0, %0, %8, %9\n v_or3_b32 %1, %1, %8, %9\n v_or3_b32 %2, %2, %8, %9\n v_or3_b32 %3, %3, %8, %9\n"
            "v_or3_b32 %4, %4, %8, %9\n v_or3_b32 %5, %5, %8, %9\n v_or3_b32 %6, %6, %8, %9\n v_or3_b32 %7, %7, %8, %9\n"
            "v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %0, %0, %8, %9 bitop3:0xe8\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0xe8\n"
            "v_bitop3_b32 %2, %2, %8, %9 bitop3:0xe8\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0xe8\n"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0xe8\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0xe8\n"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0xe8\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0xe8\n"
            "v_and_or_b32 %0, %0, %8, %9\n v_and_or_b32 %1, %1, %8, %9\n v_and_or_b32 %2, %2, %8, %9\n"
            "v_and_or_b32 %3, %3, %8, %9\n v_and_or_b32 %4, %4, %8, %9\n v_and_or_b32 %5, %5, %8, %9\n"
            "v_and_or_b32 %6, %6, %8, %9\n v_and_or_b32 %7, %7, %8, %9\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(k0), "v"(k1));
    }
    const unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) out[blockIdx.x] = r + pad[0];
}

// the same chains as k_or3 with every op a v_bitop3_b32 (OR3 0xFE, XOR3 0x96, majority 0xE8,
// and-or 0xEA): the form prop32's step and solve4's unit summary take since round 6
// (solve_kernel.h SDK_OR3); operands where the compiler puts them, as in the kernels
__global__ __launch_bounds__(64) void k_b3(unsigned* out, unsigned seed, int iters) {
    extern __shared__ unsigned pad[];
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned k0 = seed * 3u + threadIdx.x, k1 = seed ^ 0x5a5a5a5au;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_bitop3_b32 %0, %0, %8, %9 bitop3:0xfe\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0xfe\n"
            "v_bitop3_b32 %2, %2, %8, %9 bitop3:0xfe\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0xfe\n"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0xfe\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0xfe\n"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0xfe\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0xfe\n"
            "v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0x96\n"
            "v_bitop3_b32 %0, %0, %8, %9 bitop3:0xe8\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0xe8\n"
            "v_bitop3_b32 %2, %2, %8, %9 bitop3:0xe8\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0xe8\n"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0xe8\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0xe8\n"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0xe8\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0xe8\n"
            "v_bitop3_b32 %0, %0, %8, %9 bitop3:0xea\n v_bitop3_b32 %1, %1, %8, %9 bitop3:0xea\n"
            "v_bitop3_b32 %2, %2, %8, %9 bitop3:0xea\n v_bitop3_b32 %3, %3, %8, %9 bitop3:0xea\n"
            "v_bitop3_b32 %4, %4, %8, %9 bitop3:0xea\n v_bitop3_b32 %5, %5, %8, %9 bitop3:0xea\n"
            "v_bitop3_b32 %6, %6, %8, %9 bitop3:0xea\n v_bitop3_b32 %7, %7, %8, %9 bitop3:0xea\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(k0), "v"(k1));
    }
    const unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) out[blockIdx.x] = r + pad[0];
}

__global__ __launch_bounds__(64) void k_pk(unsigned* out, unsigned seed, int iters) {
    extern __shared__ unsigned pad[];
    unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    unsigned k0 = seed * 3u + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "v_pk_add_u16 %0, %0, -1\n v_pk_add_u16 %1, %1, -1\n v_pk_add_u16 %2, %2, -1\n v_pk_add_u16 %3, %3, -1\n"
            "v_pk_add_u16 %4, %4, -1\n v_pk_add_u16 %5, %5, -1\n v_pk_add_u16 %6, %6, -1\n v_pk_add_u16 %7, %7, -1\n"
            "v_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]\n v_pk_ashrrev_i16 %1, 15, %1 op_sel_hi:[0,1]\n"
            "v_pk_ashrrev_i16 %2, 15, %2 op_sel_hi:[0,1]\n v_pk_ashrrev_i16 %3, 15, %3 op_sel_hi:[0,1]\n"
            "v_pk_ashrrev_i16 %4, 15, %4 op_sel_hi:[0,1]\n v_pk_ashrrev_i16 %5, 15, %5 op_sel_hi:[0,1]\n"
            "v_pk_ashrrev_i16 %6, 15, %6 op_sel_hi:[0,1]\n v_pk_ashrrev_i16 %7, 15, %7 op_sel_hi:[0,1]\n"
            "v_pk_sub_u16 %0, 0, %0\n v_pk_sub_u16 %1, 0, %1\n v_pk_sub_u16 %2, 0, %2\n v_pk_sub_u16 %3, 0, %3\n"
            "v_pk_sub_u16 %4, 0, %4\n v_pk_sub_u16 %5, 0, %5\n v_pk_sub_u16 %6, 0, %6\n v_pk_sub_u16 %7, 0, %7\n"
            "v_pk_min_u16 %0, %0, %8\n v_pk_min_u16 %1, %1, %8\n v_pk_min_u16 %2, %2, %8\n v_pk_min_u16 %3, %3, %8\n"
            "v_pk_min_u16 %4, %4, %8\n v_pk_min_u16 %5, %5, %8\n v_pk_min_u16 %6, %6, %8\n v_pk_min_u16 %7, %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(k0));
    }
    const unsigned r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) out[blockIdx.x] = r + pad[0];
}

// one exact-wave round's VALU on registers: unit4x over nine (X, S) words, three upd4x whose
// unit words are T | a neighbour's T, the results fed back as the next iteration's cells
struct MixState {
    uint2 v[9];
    uint32_t E, x0, x1, x2, s0, s1, s2;
};
__device__ __forceinline__ void mix_iter(MixState& m, uint32_t& sink) {
    uint32_t once, T, bm, chg = 0, m0, m1, m2;
    sdk::unit4x(m.v, m.E, once, T, bm);
    sdk::upd4x(m.x0, m.s0, T | m.v[3].y, once, bm, m0, chg);
    sdk::upd4x(m.x1, m.s1, T | m.v[4].y, once, bm, m1, chg);
    sdk::upd4x(m.x2, m.s2, T | m.v[5].y, once, bm, m2, chg);
    sink ^= bm ^ chg;
    // rotate: this lane's cells become three of the next iteration's unit words (renaming only)
    m.v[8] = m.v[5];
    m.v[7] = m.v[4];
    m.v[6] = m.v[3];
    m.v[5] = m.v[2];
    m.v[4] = m.v[1];
    m.v[3] = m.v[0];
    m.v[0] = make_uint2(m.x0 | (chg & 0x00010001u), m.s0);
    m.v[1] = make_uint2(m.x1, m.s1);
    m.v[2] = make_uint2(m.x2, m.s2);
    m.x0 |= once;   // keep candidates from draining to 0 (the same work either way)
    m.x1 |= T & 0x00FF00FFu;
    m.x2 |= bm;
}
__device__ __forceinline__ void mix_init(MixState& m, unsigned seed, int k) {
    const uint32_t b = (threadIdx.x * 2654435761u) ^ (seed + 97u * k);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const uint32_t h = b * (2 * i + 1) + 0x9e3779b9u * i;
        m.v[i] = make_uint2(h & 0x01FF01FFu, (h >> 7) & 0x01000100u);
    }
    m.E = 0x01FF01FFu;
    m.x0 = b & 0x01FF01FFu;
    m.x1 = (b >> 3) & 0x01FF01FFu;
    m.x2 = (b >> 5) & 0x01FF01FFu;
    m.s0 = m.s1 = m.s2 = 0;
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(7))) void k_mix(unsigned* out, unsigned seed,
                                                                                    int iters) {
    extern __shared__ unsigned pad[];
    MixState m;
    mix_init(m, seed, 0);
    uint32_t sink = 0;
    for (int i = 0; i < iters; ++i) mix_iter(m, sink);
    if (sink == 0x12345678u) out[blockIdx.x] = sink + pad[0];
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(7))) void k_mix2(unsigned* out, unsigned seed,
                                                                                     int iters) {
    extern __shared__ unsigned pad[];
    MixState m, n;
    mix_init(m, seed, 0);
    mix_init(n, seed, 1);
    uint32_t sink = 0;
    for (int i = 0; i < iters; ++i) {
        mix_iter(m, sink);
        mix_iter(n, sink);
    }
    if (sink == 0x12345678u) out[blockIdx.x] = sink + pad[0];
}

// the real round (LDS included) on four copies of one board, no search step
template <bool EXACT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(7))) void k_round(unsigned* out, const uint8_t* board,
                                                                                      int iters) {
    using namespace sdk;
    extern __shared__ unsigned pad[];
    __shared__ uint2 s_region[2 * kRegion4];
    __shared__ uint8_t s_in[2 * 2 * 81];
    Lane4 w;
    init_lane4(w, s_region, s_in);
    Cells4 c;
    const uint32_t i0 = w.act ? board[w.c0] : 0u, i1 = w.act ? board[w.c0 + 27] : 0u,
                   i2 = w.act ? board[w.c0 + 54] : 0u;
    const uint32_t x0 = w.act ? cell_x4(i0) : 0u, x1 = w.act ? cell_x4(i1) : 0u, x2 = w.act ? cell_x4(i2) : 0u;
    const uint32_t s0 = w.act ? cell_s4(i0) : kInert4, s1 = w.act ? cell_s4(i1) : kInert4,
                   s2 = w.act ? cell_s4(i2) : kInert4;
    c.x0 = x0 | (x0 << 16);
    c.x1 = x1 | (x1 << 16);
    c.x2 = x2 | (x2 << 16);
    c.s0 = s0 | (s0 << 16);
    c.s1 = s1 | (s1 << 16);
    c.s2 = s2 | (s2 << 16);
    c.D = kC2;
    c.E = w.act ? kC2 : 0u;
    uint64_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        uint32_t badw, chg;
        round4<EXACT>(w, c, badw, chg);
        const uint64_t B0 = spread_halves(__builtin_amdgcn_ballot_w64((badw & 0xFFFFu) != 0u));
        const uint64_t B1 = spread_halves(__builtin_amdgcn_ballot_w64(badw > 0xFFFFu));
        const uint64_t C0 = spread_halves(__builtin_amdgcn_ballot_w64((chg & 0xFFFFu) != 0u));
        const uint64_t C1 = spread_halves(__builtin_amdgcn_ballot_w64(chg > 0xFFFFu));
        acc += (B0 | ~C0) ^ (B1 | ~C1);
    }
    if (acc == 0x12345678ull) out[blockIdx.x] = (unsigned)acc + pad[0];
}

int main(int argc, char** argv) {
    int dev_cus = 0;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    dev_cus = prop.multiProcessorCount;
    unsigned* d;
    CK(hipMalloc(&d, 1 << 22));
    uint8_t* dboard;
    CK(hipMalloc(&dboard, 81));
    // S1, a 17-clue board of SURVEY §8(d) C4 (its state after a few rounds is a fixpoint; the
    // round's instructions are branch-free, so the work per round does not depend on it)
    const char* s1 = "000000010400000000020000000000050407008000300001090000300400200050100000000806000";
    uint8_t hb[81];
    for (int i = 0; i < 81; ++i) hb[i] = (uint8_t)(s1[i] - '0');
    CK(hipMemcpy(dboard, hb, 81, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int only = argc > 1 ? atoi(argv[1]) : -1;   // run one kernel id only (profiling)
    struct K {
        const char* name;
        int id;
        double valu_per_iter;   // hand count (register kernels), 0 = see the counters
        int iters;
    };
    const K ks[] = {{"int2", 0, 32, 4096}, {"or3", 1, 32, 4096}, {"pk", 2, 32, 4096},
                    {"mix", 3, 0, 4096},   {"mix2", 4, 0, 2048}, {"round", 5, 0, 2048},
                    {"roundf", 6, 0, 2048}, {"b3", 7, 32, 4096}};
    for (int wps : {7, 8}) {
        const int per_cu = 4 * wps;
        const int blocks = dev_cus * per_cu;
        // LDS per workgroup so that at most per_cu workgroups fit a CU (static LDS of k_round
        // is under 4.5 KiB, well inside this)
        const size_t lds = (size_t)(kLdsPerCu / per_cu) - 64;
        for (const K& k : ks) {
            if (only >= 0 && k.id != only) continue;
            auto launch = [&](unsigned seed) {
                switch (k.id) {
                case 0: k_int2<<<blocks, 64, lds>>>(d, seed, k.iters); break;
                case 1: k_or3<<<blocks, 64, lds>>>(d, seed, k.iters); break;
                case 2: k_pk<<<blocks, 64, lds>>>(d, seed, k.iters); break;
                case 3: k_mix<<<blocks, 64, lds>>>(d, seed, k.iters); break;
                case 4: k_mix2<<<blocks, 64, lds>>>(d, seed, k.iters); break;
                case 5: k_round<true><<<blocks, 64, lds - 4200>>>(d, dboard, k.iters); break;
                case 6: k_round<false><<<blocks, 64, lds - 4200>>>(d, dboard, k.iters); break;
                case 7: k_b3<<<blocks, 64, lds>>>(d, seed, k.iters); break;
                }
            };
            launch(7);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            float ms = 0;
            CK(hipEventRecord(e0));
            for (int r = 0; r < 5; ++r) launch(7 + r);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 5;
            const double wave_iters = (double)blocks * k.iters;
            printf("%-7s waves/SIMD %d: %.3f ms/launch  %.4e wave-iterations/s", k.name, wps, ms,
                   wave_iters / (ms * 1e-3));
            if (k.valu_per_iter > 0)
                printf("  %.4e VALU wave-instr/s = %.3f per SIMD quad-cycle at 2.4 GHz",
                       wave_iters * k.valu_per_iter / (ms * 1e-3),
                       wave_iters * k.valu_per_iter / (ms * 1e-3) / (dev_cus * 4 * 2.4e9 / 4));
            printf("\n");
            fflush(stdout);
        }
    }
    CK(hipFree(d));
    CK(hipFree(dboard));
    return 0;
}
