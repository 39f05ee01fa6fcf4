// check_kernel.h -- batched Sudoku.check() (sudoku.py:43-94) as an HBM-streaming kernel.
//
// Layout: boards uint8[n][81] contiguous in HBM, verdict uint8[n].
// Algorithmic traffic: 81 B read + 1 B written per board.
//
// One 256-thread workgroup owns a tile of 256 boards = 20,736 B = 1,296 x 16 B.
// The tile is streamed HBM -> LDS with coalesced dwordx4 loads (every lane reads
// 16 B, a wave reads 1 KiB contiguous), then each thread validates one board from
// LDS: 22 ds_read_b32 + v_alignbyte re-align the 81-B record (81i mod 4 = i mod 4)
// into 21 dwords, so no unaligned global access and no byte-granular HBM reads.
//
// Per unit the reference rule is literal: `sum == 45 and len(set) == 9`.
//  * fast path (every byte of the board <= 9): acc_u = sum 2^v over the unit.
//    For 9 values in 0..9:  literal rule <=> multiset {1..9} <=> acc_u == 0x3FE
//    (merging equal powers of two reduces the term count, and 0x3FE has 9 bits).
//  * exact path (some byte >= 10, any uint8):  x = (v << 22) + 2^min(v,18);
//    pass <=> popc(acc & 0x3FFFFF) == 9 and (acc >> 22) == 45.  9 distinct
//    non-negative values summing to 45 are all <= 17, so clamping at 18 never
//    merges two passing values; with popc == 9 at most one value is >= 18, the
//    sum is then <= 363 and the 10-bit field cannot wrap.
// The raw-NameError bit needs the exact box(0,0) sum (sudoku.py:68 evaluates
// the sum before the broken set expression), accumulated separately.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Round 6 (checker): the fast path is entered on one OR over the record (every byte < 32)
// and left for the exact path on the OR of the one-hot terms (a byte in 10..31), and the verdicts
// are non-temporal stores: 1.364 ms per 100M boards against 1.392 on one box (0 to fall back)
#ifndef SDK_CHECK_FAST_OR
#define SDK_CHECK_FAST_OR 1
#endif
#ifndef SDK_CHECK_NT_STORE
#define SDK_CHECK_NT_STORE 1
#endif

namespace sdk {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kCheckThreads = 256;
constexpr int kCheckTileBytes = kCheckThreads * 81;          // 20736
constexpr int kCheckTileVec = kCheckTileBytes / 16;          // 1296 x uint4

__device__ __forceinline__ uint32_t byte_of(const uint32_t (&w)[21], int k) {
    return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
}

// the verdict byte; with SDK_CHECK_NT_STORE a non-temporal store (the stream's only writes)
__device__ __forceinline__ void put_verdict(uint8_t* p, uint8_t v) {
    if (SDK_CHECK_NT_STORE)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

__device__ __forceinline__ uint8_t check_board_lds(const uint32_t* tile_dw, int t) {
    const int start = 81 * t;
    const int d0 = start >> 2;
    const uint32_t sh = (uint32_t)(start & 3);
    uint32_t raw[22];
#pragma unroll
    for (int k = 0; k < 22; ++k) raw[k] = tile_dw[d0 + k];
    uint32_t w[21];
#pragma unroll
    for (int k = 0; k < 21; ++k) w[k] = __builtin_amdgcn_alignbyte(raw[k + 1], raw[k], sh);
    w[20] &= 0xFFu;  // only cell 80 belongs to this board

#if SDK_CHECK_FAST_OR
    // Fast path when every byte is < 32 (one OR over the record, no per-byte test): 1 << v is then
    // exact, and a byte in 10..31 shows as a bit >= 10 in the OR of the one-hot terms (an OR: no
    // carries), so such a board leaves for the exact path below after the sums.
    uint32_t orall = 0;
#pragma unroll
    for (int k = 0; k < 21; ++k) orall |= w[k];
    const bool small = (orall & 0xE0E0E0E0u) == 0u;
#else
    // any byte >= 10 ?  ((b & 0x7F) + 0x76) sets bit 7 iff (b & 0x7F) >= 10, no carry out of the byte
    uint32_t big = 0;
#pragma unroll
    for (int k = 0; k < 21; ++k) big |= (((w[k] & 0x7F7F7F7Fu) + 0x76767676u) | w[k]) & 0x80808080u;
    const bool small = big == 0;
#endif

    uint32_t rowacc[9], colacc[9], boxacc[9];
#pragma unroll
    for (int u = 0; u < 9; ++u) rowacc[u] = colacc[u] = boxacc[u] = 0;
    uint32_t box00 = 0;
    [[maybe_unused]] uint32_t allor = 0;
    uint8_t verdict = 0;
    bool exact = !small;
    if (small) {
#pragma unroll
        for (int k = 0; k < 81; ++k) {
            const int r = k / 9, c = k % 9, b = (r / 3) * 3 + c / 3;
            const uint32_t v = byte_of(w, k);
            const uint32_t p = 1u << v;
            rowacc[r] += p; colacc[c] += p; boxacc[b] += p;
            if (SDK_CHECK_FAST_OR) allor |= p;
            if (b == 0) box00 += v;
        }
#if SDK_CHECK_FAST_OR
        uint32_t bad = 0;
#pragma unroll
        for (int u = 0; u < 9; ++u) bad |= (rowacc[u] ^ 0x3FEu) | ((colacc[u] ^ 0x3FEu) << 16);
        uint32_t badb = 0;
#pragma unroll
        for (int u = 0; u < 9; ++u) badb |= boxacc[u] ^ 0x3FEu;
        exact = (allor & ~0x3FFu) != 0u;      // a byte in 10..31: the exact path
        const bool rows = (bad & 0xFFFFu) == 0u, cols = (bad >> 16) == 0u, boxes = badb == 0u;
#else
        bool rows = true, cols = true, boxes = true;
#pragma unroll
        for (int u = 0; u < 9; ++u) {
            rows &= rowacc[u] == 0x3FEu;
            cols &= colacc[u] == 0x3FEu;
            boxes &= boxacc[u] == 0x3FEu;
        }
#endif
        verdict = (uint8_t)((rows && cols && boxes) ? 1u : 0u);
        if (rows && cols && box00 == 45u) verdict |= 2u;
    }
    if (exact) {
        box00 = 0;
#pragma unroll
        for (int u = 0; u < 9; ++u) rowacc[u] = colacc[u] = boxacc[u] = 0;
#pragma unroll
        for (int k = 0; k < 81; ++k) {
            const int r = k / 9, c = k % 9, b = (r / 3) * 3 + c / 3;
            const uint32_t v = byte_of(w, k);
            const uint32_t x = (v << 22) + (1u << min(v, 18u));
            rowacc[r] += x; colacc[c] += x; boxacc[b] += x;
            if (b == 0) box00 += v;
        }
        auto ok = [](uint32_t a) { return __popc(a & 0x3FFFFFu) == 9 && (a >> 22) == 45u; };
        bool rows = true, cols = true, boxes = true;
#pragma unroll
        for (int u = 0; u < 9; ++u) {
            rows &= ok(rowacc[u]);
            cols &= ok(colacc[u]);
            boxes &= ok(boxacc[u]);
        }
        verdict = (uint8_t)((rows && cols && boxes) ? 1u : 0u);
        if (rows && cols && box00 == 45u) verdict |= 2u;
    }
    return verdict;
}

// Full tiles are software-pipelined: the 6 dwordx4 loads of tile i+1 are issued
// into registers before tile i is validated out of LDS, so every thread keeps
// 96 B of HBM reads in flight across its compute phase.
__global__ __launch_bounds__(kCheckThreads) void check_kernel(const uint8_t* __restrict__ boards,
                                                              uint8_t* __restrict__ verdict, uint64_t n) {
    // +16 B: the last thread's 22nd dword read runs one dword past the tile.
    __shared__ __attribute__((aligned(16))) u32x4 tile[kCheckTileVec + 1];
    constexpr int kFull = kCheckTileVec / kCheckThreads;   // 5 vectors per thread
    constexpr int kRem = kCheckTileVec % kCheckThreads;    // + 16 threads load a 6th
    const int t = threadIdx.x;
    const uint64_t nfull = n / kCheckThreads;              // full tiles
    const uint64_t ntiles = (n + kCheckThreads - 1) / kCheckThreads;
    u32x4 pre[kFull + 1];
    uint64_t tix = blockIdx.x;
    auto load_tile = [&](uint64_t ti) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(boards + ti * kCheckTileBytes);
#pragma unroll
        for (int j = 0; j < kFull; ++j) pre[j] = __builtin_nontemporal_load(&s4[j * kCheckThreads + t]);
        if (t < kRem) pre[kFull] = __builtin_nontemporal_load(&s4[kFull * kCheckThreads + t]);
    };
    if (tix < nfull) load_tile(tix);
    for (; tix < ntiles; tix += gridDim.x) {
        const uint64_t base = tix * kCheckThreads;
        const uint64_t cnt = min((uint64_t)kCheckThreads, n - base);
        if (cnt == (uint64_t)kCheckThreads) {
#pragma unroll
            for (int j = 0; j < kFull; ++j) tile[j * kCheckThreads + t] = pre[j];
            if (t < kRem) tile[kFull * kCheckThreads + t] = pre[kFull];
        } else {
            // ragged last tile: each thread copies its own record byte by byte
            const uint8_t* src = boards + base * 81;
            uint8_t* tb = reinterpret_cast<uint8_t*>(tile);
            if ((uint64_t)t < cnt) {
#pragma unroll
                for (int k = 0; k < 81; ++k) tb[81 * t + k] = src[81 * t + k];
            }
        }
        __syncthreads();
        const uint64_t nxt = tix + gridDim.x;
        if (nxt < nfull) load_tile(nxt);                   // in flight during validation
        if ((uint64_t)t < cnt)
            put_verdict(verdict + base + t, check_board_lds(reinterpret_cast<const uint32_t*>(tile), t));
        __syncthreads();
    }
}

// Variant: two tiles in flight per workgroup (register ring of depth 2, the loop
// unrolled by two so the ring index stays compile-time and the ring in VGPRs).
__global__ __launch_bounds__(kCheckThreads) void check_kernel_rr2(const uint8_t* __restrict__ boards,
                                                                  uint8_t* __restrict__ verdict, uint64_t n) {
    __shared__ __attribute__((aligned(16))) u32x4 tile[kCheckTileVec + 1];
    constexpr int kFull = kCheckTileVec / kCheckThreads;
    constexpr int kRem = kCheckTileVec % kCheckThreads;
    const int t = threadIdx.x;
    const uint64_t nfull = n / kCheckThreads;
    const uint64_t ntiles = (n + kCheckThreads - 1) / kCheckThreads;
    const uint64_t G = gridDim.x;
    u32x4 ra[kFull + 1], rb[kFull + 1];
    // Loads are issued unconditionally (past-the-end tiles clamp to the last full
    // tile, lanes >= kRem re-read lane t % kRem's vector): with no branch around
    // them the compiler's vmcnt waits stay counted and the other ring slot stays in
    // flight. Requires nfull >= 1 (the launcher uses check_kernel for tiny n).
    auto load_tile = [&](uint64_t ti, u32x4 (&pre)[kFull + 1]) {
        ti = min(ti, nfull - 1);
        const u32x4* s4 = reinterpret_cast<const u32x4*>(boards + ti * kCheckTileBytes);
#pragma unroll
        for (int j = 0; j < kFull; ++j) pre[j] = __builtin_nontemporal_load(&s4[j * kCheckThreads + t]);
        pre[kFull] = __builtin_nontemporal_load(&s4[kFull * kCheckThreads + (t & (kRem - 1))]);
    };
    // cur holds tile tix (if full), nxt holds tile tix + G in flight
    auto step = [&](uint64_t tix, u32x4 (&cur)[kFull + 1]) {
        const uint64_t base = tix * kCheckThreads;
        const uint64_t cnt = min((uint64_t)kCheckThreads, n - base);
        if (cnt == (uint64_t)kCheckThreads) {
#pragma unroll
            for (int j = 0; j < kFull; ++j) tile[j * kCheckThreads + t] = cur[j];
            if (t < kRem) tile[kFull * kCheckThreads + t] = cur[kFull];
        } else {
            const uint8_t* src = boards + base * 81;
            uint8_t* tb = reinterpret_cast<uint8_t*>(tile);
            if ((uint64_t)t < cnt) {
#pragma unroll
                for (int k = 0; k < 81; ++k) tb[81 * t + k] = src[81 * t + k];
            }
        }
        __syncthreads();
        load_tile(tix + 2 * G, cur);
        if ((uint64_t)t < cnt)
            put_verdict(verdict + base + t, check_board_lds(reinterpret_cast<const uint32_t*>(tile), t));
        __syncthreads();
    };
    uint64_t tix = blockIdx.x;
    load_tile(tix, ra);
    load_tile(tix + G, rb);
    // The scheduler interleaves the two prologue tiles; left pending, that order
    // would make the loop's merged waits drain both slots. Drain once here instead.
    __builtin_amdgcn_s_waitcnt(0);
    for (; tix < ntiles; tix += 2 * G) {
        step(tix, ra);
        if (tix + G >= ntiles) break;
        step(tix + G, rb);
    }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Variant: LDS-DMA ring. NBUF tile buffers in ONE __shared__ array; tiles are
// fetched HBM -> LDS with global_load_lds_dwordx4 (no VGPR staging, lane-linear
// 1 KiB per wave-instruction), NBUF-1 tiles ahead. Counted vmcnt + raw s_barrier
// keep the later tiles in flight across the barriers (a __syncthreads() would
// drain them). Global stores share the VM counter but are never counted in the
// wait: waiting for <= D*G loads outstanding retires every load of the current
// tile whatever the stores do, because loads retire in order.
template <int NBUF>
__global__ __launch_bounds__(kCheckThreads) void check_kernel_glds(const uint8_t* __restrict__ boards,
                                                                   uint8_t* __restrict__ verdict, uint64_t n) {
    __shared__ __attribute__((aligned(16))) u32x4 ring[NBUF * kCheckTileVec + 1];
    constexpr int D = NBUF - 1;
    constexpr int kFull = kCheckTileVec / kCheckThreads;   // 5 glds per wave per tile
    constexpr int kRem = kCheckTileVec % kCheckThreads;    // wave 0: a 6th for 16 lanes
    const int t = threadIdx.x;
    const int wave = t >> 6;
    const uint64_t nfull = n / kCheckThreads;
    const uint64_t ntiles = (n + kCheckThreads - 1) / kCheckThreads;
    const uint64_t G = gridDim.x;
    auto issue = [&](uint64_t ti, int buf) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(boards + ti * kCheckTileBytes);
        u32x4* d = ring + buf * kCheckTileVec;
#pragma unroll
        for (int j = 0; j < kFull; ++j)
            __builtin_amdgcn_global_load_lds((const void*)&s4[j * kCheckThreads + t],
                                             (__attribute__((address_space(3))) void*)(d + j * kCheckThreads + wave * 64),
                                             16, 0, 2);
        if (t < kRem)
            __builtin_amdgcn_global_load_lds((const void*)&s4[kFull * kCheckThreads + t],
                                             (__attribute__((address_space(3))) void*)(d + kFull * kCheckThreads),
                                             16, 0, 2);
    };
    uint64_t tix = blockIdx.x;
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (tix + d * G < nfull) issue(tix + d * G, d);
    int buf = 0;
    for (; tix < ntiles; tix += G) {
        const uint64_t ahead = tix + D * G;
        const uint64_t base = tix * kCheckThreads;
        const uint64_t cnt = min((uint64_t)kCheckThreads, n - base);
        u32x4* cur = ring + buf * kCheckTileVec;
        if (ahead < nfull) {
            int nb = buf + D;
            if (nb >= NBUF) nb -= NBUF;
            issue(ahead, nb);
            if (wave == 0) wait_vmcnt<D*(kFull + 1)>();
            else wait_vmcnt<D * kFull>();
        } else {
            wait_vmcnt<0>();
            if (cnt != (uint64_t)kCheckThreads) {
                const uint8_t* src = boards + base * 81;
                uint8_t* tb = reinterpret_cast<uint8_t*>(cur);
                if ((uint64_t)t < cnt) {
#pragma unroll
                    for (int k = 0; k < 81; ++k) tb[81 * t + k] = src[81 * t + k];
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's ds_writes (ragged path) landed
        __builtin_amdgcn_s_barrier();
        if ((uint64_t)t < cnt)
            put_verdict(verdict + base + t, check_board_lds(reinterpret_cast<const uint32_t*>(cur), t));
        __builtin_amdgcn_s_waitcnt(0xc07f);   // this wave's ds_reads of cur are done
        __builtin_amdgcn_s_barrier();         // nobody reads cur when the next iteration refills it
        buf = (buf + 1 == NBUF) ? 0 : buf + 1;
    }
    wait_vmcnt<0>();
}

// Variant: per-WAVE tiles, no workgroup barrier (round 6).  Each wave streams its own 64-board
// tiles (5,184 B = 324 x 16 B: 5 dwordx4 per lane, a 6th for lanes 0..3) through its own LDS
// region; a wave's LDS accesses execute in issue order, so the stores of a tile and the lanes'
// re-aligning reads need no barrier, and no wave waits for another's loads (the workgroup barrier
// of check_kernel makes each tile's next loads wait for the slowest wave of four).  NBUF register
// sets keep NBUF tiles of the wave in flight: the loads of tile i + NBUF are issued as soon as tile
// i is in LDS, before its boards are checked.  Tiles are dealt grid-stride by global wave index.
constexpr int kCheckWaveTileVec = 64 * 81 / 16;          // 324 x uint4 per wave tile
template <int NBUF>
__global__ __launch_bounds__(kCheckThreads) void check_kernel_wave(const uint8_t* __restrict__ boards,
                                                                   uint8_t* __restrict__ verdict, uint64_t n) {
    // +16 B per wave region: the last lane's 22nd dword read runs one dword past its tile
    __shared__ __attribute__((aligned(16))) u32x4 tiles[(kCheckThreads / 64) * (kCheckWaveTileVec + 1)];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    u32x4* my = tiles + wv * (kCheckWaveTileVec + 1);
    const uint64_t nw = (uint64_t)gridDim.x * (kCheckThreads / 64);
    const uint64_t nfull = n / 64;                              // full wave tiles
    const uint64_t ntiles = (n + 63) / 64;
    uint64_t tix = (uint64_t)blockIdx.x * (kCheckThreads / 64) + wv;
    u32x4 ring[NBUF][6];
    auto load = [&](uint64_t ti, u32x4 (&r)[6]) {
        const u32x4* s4 = reinterpret_cast<const u32x4*>(boards + ti * (64 * 81));
#pragma unroll
        for (int j = 0; j < 5; ++j) r[j] = __builtin_nontemporal_load(&s4[j * 64 + lane]);
        if (lane < 4) r[5] = __builtin_nontemporal_load(&s4[5 * 64 + lane]);
    };
#pragma unroll
    for (int b = 0; b < NBUF; ++b)
        if (tix + b * nw < nfull) load(tix + b * nw, ring[b]);
    for (int b = 0; tix < ntiles; tix += nw) {
        const uint64_t base = tix * 64;
        if (tix < nfull) {
#pragma unroll
            for (int k = 0; k < NBUF; ++k) {          // the ring slot as a compile-time index
                if (k == b) {
#pragma unroll
                    for (int j = 0; j < 5; ++j) my[j * 64 + lane] = ring[k][j];
                    if (lane < 4) my[5 * 64 + lane] = ring[k][5];
                    __builtin_amdgcn_wave_barrier();
                    const uint64_t nxt = tix + NBUF * nw;
                    if (nxt < nfull) load(nxt, ring[k]);   // in flight while this tile is checked
                }
            }
        } else {
            // ragged last tile: each lane copies its own record byte by byte
            const uint64_t cnt = n - base;
            uint8_t* tb = reinterpret_cast<uint8_t*>(my);
            if ((uint64_t)lane < cnt) {
                const uint8_t* src = boards + (base + lane) * 81;
#pragma unroll
                for (int k = 0; k < 81; ++k) tb[81 * lane + k] = src[k];
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (base + lane < n) put_verdict(verdict + base + lane, check_board_lds(reinterpret_cast<const uint32_t*>(my), lane));
        __builtin_amdgcn_wave_barrier();              // every lane's reads before the next stores
        b = (b + 1 == NBUF) ? 0 : b + 1;
    }
}

// ---------------------------------------------------------------------------
// check_kernel_i64 -- the same literal rule on int64 cells, for boards whose values
// leave 0..255 (the reference takes any Python int; JSON numbers reach it unchanged).
// One thread per board; not bandwidth-tuned (an off-nominal input path).  Valid for
// |v| < 2^59, where the sum of 9 cells cannot overflow (the host checks the bound).
__device__ __forceinline__ bool unit_ok_i64(const int64_t (&u)[9]) {
    int64_t sum = 0;
    bool distinct = true;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        sum += u[k];
#pragma unroll
        for (int j = 0; j < k; ++j) distinct &= u[j] != u[k];
    }
    return sum == 45 && distinct;
}

__global__ __launch_bounds__(256) void check_kernel_i64(const int64_t* __restrict__ boards, uint8_t* __restrict__ out,
                                                        uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int64_t* b = boards + i * 81;
        int64_t u[9];
        bool rows = true, cols = true, boxes = true;
        for (int r = 0; r < 9 && rows; ++r) {                      // sudoku.py:79-81
#pragma unroll
            for (int c = 0; c < 9; ++c) u[c] = b[9 * r + c];
            rows = unit_ok_i64(u);
        }
        for (int c = 0; c < 9 && rows && cols; ++c) {              // sudoku.py:84-86
#pragma unroll
            for (int r = 0; r < 9; ++r) u[r] = b[9 * r + c];
            cols = unit_ok_i64(u);
        }
        int64_t box00 = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) box00 += b[9 * (k / 3) + (k % 3)];
        for (int bx = 0; bx < 9 && rows && cols && boxes; ++bx) {  // sudoku.py:89-92
            const int r0 = (bx / 3) * 3, c0 = (bx % 3) * 3;
#pragma unroll
            for (int k = 0; k < 9; ++k) u[k] = b[9 * (r0 + k / 3) + c0 + k % 3];
            boxes = unit_ok_i64(u);
        }
        uint8_t v = (rows && cols && boxes) ? 1u : 0u;
        if (rows && cols && box00 == 45) v |= 2u;               // the raw call raises NameError (sudoku.py:68)
        out[i] = v;
    }
}

}  // namespace sdk
