// solve4_kernel.h -- DHTNode.solve_sudoku (DHT_Node.py:474-538) on gfx950, FOUR
// boards per wavefront: two per 32-lane half, packed as the two 16-bit halves of
// every state word (SIMD within a register).
//
// Same search, rules and orders as solve2_kernel.h (and so the same answers and
// the same search nodes per board); the lane layout is solve2's -- lane j < 27 of
// a half owns cells j, j+27, j+54 and unit j -- but every 32-bit word carries the
// same cell (or unit) of two boards: bits 0..15 board "lo", bits 16..31 board
// "hi".  All propagation arithmetic is bitwise or packed 16-bit (v_pk_sub_u16,
// v_pk_min_u16), so one instruction advances two boards and a propagation round
// costs about half the VALU instructions per board of solve2's.
//
// Cell state, per board (16-bit field), exactly one of X and S is non-zero:
//   X  candidate digits 1..9 (bits 0..8) of an OPEN cell, 0 once it is closed
//   S  the digit (one bit of 0..8) of a given or of a solved cell; bit 9 for an
//      out-of-domain given (inert); 0 while the cell is open
// so a cell is open (branchable) <=> X != 0, and an open cell that loses its last
// candidate is X = S = 0 (the contradiction test).
// Givens are not otherwise marked: what solve2 reads from its "given" field is
// static per board and kept per unit lane instead, computed once per board by a
// static pass over the input (start of every board):
//   D  digits given at least twice in the unit (given-vs-given duplicates: the
//      reference never validates clues, SURVEY §0.9, so they are no conflict);
//      Cells4::D holds its complement within the candidate bits, kC2 & ~D
//   E  0x1FF if the unit is exact (no duplicate and no inert given: every digit
//      must occur exactly once in every completion), else 0
// Unit summary (lane j, unit j, both boards): from the 9 cells (X, S) words
//   T     = OR of S                      (taken digits: givens and solved cells)
//   once  = candidates held by exactly one open cell, in exact units (hidden
//           singles; a digit of T is never applied: every update masks T first)
//   conflict: a digit taken twice that is not a duplicated given, or an exact
//             unit that lost a digit (in neither T nor any candidate set).  (A non-given cell can never be solved to
//             a given digit of its units -- every rule only picks digits outside
//             T -- so "taken twice, not in D" is solve2's solved-vs-solved /
//             solved-vs-given test.  The first-cell `range` restriction is the
//             exception: that cell starts OPEN with X = mask even when the mask
//             is one digit, so round 1 eliminates T from it like any other cell.)
// Cell update (open cells; a closed cell's X = 0 stays 0): X &= ~T; hidden single
// X & once; two hidden singles or no candidate = contradiction; one candidate left
// -> S = that digit, X = 0 (solved).
//
// Search per board: as solve2 (events = contradiction or fixpoint; count up to 2
// completions under MRV, lex re-search when two are found; lowest-open-cell
// branching under LEX).  A board's search step runs with its 16-bit field pulled
// out of the packed words; the slot (lo/hi) is a compile-time constant of the step
// (step4<0>, step4<1>), the two 32-lane halves take their steps under exec masks.
// DFS snapshot per level: one 16-bit word per cell, X of an open cell or S | 0x400
// of a closed one.
#pragma once
#include "solve2_kernel.h"

namespace sdk {

#ifndef SDK_SOLVE4_LDS_LEVELS
#define SDK_SOLVE4_LDS_LEVELS 0
#endif
#ifndef SDK_SOLVE4_TAIL_DIV
#define SDK_SOLVE4_TAIL_DIV 128       // the shared dequeue tail: n / this boards (32 to round 3: profiles/r03/ab_tail_size2.log)
#endif
#ifndef SDK_SOLVE4_TAIL_CHUNK_DIV
#define SDK_SOLVE4_TAIL_CHUNK_DIV 1   // tail chunks: chunk / this boards
#endif
#ifndef SDK_SOLVE4_WAVES_PER_EU
#define SDK_SOLVE4_WAVES_PER_EU 7
#endif
// Measurement build only (tools/build_variant.sh noout -DSDK_SOLVE4_NO_OUTPUT=1): no board is
// written (statuses still are) -- the A/B that prices the solver's whole output write, and so
// an upper bound of what its extra write sectors cost (solver traffic)
#ifndef SDK_SOLVE4_NO_OUTPUT
#define SDK_SOLVE4_NO_OUTPUT 0
#endif
// DFS levels kept in LDS (per level: 2 slots x 64 lanes x 8 B = 1 KiB; deeper levels go
// to the per-workgroup global stack).  Default 0: a 17-clue board rarely branches, so the
// stack is cold, and the 4.5 KiB block lets occupancy follow the VGPR budget: 7 waves per
// SIMD at 72 VGPRs (A/B, 10M 17-clue puzzles: 890 vs 883M/s at 6 waves / 80 VGPRs; at 72 the
// dequeue code must stay straight-line, or the round's LDS addresses spill, see next_board4).
constexpr int kLds4Levels = SDK_SOLVE4_LDS_LEVELS;

// Profiling build only (tools/build_variant.sh prof -DSDK_SOLVE4_PROFILE=1,
// tools/solve4_prof.py): shader-clock cycles of the wave per part of the loop, summed
// over all waves into g_prof4 (0 rounds, 1/2 steps of slot 0/1, 3 finish + next board,
// 4 locked candidates, 5 backtrack, 6 branch, 8 whole loop, 9 loop iterations).
#ifndef SDK_SOLVE4_PROFILE
#define SDK_SOLVE4_PROFILE 0
#endif
#if SDK_SOLVE4_PROFILE
__device__ unsigned long long g_prof4[10];
__shared__ unsigned long long s_prof4[10];   // this wave's sums (one wave per workgroup)
__device__ __forceinline__ void prof4_add(int k, uint64_t v) {
    const uint64_t em = __builtin_amdgcn_read_exec();
    if ((int)__lane_id() == __builtin_ctzll(em)) s_prof4[k] += v;
}
#define PROF4(k, ...)                                               \
    do {                                                            \
        const uint64_t t0_ = __builtin_amdgcn_s_memtime();          \
        __VA_ARGS__;                                                \
        prof4_add(k, __builtin_amdgcn_s_memtime() - t0_);           \
    } while (0)
#else
#define PROF4(k, ...) \
    do {              \
        __VA_ARGS__;  \
    } while (0)
#endif
// Timeline build only (tools/build_variant.sh tl -DSDK_SOLVE4_TIMELINE=1, tools/timeline.py):
// per workgroup, s_memrealtime (100 MHz, one clock for the whole chip) at kernel entry, once
// both slots of both halves hold their first board, at the last dequeue that returned boards,
// and at exit -- the launch's dispatch ramp, start-up and drain.
#ifndef SDK_SOLVE4_TIMELINE
#define SDK_SOLVE4_TIMELINE 0
#endif
#if SDK_SOLVE4_TIMELINE
constexpr int kTl4Max = 16384;
__device__ unsigned long long g_tl4[kTl4Max][4];
#define TL4(k)                                                                   \
    do {                                                                         \
        if (blockIdx.x < (unsigned)kTl4Max) g_tl4[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define TL4(k) \
    do {       \
    } while (0)
#endif
constexpr int kStack4WordsPerBlock = kMaxDepth * 2 * 64 * 2;
constexpr uint32_t kC2 = 0x01FF01FFu;                 // candidate bits of both boards
constexpr uint32_t kInert4 = 0x200u;                  // inert marker (one board)
constexpr uint32_t kInert4x2 = 0x02000200u;

// Packed 16-bit integer ops (every 16-bit half holds a value <= 0x3FF).  The masks
// are inline asm: written as vector code, clang turns a sign mask and the select
// it feeds into per-half compares, v_cndmask and v_perm, costing more than the
// packing saves.  Inline constants apply to both halves (op_sel_hi:[0,1] for the
// shift count).
// per 16-bit half: 0xFFFF where the half is 0, else 0     ((a - 1) >>s 15)
__device__ __forceinline__ uint32_t z16(uint32_t a) {
    uint32_t r;
    asm("v_pk_add_u16 %0, %1, -1\n\tv_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]" : "=&v"(r) : "v"(a));
    return r;
}
// per 16-bit half: 0xFFFF where the half is not 0, else 0  ((0 - a) >>s 15)
__device__ __forceinline__ uint32_t nz16(uint32_t a) {
    uint32_t r;
    asm("v_pk_sub_u16 %0, 0, %1\n\tv_pk_ashrrev_i16 %0, 15, %0 op_sel_hi:[0,1]" : "=&v"(r) : "v"(a));
    return r;
}
// per 16-bit half: a - 1 (no borrow across the halves)
__device__ __forceinline__ uint32_t dec16(uint32_t a) {
    uint32_t r;
    asm("v_pk_add_u16 %0, %1, -1" : "=v"(r) : "v"(a));
    return r;
}
__device__ __forceinline__ uint32_t min16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int HI>
__device__ __forceinline__ uint32_t fld(uint32_t w) {
    return HI ? (w >> 16) : (w & 0xFFFFu);
}
template <int HI>
__device__ __forceinline__ uint32_t setfld(uint32_t w, uint32_t v) {
    return HI ? ((w & 0xFFFFu) | (v << 16)) : ((w & 0xFFFF0000u) | v);
}

// Lane layout (solve2's).  Every lane, spare lanes 27..31 included, owns cells
// c0, c0+27, c0+54 and reads the unit summaries ucol, ur0 + {0,3,6}, ub0 + {0,3,6},
// so each group of three LDS accesses is one base register plus immediate offsets.
// Spare lanes own the inert slots 91+e, 118+e, 145+e -- banks that no real cell of the
// same ds_write_b64 lane group uses (tools/lds_banks.py: no conflict in any access of a
// round) -- and read lane 0's units (their cells are never open, so what they read
// does not matter; same addresses = broadcast).
constexpr int kCells4 = 150;                          // LDS cell slots per half
// Unit words follow the cells in the same per-half region: unit u at slot kCells4 + u,
// and every lane writes its unit word kCells4 slots past its first cell's slot (spare
// lanes into kCells4 + 91..95, read by nobody), so the cell stores and the unit store
// share one address register.  Same banks as separate arrays: the half stride,
// 2 * kRegion4 dwords, is 44 mod 64 like the cells' own 2 * kCells4.
constexpr int kRegion4 = kCells4 + 96;
struct Lane4 {
    int lane, hl, half;
    bool act;
    int c0;
    int ucol, ur0, ub0;
    int ucell[9];
    uint2* s_cell;            // this half's kCells4 (X, S) words, then its units
    uint2* s_unit;            // this half's 32 (T, once) words
    uint8_t* s_in;            // this half's input bytes, [slot][81]
};

// per-lane fields from a lane id (everything but ucell)
__device__ __forceinline__ void lane4_base(Lane4& w, uint2* s_region_all, uint8_t* s_in_all, int lane) {
    w.lane = lane;
    w.hl = lane & 31;
    w.half = lane >> 5;
    w.act = w.hl < 27;
    const int j = w.act ? w.hl : 0;
    w.c0 = w.act ? j : 91 + (w.hl - 27);
    w.ucol = 9 + j % 9;
    w.ur0 = j / 9;
    w.ub0 = 18 + (j % 9) / 3;
    w.s_cell = s_region_all + w.half * kRegion4;
    w.s_unit = w.s_cell + kCells4;
    w.s_in = s_in_all + w.half * 2 * 81;
}

// the propagation loop's lane (all fields)
__device__ __forceinline__ void init_lane4(Lane4& w, uint2* s_region_all, uint8_t* s_in_all) {
    Lane2 l2;
    init_lane2(l2, nullptr, nullptr);
    lane4_base(w, s_region_all, s_in_all, (int)threadIdx.x);
#pragma unroll
    for (int k = 0; k < 9; ++k) w.ucell[k] = l2.ucell[k];
}

// The search steps' lane: the same fields (ucell aside) from a lane id that a volatile
// asm reads, so the compiler cannot hoist what the steps derive from it out of the
// propagation loop.  Hoisted and kept live across the loop, those addresses and
// indices spilled to scratch and every step waited on memory to reload them; the
// round's own LDS addresses (the loop lane's) stay in registers.
__device__ __forceinline__ Lane4 lane4_fresh(uint2* s_region_all, uint8_t* s_in_all) {
    int lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    Lane4 w;
    lane4_base(w, s_region_all, s_in_all, lane);
    return w;
}

__device__ __forceinline__ bool half_any4(const Lane4& w, bool pred) {
    const unsigned long long b = __ballot(pred);
    return (w.half ? (uint32_t)(b >> 32) : (uint32_t)b) != 0u;
}

__device__ __forceinline__ uint32_t half_first4(const Lane4& w, uint32_t v) {
    const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 32);
    return w.half ? b : a;
}

// a wave-uniform 64-bit lane mask with every 32-lane half that has a set bit filled
__device__ __forceinline__ uint64_t spread_halves(uint64_t m) {
    // scalar compare/select (clang otherwise rebuilds this as 64-bit VALU compares)
    uint32_t lo, hi;
    asm("s_cmp_lg_u32 %1, 0\n\ts_cselect_b32 %0, -1, 0" : "=s"(lo) : "s"((uint32_t)m) : "scc");
    asm("s_cmp_lg_u32 %1, 0\n\ts_cselect_b32 %0, -1, 0" : "=s"(hi) : "s"((uint32_t)(m >> 32)) : "scc");
    return ((uint64_t)hi << 32) | lo;
}

// packed lane state: the lane's three cells of both boards of its half
struct Cells4 {
    uint32_t x0, x1, x2, s0, s1, s2;
    uint32_t D, E;            // statics of the lane's unit (both boards); D as kC2 & ~D
};

// update of one cell of both boards (see the header): a closed cell (X = 0) stays
// as it is, an open one loses T, takes a hidden single, and closes when one
// candidate is left.  One asm block (v_bitop3_b32 truth tables over S0 = 0xF0,
// S1 = 0xCC, S2 = 0xAA): split into separate statements, every packed op becomes
// its own asm statement and clang pads each one's consumer with an s_nop.
//   v1 = X & ~U              h  = v1 & H           hm = nz16(h)
//   v2 = h | (v1 & ~hm)      (the hidden single, or what is left)
//   bm |= h & dec16(h)       (two hidden singles for one cell)
//   sg = z16(v2 & dec16(v2)) (at most one candidate left)
//   m  = v2 | S              (0 in a half: an open cell without candidates)
//   S |= v2 & sg             Xn = v2 & ~sg          chg |= X ^ Xn
__device__ __forceinline__ void upd4(uint32_t& X, uint32_t& S, uint32_t U, uint32_t H, uint32_t& bm, uint32_t& m,
                                     uint32_t& chg) {
    uint32_t xn, v1, h, t, v2;
    asm("v_bitop3_b32 %[v1], %[x], %[u], %[u] bitop3:0x30\n\t"
        "v_and_b32 %[h], %[v1], %[hh]\n\t"
        "v_pk_sub_u16 %[t], 0, %[h]\n\t"
        "v_pk_ashrrev_i16 %[t], 15, %[t] op_sel_hi:[0,1]\n\t"
        "v_bitop3_b32 %[v2], %[h], %[v1], %[t] bitop3:0xf4\n\t"
        "v_pk_add_u16 %[t], %[h], -1\n\t"
        SDK_ANDOR("%[bm]", "%[h]", "%[t]", "%[bm]")
        "v_pk_add_u16 %[t], %[v2], -1\n\t"
        "v_and_b32 %[t], %[v2], %[t]\n\t"
        "v_or_b32 %[m], %[v2], %[s]\n\t"
        "v_pk_add_u16 %[t], %[t], -1\n\t"
        "v_pk_ashrrev_i16 %[t], 15, %[t] op_sel_hi:[0,1]\n\t"
        SDK_ANDOR("%[s]", "%[v2]", "%[t]", "%[s]")
        "v_bitop3_b32 %[xn], %[v2], %[t], %[t] bitop3:0x30\n\t"
        "v_bitop3_b32 %[chg], %[chg], %[x], %[xn] bitop3:0xf6"
        : [xn] "=&v"(xn), [v1] "=&v"(v1), [h] "=&v"(h), [t] "=&v"(t), [v2] "=&v"(v2), [m] "=&v"(m),
          [s] "+v"(S), [bm] "+v"(bm), [chg] "+v"(chg)
        : [x] "v"(X), [u] "v"(U), [hh] "v"(H));
    X = xn;
}

// upd4 for waves whose boards are all exact (see unit4x): no "two hidden singles" test and
// no empty-cell test (an open cell with no candidate left closes with S = 0: its units then
// miss a digit, which the missing-digit test reports at the latest in the round that finds
// the board complete).
// Such a cell keeps both digits as candidates, each the only place of its digit in some
// unit; every completion then misses one of them, so the missing-digit test refutes each
// branch on it -- only later, in states that are contradictory anyway.
__device__ __forceinline__ void upd4x(uint32_t& X, uint32_t& S, uint32_t U, uint32_t H, uint32_t& bm, uint32_t& m,
                                      uint32_t& chg) {
    uint32_t xn, v1, h, t, v2;
    asm("v_bitop3_b32 %[v1], %[x], %[u], %[u] bitop3:0x30\n\t"
        "v_and_b32 %[h], %[v1], %[hh]\n\t"
        "v_pk_sub_u16 %[t], 0, %[h]\n\t"
        "v_pk_ashrrev_i16 %[t], 15, %[t] op_sel_hi:[0,1]\n\t"
        "v_bitop3_b32 %[v2], %[h], %[v1], %[t] bitop3:0xf4\n\t"
        "v_pk_add_u16 %[t], %[v2], -1\n\t"
        "v_and_b32 %[t], %[v2], %[t]\n\t"
        "v_pk_add_u16 %[t], %[t], -1\n\t"
        "v_pk_ashrrev_i16 %[t], 15, %[t] op_sel_hi:[0,1]\n\t"
        SDK_ANDOR("%[s]", "%[v2]", "%[t]", "%[s]")
        "v_bitop3_b32 %[xn], %[v2], %[t], %[t] bitop3:0x30\n\t"
        "v_bitop3_b32 %[chg], %[chg], %[x], %[xn] bitop3:0xf6"
        : [xn] "=&v"(xn), [v1] "=&v"(v1), [h] "=&v"(h), [t] "=&v"(t), [v2] "=&v"(v2),
          [s] "+v"(S), [bm] "+v"(bm), [chg] "+v"(chg)
        : [x] "v"(X), [u] "v"(U), [hh] "v"(H));
    X = xn;
    m = 0x00010001u;   // no empty-cell test (see above)
}

// Unit summary of the lane's unit from its nine (X, S) cell words, one asm block.
// "In two or more cells" is accumulated two cells at a time: a bit is set in at
// least two of (acc, a, b) exactly when it is in their majority (bitop3 0xe8).
//   once = OR X & ~twice(X) & E            T = OR S & kC2
//   bm   = (twice(S) & Dn) | (E & ~(OR X | OR S))      (Dn = kC2 & ~D of the header)
__device__ __forceinline__ void unit4(const uint2 (&v)[9], uint32_t E, uint32_t Dn, uint32_t& once, uint32_t& T,
                                      uint32_t& bm) {
    uint32_t ox, os, t0, t1, t2, t3;
    asm(SDK_OR3("%[ox]", "%[a0]", "%[a1]", "%[a2]")
        "v_bitop3_b32 %[t0], %[a0], %[a1], %[a2] bitop3:0xe8\n\t"
        "v_bitop3_b32 %[t1], %[ox], %[a3], %[a4] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a3]", "%[a4]")
        "v_bitop3_b32 %[t2], %[ox], %[a5], %[a6] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a5]", "%[a6]")
        "v_bitop3_b32 %[t3], %[ox], %[a7], %[a8] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a7]", "%[a8]")
        SDK_OR3("%[t0]", "%[t0]", "%[t1]", "%[t2]")
        "v_bitop3_b32 %[t0], %[ox], %[t0], %[t3] bitop3:0x10\n\t"
        "v_and_b32 %[once], %[t0], %[e]\n\t"
        SDK_OR3("%[os]", "%[b0]", "%[b1]", "%[b2]")
        "v_bitop3_b32 %[t0], %[b0], %[b1], %[b2] bitop3:0xe8\n\t"
        "v_bitop3_b32 %[t1], %[os], %[b3], %[b4] bitop3:0xe8\n\t"
        SDK_OR3("%[os]", "%[os]", "%[b3]", "%[b4]")
        "v_bitop3_b32 %[t2], %[os], %[b5], %[b6] bitop3:0xe8\n\t"
        SDK_OR3("%[os]", "%[os]", "%[b5]", "%[b6]")
        "v_bitop3_b32 %[t3], %[os], %[b7], %[b8] bitop3:0xe8\n\t"
        SDK_OR3("%[os]", "%[os]", "%[b7]", "%[b8]")
        SDK_OR3("%[t0]", "%[t0]", "%[t1]", "%[t2]")
        "v_bitop3_b32 %[t0], %[t0], %[t3], %[dn] bitop3:0xa8\n\t"
        "v_bitop3_b32 %[t1], %[e], %[ox], %[os] bitop3:0x10\n\t"
        "v_or_b32 %[bm], %[t0], %[t1]\n\t"
        "v_and_b32 %[tt], 0x1ff01ff, %[os]"
        : [ox] "=&v"(ox), [os] "=&v"(os), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
          [once] "=&v"(once), [bm] "=&v"(bm), [tt] "=&v"(T)
        : [a0] "v"(v[0].x), [a1] "v"(v[1].x), [a2] "v"(v[2].x), [a3] "v"(v[3].x), [a4] "v"(v[4].x),
          [a5] "v"(v[5].x), [a6] "v"(v[6].x), [a7] "v"(v[7].x), [a8] "v"(v[8].x),
          [b0] "v"(v[0].y), [b1] "v"(v[1].y), [b2] "v"(v[2].y), [b3] "v"(v[3].y), [b4] "v"(v[4].y),
          [b5] "v"(v[5].y), [b6] "v"(v[6].y), [b7] "v"(v[7].y), [b8] "v"(v[8].y),
          [e] "v"(E), [dn] "v"(Dn));
}

// A board's statics (D, E of every unit) from its FIRST round instead of a pass of their own
// (statics4: 3 stores, 9 unit reads and two wave barriers per board start).  A board that starts
// carries E = kFresh4 in its half; a round of a wave with such a board reads the same nine cell
// words a statics pass would -- at the first round a board's closed cells are exactly its givens --
// and derives D and E from them (unit4f) before they are used.
constexpr uint32_t kFresh4 = 0x8000u;                 // E of a board whose statics are pending
// the plain kernel only: the donation kernel keeps statics4 (its 96-VGPR build spills a 64-bit
// value to an odd register pair with unit4f, which the gfx950 backend rejects)
constexpr bool kFresh4Round = true;   // round 4: +1.9 % on 10M 17-clue (4 A/B pairs), the rest within noise


// unit4 for a round of a wave where some board just started (its E half = kFresh4): that
// board's statics come from the nine cells read here (its closed cells are its givens):
//   dup = digits taken twice (given twice), inert = an out-of-domain given in the unit,
//   E = 0x1FF if neither, D (as Dn = kC2 & ~dup); the other boards keep theirs.
// Then once / T / bm as unit4 with the new statics.  E and Dn are rewritten in place.
__device__ __forceinline__ void unit4f(const uint2 (&v)[9], uint32_t& E, uint32_t& Dn, uint32_t& once, uint32_t& T,
                                       uint32_t& bm) {
    // as many temporaries as unit4 (its register budget): t1..t3 are reused once twice(S) is
    // formed (t1 = fresh mask, t2 = exact digits, t3 = dup), E and Dn are rewritten in place
    uint32_t ox, os, t0, t1, t2, t3;
    asm(SDK_OR3("%[ox]", "%[a0]", "%[a1]", "%[a2]")
        "v_bitop3_b32 %[t0], %[a0], %[a1], %[a2] bitop3:0xe8\n\t"
        "v_bitop3_b32 %[t1], %[ox], %[a3], %[a4] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a3]", "%[a4]")
        "v_bitop3_b32 %[t2], %[ox], %[a5], %[a6] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a5]", "%[a6]")
        "v_bitop3_b32 %[t3], %[ox], %[a7], %[a8] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a7]", "%[a8]")
        SDK_OR3("%[t0]", "%[t0]", "%[t1]", "%[t2]")
        "v_bitop3_b32 %[once], %[ox], %[t0], %[t3] bitop3:0x10\n\t"   // candidates in exactly one cell
        SDK_OR3("%[os]", "%[b0]", "%[b1]", "%[b2]")
        "v_bitop3_b32 %[t0], %[b0], %[b1], %[b2] bitop3:0xe8\n\t"
        "v_bitop3_b32 %[t1], %[os], %[b3], %[b4] bitop3:0xe8\n\t"
        SDK_OR3("%[os]", "%[os]", "%[b3]", "%[b4]")
        "v_bitop3_b32 %[t2], %[os], %[b5], %[b6] bitop3:0xe8\n\t"
        SDK_OR3("%[os]", "%[os]", "%[b5]", "%[b6]")
        "v_bitop3_b32 %[t3], %[os], %[b7], %[b8] bitop3:0xe8\n\t"
        SDK_OR3("%[os]", "%[os]", "%[b7]", "%[b8]")
        SDK_OR3("%[t0]", "%[t0]", "%[t1]", "%[t2]")
        "v_or_b32 %[t0], %[t0], %[t3]\n\t"                                // twice(S)
        "v_pk_ashrrev_i16 %[t1], 15, %[e] op_sel_hi:[0,1]\n\t"          // fm: 0xFFFF in fresh halves
        "v_and_b32 %[t2], 0x2000200, %[os]\n\t"                         // an inert given
        "v_and_b32 %[t3], 0x1ff01ff, %[t0]\n\t"                         // dup
        "v_or_b32 %[t2], %[t2], %[t3]\n\t"
        "v_pk_add_u16 %[t2], %[t2], -1\n\t"
        "v_pk_ashrrev_i16 %[t2], 15, %[t2] op_sel_hi:[0,1]\n\t"
        "v_and_b32 %[t2], 0x1ff01ff, %[t2]\n\t"                         // exact: 0x1FF
        "v_bitop3_b32 %[e], %[e], %[t2], %[t1] bitop3:0xd8\n\t"         // E = fresh ? exact : E
        "v_xor_b32 %[t3], 0x1ff01ff, %[t3]\n\t"                         // kC2 & ~dup
        "v_bitop3_b32 %[dn], %[dn], %[t3], %[t1] bitop3:0xd8\n\t"       // Dn = fresh ? kC2 & ~dup : Dn
        "v_and_b32 %[once], %[once], %[e]\n\t"
        "v_and_b32 %[t0], %[t0], %[dn]\n\t"
        "v_bitop3_b32 %[t1], %[e], %[ox], %[os] bitop3:0x10\n\t"
        "v_or_b32 %[bm], %[t0], %[t1]\n\t"
        "v_and_b32 %[tt], 0x1ff01ff, %[os]"
        : [ox] "=&v"(ox), [os] "=&v"(os), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
          [once] "=&v"(once), [bm] "=&v"(bm), [tt] "=&v"(T), [e] "+v"(E), [dn] "+v"(Dn)
        : [a0] "v"(v[0].x), [a1] "v"(v[1].x), [a2] "v"(v[2].x), [a3] "v"(v[3].x), [a4] "v"(v[4].x),
          [a5] "v"(v[5].x), [a6] "v"(v[6].x), [a7] "v"(v[7].x), [a8] "v"(v[8].x),
          [b0] "v"(v[0].y), [b1] "v"(v[1].y), [b2] "v"(v[2].y), [b3] "v"(v[3].y), [b4] "v"(v[4].y),
          [b5] "v"(v[5].y), [b6] "v"(v[6].y), [b7] "v"(v[7].y), [b8] "v"(v[8].y));
}

// Ordering point between LDS phases of the one-wave workgroup.  A wave's LDS
// instructions execute in issue order, so a read after a store sees it and a store
// after a read cannot overtake it; all that is needed is that the compiler keeps
// the program order of the accesses (may-alias LDS accesses are never reordered
// across a wave barrier).  __syncthreads() adds s_waitcnt lgkmcnt(0) before every
// phase (and would also drain the VM counter, see DESIGN.md on LDS-DMA prefetch).
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }

// LDS byte address of a __shared__ object (for inline-asm ds_* operands)
__device__ __forceinline__ uint32_t lds_addr4(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// The unit summary when every board of the wave has only exact units (no duplicated
// and no inert given; SDK_OPT_LOCKED != 0): no "taken twice" test and T = OR S.  A
// digit taken twice in an exact unit leaves another digit of the unit with no cell, so
// the missing-digit test still refutes every such state -- at the latest when its last
// cell closes -- and no completion is accepted or lost.
__device__ __forceinline__ void unit4x(const uint2 (&v)[9], uint32_t E, uint32_t& once, uint32_t& T, uint32_t& bm) {
    uint32_t ox, os, t0, t1, t2, t3;
    asm(SDK_OR3("%[ox]", "%[a0]", "%[a1]", "%[a2]")
        "v_bitop3_b32 %[t0], %[a0], %[a1], %[a2] bitop3:0xe8\n\t"
        "v_bitop3_b32 %[t1], %[ox], %[a3], %[a4] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a3]", "%[a4]")
        "v_bitop3_b32 %[t2], %[ox], %[a5], %[a6] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a5]", "%[a6]")
        "v_bitop3_b32 %[t3], %[ox], %[a7], %[a8] bitop3:0xe8\n\t"
        SDK_OR3("%[ox]", "%[ox]", "%[a7]", "%[a8]")
        SDK_OR3("%[t0]", "%[t0]", "%[t1]", "%[t2]")
        "v_bitop3_b32 %[t0], %[ox], %[t0], %[t3] bitop3:0x10\n\t"
        "v_and_b32 %[once], %[t0], %[e]\n\t"
        SDK_OR3("%[os]", "%[b0]", "%[b1]", "%[b2]")
        SDK_OR3("%[os]", "%[os]", "%[b3]", "%[b4]")
        SDK_OR3("%[os]", "%[os]", "%[b5]", "%[b6]")
        SDK_OR3("%[os]", "%[os]", "%[b7]", "%[b8]")
        "v_bitop3_b32 %[bm], %[e], %[ox], %[os] bitop3:0x10"
        : [ox] "=&v"(ox), [os] "=&v"(os), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3),
          [once] "=&v"(once), [bm] "=&v"(bm)
        : [a0] "v"(v[0].x), [a1] "v"(v[1].x), [a2] "v"(v[2].x), [a3] "v"(v[3].x), [a4] "v"(v[4].x),
          [a5] "v"(v[5].x), [a6] "v"(v[6].x), [a7] "v"(v[7].x), [a8] "v"(v[8].x),
          [b0] "v"(v[0].y), [b1] "v"(v[1].y), [b2] "v"(v[2].y), [b3] "v"(v[3].y), [b4] "v"(v[4].y),
          [b5] "v"(v[5].y), [b6] "v"(v[6].y), [b7] "v"(v[7].y), [b8] "v"(v[8].y),
          [e] "v"(E));
    T = os;
}

// One propagation round for all four boards, branch-free.  Out: per-lane packed
// contradiction bits (bad: non-zero in a half = that board is contradictory) and change
// bits (chg).
template <bool EXACT, bool FRESH = false>
__device__ __forceinline__ void round4(const Lane4& w, Cells4& c, uint32_t& bad, uint32_t& chg) {
    w.s_cell[w.c0] = make_uint2(c.x0, c.s0);
    w.s_cell[w.c0 + 27] = make_uint2(c.x1, c.s1);
    w.s_cell[w.c0 + 54] = make_uint2(c.x2, c.s2);
    wave_sync();
    uint2 v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = w.s_cell[w.ucell[k]];
    uint32_t once, T, bm;
    if (EXACT)
        unit4x(v, c.E, once, T, bm);
    else if (FRESH)
        unit4f(v, c.E, c.D, once, T, bm);
    else
        unit4(v, c.E, c.D, once, T, bm);
    w.s_unit[w.c0] = make_uint2(T, once);
    wave_sync();
    uint32_t m0, m1, m2;
    chg = 0;
    // The seven unit reads as single ds_read_b64s: left to itself the compiler pairs
    // them into ds_read2_b64, which takes 8 LDS-array cycles per wave-instruction
    // against 2 x 2 for two ds_read_b64 (MI355X_MICROARCH.md, LDS table).  Issued in
    // the order the three cell updates consume them; each update waits only for its
    // own reads (LDS returns in order, so a counted lgkmcnt stays correct whatever
    // else is in flight); the previous update's results pass through each wait so
    // the compiler cannot sink that update below it.
    uint64_t uc, r0, b0, r1, b1, r2, b2;
    asm volatile(
        "ds_read_b64 %0, %7\n\t"
        "ds_read_b64 %1, %8\n\t"
        "ds_read_b64 %2, %9\n\t"
        "ds_read_b64 %3, %8 offset:24\n\t"
        "ds_read_b64 %4, %9 offset:24\n\t"
        "ds_read_b64 %5, %8 offset:48\n\t"
        "ds_read_b64 %6, %9 offset:48"
        : "=&v"(uc), "=&v"(r0), "=&v"(b0), "=&v"(r1), "=&v"(b1), "=&v"(r2), "=&v"(b2)
        : "v"(lds_addr4(w.s_unit + w.ucol)), "v"(lds_addr4(w.s_unit + w.ur0)), "v"(lds_addr4(w.s_unit + w.ub0))
        : "memory");
    asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(uc), "+v"(r0), "+v"(b0)::"memory");
    const uint32_t ucx = (uint32_t)uc, ucy = (uint32_t)(uc >> 32);
    (EXACT ? upd4x : upd4)(c.x0, c.s0, sdk_or3(ucx, (uint32_t)r0, (uint32_t)b0),
         sdk_or3(ucy, (uint32_t)(r0 >> 32), (uint32_t)(b0 >> 32)), bm, m0,
         chg);
    asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(r1), "+v"(b1), "+v"(c.x0), "+v"(c.s0)::"memory");
    (EXACT ? upd4x : upd4)(c.x1, c.s1, sdk_or3(ucx, (uint32_t)r1, (uint32_t)b1),
         sdk_or3(ucy, (uint32_t)(r1 >> 32), (uint32_t)(b1 >> 32)), bm, m1,
         chg);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r2), "+v"(b2), "+v"(c.x1), "+v"(c.s1)::"memory");
    (EXACT ? upd4x : upd4)(c.x2, c.s2, sdk_or3(ucx, (uint32_t)r2, (uint32_t)b2),
         sdk_or3(ucy, (uint32_t)(r2 >> 32), (uint32_t)(b2 >> 32)), bm, m2,
         chg);
    // an open cell without candidates (a zero half of m0..m2); exact waves leave it to the
    // missing-digit test (upd4x)
    bad = EXACT ? bm : bm | z16(min16(min16(m0, m1), m2));
}

// per-slot search state, uniform within the half.  It lives in LDS between steps
// (s_slot[half][slot]) and in registers only inside a step; the propagation loop
// keeps just `active`.  Rounds are counted by the loop iteration (wave-uniform)
// minus the iteration the board started at.
struct Slot4 {
    uint32_t bidx, bend;
    uint32_t depth, order, count, lim;
    uint32_t rstart, active;  // active: bit 0 a board is loaded, bit 1 the home segment is drained (heads)
    uint32_t maxd;            // deepest DFS level reached (SDK_WORK_DEPTH)
    uint64_t nodes;
};
static __shared__ Slot4 s_slot4[4];      // per-slot search state between steps: s_slot4[half * 2 + slot]

__device__ __forceinline__ uint32_t cell_x4(uint32_t v) {
    return v == 0 ? kCands : 0u;
}
__device__ __forceinline__ uint32_t cell_s4(uint32_t v) {
    return v == 0 ? 0u : (v <= 9 ? (1u << (v - 1u)) : kInert4);
}
// 16-bit snapshot of a cell and back: X if open, S | 0x400 if closed
__device__ __forceinline__ uint32_t snap4(uint32_t x, uint32_t s) {
    return x ? x : (s | 0x400u);
}
__device__ __forceinline__ uint32_t snap_x4(uint32_t y) {
    return (y & 0x400u) ? 0u : y;
}
__device__ __forceinline__ uint32_t snap_s4(uint32_t y) {
    return (y & 0x400u) ? (y & 0x3FFu) : 0u;
}

// kernel arguments as plain values plus the wave's propagation-loop iteration
struct Args4 : Args2 {
    uint32_t iter;
    int locked;
    uint32_t* heads;
    uint32_t seg_size;        // boards per dequeue segment (heads)
    uint32_t tail0;           // first board of the shared tail (heads)
    uint32_t nseg;            // segments in use: min(kHeads, workgroups)
    uint32_t tail_chunk;      // boards per dequeue from the shared tail
    // count mode (frontier counts): every completion of each board is counted (MRV order,
    // same propagation), summed into *count; no boards are written
    int count_mode;
    uint32_t count_lim;       // per-board stop: the count limit, or the flush point 2^31
    bool count_stop;          // count_lim is the caller's limit (stop there), not a flush point
    unsigned long long* count;
    // subtree donation (solve4_kernel<true>, see below): control block, then records, items,
    // registrations and mailboxes at fixed offsets
    struct DnCtl* dn;
};

// ------------------------------------------------------------------ subtree donation
// solve4_kernel<true> (SDK_OPT_DONATE, LEX solves): the reference splits a running search
// at any depth and hands the other half to a free node (DHT_Node.py:491-510).  Here a
// board that has searched kDnEvery more nodes while whole waves sit idle at the end of
// the launch gives away the highest untried digits of its SHALLOWEST stack level -- the
// largest untried subtrees and the lex-greatest part of its remaining search -- as
// "items": the level's propagated state with the branch cell set to one digit each (216 B
// in the lane layout).  Each item goes straight to one idle wave, which searches it like
// a board (a "part" of the board); a part can donate again.
//
// Lex-first answer (ordered acceptance).  In LEX order every cell before a node's branch
// cell is closed, so a part's completions all start with its root prefix: the digits of
// cells 0..cell (plen = cell + 1) of its root; the donor keeps only completions below
// every donated prefix.  Each part stops at its own first completion (its region's
// lex-first one).  A part whose prefix is above some completion already found can hold no
// better one and stops (pruned).  When the last part of a board ends, the finisher
// writes the smallest completion found -- the board's lex-first completion, the
// reference's answer -- unless a part that hit the node budget could still hold a
// smaller one (then SDK_BUDGET_HIT, as for an undonated board).  Only boards whose units
// are all exact donate (no duplicated or inert given: every closed cell is a digit).
//
// Exhaustive mode (launch order MRV: the two-phase solve's phase 2, see sudoku_hip.hip).
// The boards are searched with MRV branching for at most two completions -- a unique
// completion is the lex-first one (the reference's answer).  Every part of a board must
// then be searched to its end, so every donated subtree is needed work.  The parts add
// their completions to the record's `total`; at two the board has several completions
// and every part stops; the finisher writes the unique completion (total 1), restores the
// input (total 0), or marks the board kDnRetryLex (several completions, or a part that
// hit the node budget) for a LEX donation launch.
//
// Hand-off without a shared queue word: once its four slots are idle a wave registers its
// id once (reg[reg_tail++]) and polls only its own mailbox.  A donor takes registrations
// (reg_head moves by compare-and-swap, never past reg_tail), counts the items in the
// board record's `open` parts and only then stores each item index in its receiver's
// mailbox.
// Termination counts BOARDS, not waves: a board is done when its slot finishes it without
// having donated, or when the last open part of its record ends (the record is finalized);
// each adds one to its XCD's `done`.  An idle wave leaves once the eight `done` words add
// up to the launch's board count.  The words only grow, so a sum of eight separate loads
// never exceeds the true total: reaching n means every board is done -- no part runs and no
// item is on its way (an item is counted open before its delivery).  Nothing depends on
// which waves are resident: a launch whose grid is only partly dispatched (a GPU shared
// with another kernel) ends when its boards are done, and a wave dispatched after that
// finds the count complete and leaves.  (Round 4 first counted waves busy at entry and
// idle when they ran dry, with `delivered` read around the sum as a snapshot check; the
// idle waves' loads of those hot words slowed the donors' atomics on them, and a 780-board
// donation launch took 1.75 ms against round 3's 0.89.)
// Every wait on another wave is bounded in time (kDnWaitTicks); one that runs out sets
// `err` (the host fails the solve with SDK_EHIP) and stops all further donation; idle
// waves read `err` every 256th poll and leave once it is set, whatever is still open.  The
// counters and registries are kept per XCD (workgroup % 8, the dispatch's round robin),
// each on its own cache line: thousands of waves go idle at once, and one shared counter
// would serialise their atomics; a donor serves its own XCD's idle waves first (the item it
// writes is then in that XCD's L2).
constexpr int kDnXcds = 8;
struct DnXcd {
    uint32_t done;            // boards finished on this XCD
    uint32_t reg_tail;        // registrations of idle waves
    uint32_t reg_head;        // registrations taken by donors (<= reg_tail)
    uint32_t pad[29];
};
// Resumed split boards (round 4).  The split phase leaves the stack of a board that reaches
// the split budget (split_save4); the collect kernel reserves records and items for it, and
// dn_seed_kernel (sudoku_hip.hip) turns its open subtrees -- the current node's and every
// level's untried digits -- into items of a board record before the donation launch.  Idle
// waves take those items from the seed queue first (dn_idle4), so the heavy boards go on
// from where the split phase left them, spread over the grid, instead of restarting.
struct DnSeed {
    uint32_t next;            // seed-queue entries taken by idle waves
    uint32_t total;           // seed-queue entries (items of the resumed boards)
    uint32_t boards;          // resumed boards: each ends as a record (counted at the exit)
    uint32_t res_boards, res_items;   // the collect kernel's reservations (<= kSeedBoards / kSeedItems)
    uint32_t pad[27];
};
struct DnCtl {
    uint32_t epoch;           // launch number (host): mailbox and registration entries carry it
    uint32_t delivered;       // items handed out by the launch

    uint32_t item_alloc;      // item records handed out
    uint32_t nrec;            // board records handed out
    uint32_t exit_all, parts_ended, finalized;   // diagnostics
    uint32_t next;            // the launch's board dequeue counter
    uint32_t err;             // sticky (not cleared by the prep launch; the host reads and clears
                              // it): kDnErrReg / kDnErrLock, a bounded wait ran out
    uint32_t fault;           // test only (SDK_OPT_DN_FAULT): registrations are not written
    uint32_t started;         // diagnostics: waves taking part (written by workgroup 0)
    uint32_t helpers;         // waves taking part per listed board (SDK_OPT_DONATE_HELPERS), plus 64
    uint32_t pad[20];
    DnXcd x[kDnXcds];
    DnSeed seed;              // own cache line: idle waves take seed items at the launch's start
};
constexpr uint32_t kDnErrReg = 1u, kDnErrLock = 2u, kDnErrSeed = 4u;
// ticket reservation: an add, then the tickets past reg_tail handed back by one compare-and-swap
// (round 4 A/B, profiles/r04 via tools/gpu_r04j.sh: a compare-and-swap loop never passes reg_tail,
// but under contention most donation checks fail -- 1,300 instead of 1,765 items on the heavy-1000
// launch, 1.25 vs 1.08 ms).  SDK_DN_ERRCHECK=0: no error-word read (measurement)
#ifndef SDK_DN_ERRCHECK
#define SDK_DN_ERRCHECK 1
#endif
// bound of every wait on another wave, in s_memrealtime ticks (100 MHz): 0.2 s -- a
// registration is written right after its ticket is drawn and a lock is held for a few
// hundred cycles, so only a wave that cannot run (a fault, or a preempted queue) gets near it
constexpr uint64_t kDnWaitTicks = 20000000ull;
#ifndef SDK_DN_HELP_CAP
#define SDK_DN_HELP_CAP 256
#endif
constexpr uint64_t kDnHelpCap = SDK_DN_HELP_CAP;   // listed boards that get helper waves
constexpr uint32_t kDnItems = 1u << 16;
constexpr uint32_t kDnRecs = 1u << 14;
constexpr uint32_t kDnRegX = 1u << 14;        // registrations per XCD
constexpr uint32_t kDnReg = kDnRegX * kDnXcds;
constexpr uint32_t kDnMbox = 1u << 14;        // workgroups of a donating launch, at most
constexpr int kDnList = 16;
constexpr uint32_t kDnNone = 0xFFFFFFFFu, kDnOwner = 0xFFFFFFFEu;
#ifndef SDK_DN_EVERY
#define SDK_DN_EVERY 16
#endif
constexpr uint32_t kDnEvery = SDK_DN_EVERY;   // nodes between a part's donation / pruning checks
#ifndef SDK_DN_SLEEP
// s_sleep argument between an idle wave's mailbox polls (x 64 clocks: ~3.4 us).  Shorter
// sleeps let the ~23 idle waves of a CU take issue slots and memory bandwidth from the one
// that still searches (s_sleep 4: the 64 heaviest hard boards 1.5 -> 9.7 ms).
#define SDK_DN_SLEEP 127
#endif
constexpr int kDnPruned = 3;                  // part status: stopped above a known completion
constexpr int kDnRetryLex = 3;                // board status of an exhaustive launch: solve again in LEX
struct DnItem {
    uint32_t board, rec, plen, pad0;
    uint32_t pad[4];
    uint2 w[27];              // root state, lane j: (y0 | y1 << 16, y2), snapshot encoding
    uint8_t sol[96];          // the part's completion
    uint32_t pad2[10];
};
struct DnRec {                // one per donating board
    uint32_t board, open, nhit, flags, maxd;
    uint32_t lock;            // LEX: guards `best` (taken by one half-wave at a time, see dn_finish_part4)
    uint32_t version;         // LEX: seqlock of `best` (odd while it is rewritten)
    uint32_t have;            // LEX: `best` holds a completion
    unsigned long long work;
    uint32_t first;           // exhaustive: the part that met the board's first completion
    uint32_t total;           // exhaustive: completions met by all parts
    uint32_t hit[kDnList];    // parts that hit the node budget (more: flags bit 0, undecided)
    uint8_t best[96];         // LEX: the smallest completion any part met
    uint8_t owner_sol[96];    // the board's own slot's completion
    uint32_t pad[20];
};
static_assert(sizeof(DnItem) == 384 && sizeof(DnRec) == 384 && sizeof(DnCtl) == 128 * (2 + kDnXcds), "donation layout");
constexpr size_t kDnRecOffset = sizeof(DnCtl);
constexpr size_t kDnItemOffset = kDnRecOffset + (size_t)kDnRecs * sizeof(DnRec);
constexpr size_t kDnRegOffset = kDnItemOffset + (size_t)kDnItems * sizeof(DnItem);
constexpr size_t kDnMboxOffset = kDnRegOffset + (size_t)kDnReg * 8;
constexpr size_t kDnSeedQOffset = kDnMboxOffset + (size_t)kDnMbox * 8;
constexpr size_t kDnBytes = kDnSeedQOffset + (size_t)kDnItems * 4;
constexpr uint32_t kSeedBoards = kDnRecs / 2;   // the other half stays for the launch's own donations
constexpr uint32_t kSeedItems = kDnItems / 2;
// the split phase's saved stacks: a board's levels 0..depth-1, the 32 lanes of its half each
constexpr uint32_t kSaveLv = 16;
constexpr uint32_t kSaveCap = 8192;
struct SplitSave {
    uint32_t count;           // saves claimed (those past kSaveCap are not written)
    uint32_t pad[31];
    uint2 hdr[kSaveCap];      // (board, depth)
    uint2 lv[kSaveCap][kSaveLv][32];
};
__device__ __forceinline__ DnRec* dn_recs4(const Args4& a) {
    return reinterpret_cast<DnRec*>(reinterpret_cast<char*>(a.dn) + kDnRecOffset);
}
__device__ __forceinline__ DnItem* dn_items4(const Args4& a) {
    return reinterpret_cast<DnItem*>(reinterpret_cast<char*>(a.dn) + kDnItemOffset);
}
__device__ __forceinline__ unsigned long long* dn_reg4(const Args4& a) {
    return reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(a.dn) + kDnRegOffset);
}
__device__ __forceinline__ unsigned long long* dn_mbox4(const Args4& a) {
    return reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(a.dn) + kDnMboxOffset);
}
__device__ __forceinline__ uint32_t* dn_seedq4(const Args4& a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.dn) + kDnSeedQOffset);
}
struct SlotDn {
    uint32_t rec, part, base, plen;   // record, part id (item / kDnOwner), first live stack level,
                                      // prefix length (bit 31: pruned, end the part at its next step)
};
constexpr uint32_t kDnAbort = 0x80000000u;
// a part that ended, waiting for its bookkeeping (dn_finish_part4, run once per loop
// iteration: inlined at one place instead of at every end of a search step)
struct DnFin {
    uint32_t rec, part;
    int st;
    uint32_t maxd;
    unsigned long long work;
};
static __shared__ SlotDn s_dn4[4];    // per slot (half * 2 + slot); referenced by solve4_kernel<true> only
static __shared__ DnFin s_dnfin4[4];
static __shared__ uint32_t s_dnpend4; // bit k: s_dnfin4[k] waits; bit 4 + k: slot k's check is due
static __shared__ uint32_t s_dnwave4; // bit 1: registered, bit 2: seed queue drained, bits 8..: polls
static __shared__ uint32_t s_dntarget4;  // boards of the launch: listed + resumed (the exit count)
static __shared__ uint32_t s_dnseedn4;   // seed-queue entries
static __shared__ uint32_t s_dnepoch4;
static __shared__ uint32_t s_dnfault4; // DnCtl.fault, read once at entry (registrations must not wait on it)
static __shared__ uint32_t s_dngrid4;  // waves taking part (dn_grid4); the rest left at once
static __shared__ uint32_t s_deq4;     // the wave's dequeue stage (next_board4)
// the split phase's save area (split_save4), in LDS rather than kernel-argument SGPRs: it is read
// only when a board is saved, and every SGPR live across the round loop is one the allocator may
// spill into a VGPR lane (and then a round address to scratch)
struct SaveP4 {
    struct SplitSave* save;
    uint32_t* save_idx;
};
static __shared__ SaveP4 s_save4;
// First-solution scan of a lex-ordered frontier (solve4_kernel<false, false, true>, sdk_frontier_first):
// frontier board i's completions all precede board i+1's (frontier_kernel.h), so once board i has a
// completion -- or hit the node budget, which decides the answer just the same (status -2) -- no
// board above i can matter.  A board that ends with status 1 or -2 lowers the launch's found word
// to its index (atomicMin); every board polls the word at its first search step and every
// kFsEvery nodes after it and stops, with status kStCancelled, once it lies above it (the
// survey's "shards whose index is above the minimum may stop").  Boards below the
// lowest hit never stop.  The pointer is kept in LDS like the split phase's save area.
constexpr uint32_t kFsEvery = 8;
static __shared__ long long* s_found4;
static __shared__ unsigned long long s_count4;   // count mode: the wave's completions (added to
                                                 // *count once, at the end: same-address atomics
                                                 // per board serialize at ~10 ns)

// runtime-slot field access (the donation paths run once per loop iteration for any slot)
__device__ __forceinline__ uint32_t fld_rt(uint32_t w, uint32_t hi) {
    return hi ? (w >> 16) : (w & 0xFFFFu);
}
__device__ __forceinline__ uint32_t setfld_rt(uint32_t w, uint32_t v, uint32_t hi) {
    return hi ? ((w & 0xFFFFu) | (v << 16)) : ((w & 0xFFFF0000u) | v);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_agent64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// digit of a closed cell in the 16-bit snapshot encoding (S | 0x400 with S = 1 << (digit-1))
__device__ __forceinline__ uint32_t snap_digit4(uint32_t y) {
    return (uint32_t)__ffs(y & 0x1FFu);
}
// A[:L] < B[:L] lexicographically, per 32-lane half; a*, b* = the lane's digits of cells
// c0, c0 + 27, c0 + 54 (every cell index < 81, so three ballots order all cells)
__device__ __forceinline__ bool half_less4(const Lane4& w, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t b0,
                                           uint32_t b1, uint32_t b2, int L) {
    const bool d0 = w.act && w.c0 < L && a0 != b0;
    const bool d1 = w.act && w.c0 + 27 < L && a1 != b1;
    const bool d2 = w.act && w.c0 + 54 < L && a2 != b2;
    const uint64_t D0 = __ballot(d0), D1 = __ballot(d1), D2 = __ballot(d2);
    const uint64_t L0 = __ballot(d0 && a0 < b0), L1 = __ballot(d1 && a1 < b1), L2 = __ballot(d2 && a2 < b2);
    const int sh = 32 * w.half;
    const uint32_t e0 = (uint32_t)(D0 >> sh), e1 = (uint32_t)(D1 >> sh), e2 = (uint32_t)(D2 >> sh);
    const uint32_t l0 = (uint32_t)(L0 >> sh), l1 = (uint32_t)(L1 >> sh), l2 = (uint32_t)(L2 >> sh);
    if (e0) return (l0 >> __builtin_ctz(e0)) & 1u;
    if (e1) return (l1 >> __builtin_ctz(e1)) & 1u;
    if (e2) return (l2 >> __builtin_ctz(e2)) & 1u;
    return false;
}
__device__ __forceinline__ const uint8_t* dn_sol4(const Args4& a, const DnRec* r, uint32_t id) {
    return id == kDnOwner ? r->owner_sol : dn_items4(a)[id].sol;
}
// the lane's three digits of an 81-byte completion
__device__ __forceinline__ void dn_digits4(const Lane4& w, const uint8_t* s, uint32_t& v0, uint32_t& v1, uint32_t& v2) {
    v0 = w.act ? s[w.c0] : 0u;
    v1 = w.act ? s[w.c0 + 27] : 0u;
    v2 = w.act ? s[w.c0 + 54] : 0u;
}
// the lane's three root-prefix digits of item `id`
__device__ __forceinline__ void dn_prefix4(const Lane4& w, const Args4& a, uint32_t id, uint32_t& p0, uint32_t& p1,
                                           uint32_t& p2) {
    p0 = p1 = p2 = 0u;
    if (w.act) {
        const uint2 v = dn_items4(a)[id].w[w.hl];
        p0 = snap_digit4(v.x & 0xFFFFu);
        p1 = snap_digit4(v.x >> 16);
        p2 = snap_digit4(v.y & 0xFFFFu);
    }
}

// an item part: is the smallest completion of its board met so far below its root prefix?
// (`best` is read under its seqlock: a copy torn by a concurrent rewrite is discarded)
__device__ __forceinline__ bool dn_pruned4(const Lane4& w, const Args4& a, const SlotDn& d) {
    const DnRec* r = dn_recs4(a) + d.rec;
    const uint32_t v0 = ld_agent(&r->version);
    if ((v0 & 1u) || !ld_agent(&r->have)) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    uint32_t s0, s1, s2, p0, p1, p2;
    dn_digits4(w, r->best, s0, s1, s2);
    dn_prefix4(w, a, d.part, p0, p1, p2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (ld_agent(&r->version) != v0) return false;
    return half_less4(w, s0, s1, s2, p0, p1, p2, (int)(d.plen & ~kDnAbort));
}

// give the highest untried digits of stack level d.base (the shallowest live one) to idle
// waves, one item each: as many as there are registered idle waves
__device__ __forceinline__ void dn_donate4(const Lane4& w, const Args4& a, const Slot4& b, const Cells4& c,
                                           uint32_t hi, SlotDn* pd, uint2* g_stk) {
    DnCtl* ctl = a.dn;
    const SlotDn d = *pd;
    if (b.depth <= d.base) return;
    // the first XCD (from this workgroup's own) with registered idle waves; all sixteen
    // counters are read at once (one memory round trip, not eight)
    uint32_t tl[kDnXcds], hd[kDnXcds];
#pragma unroll
    for (int k = 0; k < kDnXcds; ++k) {
        tl[k] = ld_agent(&ctl->x[k].reg_tail);
        hd[k] = ld_agent(&ctl->x[k].reg_head);
    }
    uint32_t x = kDnXcds, tail = 0, head = 0;
    for (uint32_t k = 0; k < (uint32_t)kDnXcds && x == kDnXcds; ++k) {
        const uint32_t xx = (blockIdx.x + k) % kDnXcds;
        uint32_t t = 0, h = 0;
#pragma unroll
        for (int q = 0; q < kDnXcds; ++q) {
            t = (uint32_t)q == xx ? tl[q] : t;
            h = (uint32_t)q == xx ? hd[q] : h;
        }
        if (t > h && h < kDnRegX) {
            x = xx;
            tail = t;
            head = h;
        }
    }
    if (x == kDnXcds) return;                                     // no idle wave waits
    if (half_any4(w, w.act && fld_rt(c.E, hi) == 0u)) return;   // only boards with every unit exact
    const uint32_t lvl = d.base;
    uint2* lp = g_stk + (lvl * 2 + hi) * 64 + w.lane;
    const uint2 snap = *lp;
    const uint32_t rec16 = snap.y >> 16;
    const int cell = (int)(rec16 & 0x7Fu);
    const uint32_t rest = rec16 >> 7;
    const uint32_t cnt = (uint32_t)__popc(rest);
    // registrations: tickets t0 .. t0 + valid - 1 are registered idle waves.  The add may take
    // tickets past reg_tail (a stale head): the donor serves only those below the tail it reads
    // after the add and hands the rest back by one compare-and-swap, which fails only if
    // another donor took tickets in between -- then those registrations stay unserved (a
    // wave left idle until the launch ends: throughput, never an answer or termination)
    uint32_t t0 = 0, valid = 0;
    if (w.hl == 0) {
        const uint32_t want = min(cnt, tail - head);
        t0 = atomicAdd(&ctl->x[x].reg_head, want);
        const uint32_t tail2 = min(ld_agent(&ctl->x[x].reg_tail), kDnRegX);
        valid = tail2 > t0 ? min(want, tail2 - t0) : 0u;
        if (valid < want) atomicCAS(&ctl->x[x].reg_head, t0 + want, t0 + valid);
    }
    // a bounded wait ran out: no more donation (the error word is read only by a donor that
    // holds tickets -- in every donation check it cost the heavy-1000 launch ~15 %: the
    // header line it sits on takes the donors' atomics)
    if (SDK_DN_ERRCHECK && w.hl == 0 && valid != 0u && ld_agent(&ctl->err) != 0u) valid = 0u;
    t0 = half_first4(w, t0);
    valid = half_first4(w, valid);
    if (valid == 0) return;
    // board record (first donation of this board)
    DnRec* recs = dn_recs4(a);
    uint32_t r = d.rec;
    if (r == kDnNone) {
        uint32_t v = 0;
        if (w.hl == 0) v = atomicAdd(&ctl->nrec, 1u);
        r = half_first4(w, v);
        if (r >= kDnRecs) return;                                 // the tickets stay unserved
        DnRec* R = recs + r;
        // exhaustive mode: an owner that already met a completion (written to out) carries it
        const bool carry = b.count > 0u;
        if (carry && w.act) {
            const uint8_t* o = a.out + (uint64_t)b.bidx * 81;
            R->owner_sol[w.c0] = o[w.c0];
            R->owner_sol[w.c0 + 27] = o[w.c0 + 27];
            R->owner_sol[w.c0 + 54] = o[w.c0 + 54];
        }
        if (w.hl == 0) {
            R->board = b.bidx;
            R->open = 1;
            R->nhit = R->flags = R->maxd = R->lock = R->version = R->have = 0;
            R->work = 0;
            R->total = b.count;
            R->first = carry ? kDnOwner : kDnNone;
        }
        if (w.hl < kDnList) R->hit[w.hl] = kDnNone;
        if (w.hl == 0) pd->rec = r;
    }
    uint32_t i0 = 0;
    if (w.hl == 0) {
        i0 = atomicAdd(&ctl->item_alloc, valid);
        if (i0 + valid <= kDnItems) atomicAdd(&recs[r].open, valid);
    }
    i0 = half_first4(w, i0);
    if (i0 + valid > kDnItems) return;
    // the `valid` highest digits of the level go
    uint32_t gone = rest;
    for (uint32_t k = valid; k < cnt; ++k) gone &= gone - 1u;       // drop the lowest cnt - valid
    const uint32_t stay = rest & ~gone;
    const uint32_t y0 = snap.x & 0xFFFFu, y1 = snap.x >> 16, y2 = snap.y & 0xFFFFu;
    const bool k0 = w.act && cell == w.c0, k1 = w.act && cell == w.c0 + 27, k2 = w.act && cell == w.c0 + 54;
    DnItem* items = dn_items4(a);
    uint32_t g = gone;
    for (uint32_t k = 0; k < valid; ++k) {
        const uint32_t dbit = g & (0u - g);
        g ^= dbit;
        DnItem* it = items + i0 + k;
        const uint32_t v = dbit | 0x400u;
        if (w.act) it->w[w.hl] = make_uint2((k0 ? v : y0) | ((k1 ? v : y1) << 16), k2 ? v : y2);
        if (w.hl == 0) {
            it->board = b.bidx;
            it->rec = r;
            it->plen = (uint32_t)cell + 1u;
        }
    }
    __threadfence();
    if (w.hl == 0) {
        const uint32_t epoch = s_dnepoch4;
        unsigned long long* reg = dn_reg4(a) + (size_t)x * kDnRegX;
        unsigned long long* mbox = dn_mbox4(a);
        for (uint32_t k = 0; k < valid; ++k) {
            // the registrant writes its entry right after drawing the ticket: a bounded wait
            unsigned long long e;
            bool ok = true;
            const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
            for (uint32_t it = 1; ((e = ld_agent64(reg + t0 + k)) >> 32) != epoch; ++it) {
                if ((it & 31u) == 0u && __builtin_amdgcn_s_memrealtime() - t_start > kDnWaitTicks) {
                    ok = false;     // the clock is read every 32 polls: the wait stays a plain poll
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) {   // the items left stay undelivered (and not open): the solve reports SDK_EHIP
                atomicSub(&recs[r].open, valid - k);
                atomicOr(&ctl->err, kDnErrReg);
                break;
            }
            __hip_atomic_store(mbox + (uint32_t)e, ((unsigned long long)epoch << 32) | (i0 + k), __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        atomicAdd(&ctl->delivered, valid);   // diagnostics
    }
    // the level keeps its lower untried digits; with none left it is the donor's no more
    if (stay == 0u) {
        if (w.hl == 0) pd->base = lvl + 1u;   // the part ends when it backtracks to it
    } else {
        lp->y = (snap.y & 0xFFFFu) | (((uint32_t)cell | (stay << 7)) << 16);
    }
}

// the last part of a board: write its answer (see above)
__device__ __forceinline__ void dn_finalize4(const Lane4& w, const Args4& a, const DnRec* r) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t board = ld_agent(&r->board);
    const uint32_t nhit = ld_agent(&r->nhit), flags = ld_agent(&r->flags);
    const uint32_t nh = min(nhit, (uint32_t)kDnList);
    const bool exhaustive = a.order != ORDER_LEX;
    const uint32_t total = ld_agent(&r->total);
    // LEX: the running minimum; exhaustive: the completion of the part that met the first one
    const bool have = exhaustive ? total == 1u : ld_agent(&r->have) != 0u;
    uint32_t b0 = 0, b1 = 0, b2 = 0;
    if (have) dn_digits4(w, exhaustive ? dn_sol4(a, r, ld_agent(&r->first)) : r->best, b0, b1, b2);
    bool blocked = flags != 0u;   // the hit list overflowed: undecided
    for (uint32_t k = 0; k < (exhaustive ? 0u : nh) && !blocked; ++k) {
        const uint32_t id = ld_agent(&r->hit[k]);
        if (id == kDnOwner) {
            blocked = true;       // the board's own part: its region holds the smallest prefixes
        } else {
            uint32_t p0, p1, p2;
            dn_prefix4(w, a, id, p0, p1, p2);
            blocked = !have || !half_less4(w, b0, b1, b2, p0, p1, p2, (int)dn_items4(a)[id].plen);
        }
    }
    int st = blocked ? -2 : (have ? 1 : 0);
    if (exhaustive) st = (total >= 2u || nhit != 0u || flags != 0u) ? kDnRetryLex : (total == 1u ? 1 : 0);
    uint8_t* dst = a.out + (uint64_t)board * 81;
    if (w.act) {
        if (st == 1) {
            dst[w.c0] = (uint8_t)b0;
            dst[w.c0 + 27] = (uint8_t)b1;
            dst[w.c0 + 54] = (uint8_t)b2;
        } else {   // the reference restores the grid (DHT_Node.py:535)
            const uint8_t* src = a.in + (a.in_first + (uint64_t)board * a.in_step) * 81;
            dst[w.c0] = src[w.c0];
            dst[w.c0 + 27] = src[w.c0 + 27];
            dst[w.c0 + 54] = src[w.c0 + 54];
        }
    }
    if (w.hl == 0) {
        a.status[board] = (int8_t)st;
        if (a.work)
            a.work[board] = a.work_rounds == 2 ? (uint64_t)ld_agent(&r->maxd)
                                               : (uint64_t)ld_agent64(&r->work);
    }
}

// a part of a donating board ended (st: 1 completion written to its sol, 0 refuted, -2 budget
// hit, kDnPruned); the last one to end finalizes the board
__device__ __forceinline__ void dn_finish_part4(const Lane4& w, const Args4& a, const DnFin& f) {
    DnRec* r = dn_recs4(a) + f.rec;
    const int st = f.st;
    __threadfence();              // this part's completion bytes before what follows
    if (st == 1 && a.order == ORDER_LEX) {
        // fold the part's completion into the board's running minimum.  Only this half of the
        // wave runs here (the caller's loop takes one slot at a time), so the spinning lane
        // never waits on its own wave; other waves' holders finish without it.
        // test-and-set, bounded: a holder that cannot finish sets `err` (the fold goes on
        // unlocked; the solve then reports SDK_EHIP and its boards are not used)
        if (w.hl == 0) {
            const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
            while (atomicExch(&r->lock, 1u) != 0u) {
                if (__builtin_amdgcn_s_memrealtime() - t_start > kDnWaitTicks) {
                    atomicOr(&a.dn->err, kDnErrLock);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const bool had = ld_agent(&r->have) != 0u;
        uint32_t s0, s1, s2, b0, b1, b2;
        dn_digits4(w, dn_sol4(a, r, f.part), s0, s1, s2);
        dn_digits4(w, r->best, b0, b1, b2);
        if (!had || half_less4(w, s0, s1, s2, b0, b1, b2, 81)) {
            DnRec* rw = const_cast<DnRec*>(r);
            if (w.hl == 0) __hip_atomic_store(&rw->version, ld_agent(&r->version) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence();
            if (w.act) {
                rw->best[w.c0] = (uint8_t)s0;
                rw->best[w.c0 + 27] = (uint8_t)s1;
                rw->best[w.c0 + 54] = (uint8_t)s2;
            }
            __threadfence();
            if (w.hl == 0) {
                __hip_atomic_store(&rw->have, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&rw->version, ld_agent(&r->version) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        __threadfence();
        if (w.hl == 0) atomicExch(&r->lock, 0u);
    }
    if (w.hl == 0) {
        if (st == -2) {
            const uint32_t k = atomicAdd(&r->nhit, 1u);
            if (k < (uint32_t)kDnList)
                __hip_atomic_store(r->hit + k, f.part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                atomicOr(&r->flags, 1u);
        }
        atomicAdd(&r->work, f.work);
        atomicMax(&r->maxd, f.maxd);
    }
    __threadfence();              // list entries and counters before the open count
    uint32_t old = 0;
    if (w.hl == 0) {
        old = atomicSub(&r->open, 1u);
        atomicAdd(&a.dn->parts_ended, 1u);
        if (old == 1u) atomicAdd(&a.dn->finalized, 1u);
    }
    old = half_first4(w, old);
    if (old == 1u) {
        dn_finalize4(w, a, r);
        if (w.hl == 0) atomicAdd(&a.dn->x[blockIdx.x % kDnXcds].done, 1u);   // the board is done
    }
}

// start item `idx` in slot `hi` of this half
__device__ __forceinline__ void dn_start_item4(const Lane4& w, const Args4& a, Cells4& c, uint32_t hi, uint32_t idx,
                                               Slot4* s_slot) {
    const DnItem* it = dn_items4(a) + idx;
    const uint32_t board = it->board, rec = it->rec, plen = it->plen;
    uint32_t y0 = 0, y1 = 0, y2 = 0;
    if (w.act) {
        const uint2 v = it->w[w.hl];
        y0 = v.x & 0xFFFFu;
        y1 = v.x >> 16;
        y2 = v.y & 0xFFFFu;
    }
    c.x0 = setfld_rt(c.x0, w.act ? snap_x4(y0) : 0u, hi);
    c.x1 = setfld_rt(c.x1, w.act ? snap_x4(y1) : 0u, hi);
    c.x2 = setfld_rt(c.x2, w.act ? snap_x4(y2) : 0u, hi);
    c.s0 = setfld_rt(c.s0, w.act ? snap_s4(y0) : kInert4, hi);
    c.s1 = setfld_rt(c.s1, w.act ? snap_s4(y1) : kInert4, hi);
    c.s2 = setfld_rt(c.s2, w.act ? snap_s4(y2) : kInert4, hi);
    c.D = setfld_rt(c.D, kCands, hi);  // donating boards are exact: no duplicated given
    c.E = setfld_rt(c.E, kCands, hi);
    Slot4 b;
    b.bidx = board;
    b.bend = board + 1u;              // the next dequeue goes to the (drained) shared tail
    b.depth = 0;
    b.order = a.order == ORDER_LEX ? ORDER_LEX : ORDER_MRV;
    b.count = 0;
    b.lim = a.order == ORDER_LEX ? 1u : 2u;
    b.rstart = a.iter;
    b.active = 3u;
    b.maxd = 0;
    b.nodes = 0;
    if (w.hl == 0) {
        s_slot[w.half * 2 + hi] = b;
        s_dn4[w.half * 2 + hi] = SlotDn{rec, idx, 0u, plen};
    }
}

// slot k's donation / pruning check (its step flagged it): an item part already above a
// known completion is marked to end at its next step; otherwise donate to idle waves
__device__ __forceinline__ void dn_check4(const Lane4& w, const Args4& a, const Cells4& c, uint32_t k, Slot4* s_slot,
                                          uint2* g_stk) {
    SlotDn* pd = s_dn4 + k;
    const SlotDn d = *pd;
    if (a.order != ORDER_LEX) {
        // exhaustive mode: every part stops once its board has two completions
        if (d.rec != kDnNone && ld_agent(&dn_recs4(a)[d.rec].total) >= 2u) {
            if (w.hl == 0) pd->plen = d.plen | kDnAbort;
            return;
        }
    } else if (d.rec != kDnNone && d.part != kDnOwner) {
        if (dn_pruned4(w, a, d)) {
            if (w.hl == 0) pd->plen = d.plen | kDnAbort;
            return;
        }
    }
    dn_donate4(w, a, s_slot[k], c, k & 1u, pd, g_stk);
}

// a wave whose four slots are idle: take an item of a resumed board from the seed queue while
// there are any, else register once and poll the mailbox.  Returns 0 to leave (every board of
// the launch done), 1 to poll again, 2 when an item was started in slot 0 of half 0 (A0 then
// covers that half).
__device__ __forceinline__ int dn_idle4(const Lane4& w, const Args4& a, Cells4& c, uint64_t& A0, Slot4* s_slot) {
    DnCtl* ctl = a.dn;
    DnXcd* mx = ctl->x + blockIdx.x % kDnXcds;
    uint32_t st = __builtin_amdgcn_readfirstlane(s_dnwave4);
    const uint32_t epoch = __builtin_amdgcn_readfirstlane(s_dnepoch4);
    unsigned long long* mbox = dn_mbox4(a) + blockIdx.x;
    uint32_t idx = kDnNone;
    if (!(st & 4u)) {
        // seed items first (never while registered: registration follows the first empty
        // claim, and a delivery keeps the drained bit)
        uint32_t q = 0;
        if (w.lane == 0) q = atomicAdd(&ctl->seed.next, 1u);
        q = __builtin_amdgcn_readfirstlane(q);
        if (q < __builtin_amdgcn_readfirstlane(s_dnseedn4))
            idx = __builtin_amdgcn_readfirstlane(ld_agent(dn_seedq4(a) + q));
        else
            st |= 4u;
    }
    if (idx == kDnNone) {
    if (!(st & 2u)) {
        if (w.lane == 0) {
            const uint32_t t = atomicAdd(&mx->reg_tail, 1u);
            if (t < kDnRegX && s_dnfault4 == 0u)
                __hip_atomic_store(dn_reg4(a) + (size_t)(blockIdx.x % kDnXcds) * kDnRegX + t,
                                   ((unsigned long long)epoch << 32) | blockIdx.x, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        st |= 2u;
    }
    // relaxed polls: an acquire at agent scope invalidates the XCD's L2, and thousands of idle
    // waves doing that every few microseconds evict the working waves' stacks and inputs
    const unsigned long long m = ld_agent64(mbox);
    const uint32_t mhi = __builtin_amdgcn_readfirstlane((uint32_t)(m >> 32));
    if (mhi == epoch) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the item's words
        // delivered: the item is an open part of its board; the registration is spent
        idx = __builtin_amdgcn_readfirstlane((uint32_t)m);
        if (w.lane == 0) __hip_atomic_store(mbox, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (w.lane == 0) s_dnwave4 = 4u;   // not registered; the seed queue was drained before
    }
    }
    if (idx != kDnNone) {
        if (w.half == 0) dn_start_item4(w, a, c, 0u, idx, s_slot);
        A0 = 0x00000000FFFFFFFFull;
        return 2;
    }
    st += 0x100u;                             // polls; the boards done every 16th
    if (w.lane == 0) s_dnwave4 = st;
    if (((st >> 8) & 15u) == 1u) {
        // leave when the launch's boards are all done (see the hand-off above: eight monotone
        // words, loaded at once; no agent-scope acquire -- one per check would invalidate the
        // XCD's L2 under the working waves), or (every 256th poll) a bounded wait ran out
        uint32_t done = 0;
#pragma unroll
        for (int k = 0; k < kDnXcds; ++k) done += ld_agent(&ctl->x[k].done);
        const bool err = ((st >> 8) & 255u) == 1u && ld_agent(&ctl->err) != 0u;
        if (__builtin_amdgcn_readfirstlane(done) >= __builtin_amdgcn_readfirstlane(s_dntarget4) ||
            __builtin_amdgcn_readfirstlane(err)) {
            if (w.lane == 0) atomicAdd(&ctl->exit_all, 1u);
            return 0;
        }
    }
    __builtin_amdgcn_s_sleep(SDK_DN_SLEEP);
    return 1;
}

// Locked candidates (pointing and claiming) for the board in slot HI, run at its
// propagation fixpoints before it branches (SDK_OPT_LOCKED).  Over the 54 box-line
// intersections ("triads": row r x stack s, column c x band b, three cells each):
//   pointing  the digits of a box confined to one of its triads leave the rest of
//             that triad's line;
//   claiming  the digits of a line confined to one of its triads leave the rest of
//             that triad's box.
// Both only remove digits that occur in no completion of the node (every unit of
// the board exact: each digit exactly once per unit), so the set of completions,
// and with it the lex-first one the reference returns, is unchanged; only the
// search takes fewer nodes (tools/round_model.py: the five 17-clue classes need no
// branch at all, 1.78 -> 1.00 nodes per puzzle).  Boards with a unit that is not
// exact (duplicated or inert givens) skip the rule.
// Layout: triad t = 3 * line + (index of the crossing box along the line), so the 9
// triads of a band (rows) or stack (columns) are t = 9g .. 9g + 8 and "row k of box s'"
// of that group is t = 9g + 3k + s'.  Lane j < 27 owns row triad j and column triad
// j; phase 1 stores (row OR, column OR) of X at s_unit[kTri4 + t], phase 2 reads the
// 8 other triads of its group in an order rotated to put its own first and stores
// the eliminations of its two triads at s_unit[kElim4 + t], phase 3 applies them to
// the lane's cells (cell (R, C): row triad 3R + C/3, column triad 3C + R/3).
// Returns whether a candidate of slot HI was removed (uniform in the half).
constexpr int kTri4 = 32, kElim4 = 59;                // scratch slots in the unit region
template <int HI>
__device__ __forceinline__ bool lc4(const Lane4& w, Cells4& c) {
    if (half_any4(w, w.act && fld<HI>(c.E) == 0u)) return false;
    // The cell words in LDS are this board's current ones: its last round stored them and
    // changed nothing (a fixpoint), and nothing but a round or statics4 -- which stores
    // the registers -- writes them in between.
    const int j = w.hl;
    if (w.act) {
        const int rb = (j / 3) * 9 + 3 * (j % 3), cb = 27 * (j % 3) + j / 3;
        const uint32_t rt = w.s_cell[rb].x | w.s_cell[rb + 1].x | w.s_cell[rb + 2].x;
        const uint32_t ct = w.s_cell[cb].x | w.s_cell[cb + 9].x | w.s_cell[cb + 18].x;
        w.s_unit[kTri4 + j] = make_uint2(rt, ct);
    }
    wave_sync();
    if (w.act) {
        const int g = 9 * (j / 9), k0 = (j % 9) / 3, s0 = j % 3;
        const int r0 = g + 3 * k0, ra = g + 3 * ((k0 + 1) % 3), rb = g + 3 * ((k0 + 2) % 3);
        const int c1 = (s0 + 1) % 3, c2 = (s0 + 2) % 3;
        const uint2* t = w.s_unit + kTri4;
        const uint2 a01 = t[r0 + c1], a02 = t[r0 + c2];
        const uint2 a10 = t[ra + s0], a11 = t[ra + c1], a12 = t[ra + c2];
        const uint2 a20 = t[rb + s0], a21 = t[rb + c1], a22 = t[rb + c2];
        // pointing from the two other boxes of the line | claiming by the two other lines of the box
        const uint32_t er = (a01.x & ~(a11.x | a21.x)) | (a02.x & ~(a12.x | a22.x)) | (a10.x & ~(a11.x | a12.x)) |
                            (a20.x & ~(a21.x | a22.x));
        const uint32_t ec = (a01.y & ~(a11.y | a21.y)) | (a02.y & ~(a12.y | a22.y)) | (a10.y & ~(a11.y | a12.y)) |
                            (a20.y & ~(a21.y | a22.y));
        w.s_unit[kElim4 + j] = make_uint2(er, ec);
    }
    wave_sync();
    bool ch = false;
    if (w.act) {
        const uint32_t fm = HI ? 0x01FF0000u : 0x1FFu;
        const int rt0 = (j / 9) * 3 + (j % 9) / 3, ct0 = (j % 9) * 3;
        const uint2* e = w.s_unit + kElim4;
        const uint32_t e0 = (e[rt0].x | e[ct0].y) & fm, e1 = (e[rt0 + 9].x | e[ct0 + 1].y) & fm,
                       e2 = (e[rt0 + 18].x | e[ct0 + 2].y) & fm;
        ch = ((c.x0 & e0) | (c.x1 & e1) | (c.x2 & e2)) != 0u;
        c.x0 &= ~e0;
        c.x1 &= ~e1;
        c.x2 &= ~e2;
    }
    return half_any4(w, ch);
}

template <int HI>
__device__ __forceinline__ void start_board4(const Lane4& w, const Args4& a, Slot4& b, Cells4& c, bool reload) {
    uint32_t i0, i1, i2;
    uint8_t* sin = w.s_in + HI * 81;
    if (reload) {
        const uint8_t* src = a.in + (a.in_first + (uint64_t)b.bidx * a.in_step) * 81;
        i0 = w.act ? (uint32_t)src[w.c0] : 0u;
        i1 = w.act ? (uint32_t)src[w.c0 + 27] : 0u;
        i2 = w.act ? (uint32_t)src[w.c0 + 54] : 0u;
        if (w.act) {
            sin[w.c0] = (uint8_t)i0;
            sin[w.c0 + 27] = (uint8_t)i1;
            sin[w.c0 + 54] = (uint8_t)i2;
        }
    } else {
        i0 = w.act ? (uint32_t)sin[w.c0] : 0u;
        i1 = w.act ? (uint32_t)sin[w.c0 + 27] : 0u;
        i2 = w.act ? (uint32_t)sin[w.c0 + 54] : 0u;
    }
    uint32_t x0 = w.act ? cell_x4(i0) : 0u, x1 = w.act ? cell_x4(i1) : 0u, x2 = w.act ? cell_x4(i2) : 0u;
    const uint32_t s0 = w.act ? cell_s4(i0) : kInert4, s1 = w.act ? cell_s4(i1) : kInert4,
                   s2 = w.act ? cell_s4(i2) : kInert4;
    if (a.mask) {
        // TASK `range` restricts the lowest-index empty input cell only (DHT_Node.py:474,522,531);
        // that cell starts open with X = mask, whatever the mask's size (see the header)
        const uint32_t fm = ((uint32_t)a.mask[b.bidx] >> 1) & kCands;
        uint32_t z = ~0u;
        if (w.act)
            z = i0 == 0 ? (uint32_t)w.c0 : (i1 == 0 ? (uint32_t)w.c0 + 27 : (i2 == 0 ? (uint32_t)w.c0 + 54 : ~0u));
        z = half_min(z);
        x0 = (w.act && z == (uint32_t)w.c0) ? fm : x0;
        x1 = (w.act && z == (uint32_t)w.c0 + 27) ? fm : x1;
        x2 = (w.act && z == (uint32_t)w.c0 + 54) ? fm : x2;
    }
    c.x0 = setfld<HI>(c.x0, x0);
    c.x1 = setfld<HI>(c.x1, x1);
    c.x2 = setfld<HI>(c.x2, x2);
    c.s0 = setfld<HI>(c.s0, s0);
    c.s1 = setfld<HI>(c.s1, s1);
    c.s2 = setfld<HI>(c.s2, s2);
    b.depth = 0;
    b.count = 0;
}

// statics (D, E) of the lane's unit for the board in slot HI, from its input givens
template <int HI>
__device__ __forceinline__ void statics4(const Lane4& w, Cells4& c) {
    w.s_cell[w.c0] = make_uint2(c.x0, c.s0);
    w.s_cell[w.c0 + 27] = make_uint2(c.x1, c.s1);
    w.s_cell[w.c0 + 54] = make_uint2(c.x2, c.s2);
    wave_sync();
    uint32_t os = 0, ts = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const uint32_t v = fld<HI>(w.s_cell[w.ucell[k]].y);
        ts |= os & v;
        os |= v;
    }
    wave_sync();   // the next round's stores must not overtake these reads
    const uint32_t dup = ts & kCands;
    const uint32_t exact = (dup == 0u && (os & kInert4) == 0u) ? kCands : 0u;
    c.D = setfld<HI>(c.D, kCands & ~dup);
    c.E = setfld<HI>(c.E, exact);
}

template <int HI, bool FR = false>
__device__ __forceinline__ void next_board4(const Lane4& w, const Lane4& wr, const Args4& a, Slot4& b, Cells4& c) {
    ++b.bidx;
    if (b.bidx >= b.bend) {
        if (a.heads) {
            // XCD-local segment (see kHeads), then the shared tail: straight-line code, no
            // segment-walking loop (its control flow alone made the allocator spill the
            // round's LDS addresses at 72 VGPRs)
            uint32_t base = 0, end = 0;
            // the wave's dequeue stage (s_deq4: 0 segment, 1 shared tail, 2 empty) is shared by
            // its four slots, so a drained head is hit once per wave, not once per slot.  At the
            // end of a launch every wave meets the drained heads at about the same time and
            // same-address atomics serialize (~10 ns each): per slot, 28672 failing atomics
            // on the shared tail cost the 1M 30-clue launch 0.12 ms of its 0.81
            const uint32_t seg = blockIdx.x % a.nseg;   // the home segment (of this workgroup's XCD)
            const uint32_t lo = seg * a.seg_size, hi = min(lo + a.seg_size, a.tail0);
            // a segment's first chunks are dealt, one per slot of its workgroups, so a launch
            // does not open with every slot's atomic on eight heads (3,584 each at 28 waves per
            // CU); the head counts the chunks after them.  A dealt chunk past the segment says
            // nothing about the other slots' (the wave stage only follows the heads)
            const uint32_t dealt_base = lo + ((blockIdx.x / a.nseg) * 4u + (uint32_t)w.half * 2u + HI) * a.chunk;
            const bool dealt_ok = b.bend == 0u && dealt_base < hi;
            bool drained = false;
            if (dealt_ok) {
                base = dealt_base;
                end = hi;
            } else {
                const uint32_t stage = __builtin_amdgcn_readfirstlane(s_deq4);
                drained = stage != 0u;
                bool empty = stage == 2u;
                if (!drained) {
                    const uint32_t dealt = ((gridDim.x - seg + a.nseg - 1u) / a.nseg) * 4u * a.chunk;
                    if (w.hl == 0) base = atomicAdd(a.heads + seg * kHeadStride, a.chunk);
                    base = lo + dealt + half_first4(w, base);
                    end = hi;
                    drained = base >= hi;
                }
                if (drained && !empty) {
                    if (w.hl == 0) base = atomicAdd(a.heads + kHeads * kHeadStride, a.tail_chunk);
                    base = a.tail0 + half_first4(w, base);
                    end = (uint32_t)a.n;
                    empty = base >= end;
                }
                if (empty) base = (uint32_t)a.n;
                if (w.hl == 0) atomicMax(&s_deq4, empty ? 2u : (drained ? 1u : 0u));
            }
            b.bidx = min(base, (uint32_t)a.n);
            b.bend = min(base + (drained ? a.tail_chunk : a.chunk), end);
            b.active = drained ? 2u : 0u;
#if SDK_SOLVE4_TIMELINE
            if (w.hl == 0 && b.bidx < b.bend) TL4(2);
#endif
        } else {
            uint32_t base = 0;
            if (w.hl == 0) base = atomicAdd(a.next, a.chunk);
            base = half_first4(w, base);
            b.bidx = base;
            b.bend = (uint32_t)min((uint64_t)base + a.chunk, a.n);
        }
    }
    b.active = (b.active & 2u) | ((uint64_t)b.bidx < a.n ? 1u : 0u);
    b.order = (a.order == ORDER_LEX && !a.count_mode) ? ORDER_LEX : ORDER_MRV;
    b.lim = a.count_mode ? a.count_lim : (b.order == ORDER_LEX ? 1u : 2u);
    b.nodes = 0;
    b.maxd = 0;
    b.rstart = a.iter;
    if (b.active & 1u) {
        start_board4<HI>(w, a, b, c, true);
    } else {
        c.x0 = setfld<HI>(c.x0, 0u);
        c.x1 = setfld<HI>(c.x1, 0u);
        c.x2 = setfld<HI>(c.x2, 0u);
        c.s0 = setfld<HI>(c.s0, kInert4);
        c.s1 = setfld<HI>(c.s1, kInert4);
        c.s2 = setfld<HI>(c.s2, kInert4);
    }
    if (FR) {
        // statics pending: the board's first round derives them (unit4f); an empty slot is inert
        // (not exact, no duplicated digit), which is what statics4 would give it
        c.E = setfld<HI>(c.E, (b.active & 1u) ? kFresh4 : 0u);
        c.D = setfld<HI>(c.D, kCands);
    } else {
        statics4<HI>(wr, c);   // the loop lane's LDS addresses: the round's, live anyway
    }
}

template <bool DN, int HI, bool FS = false>
__device__ __forceinline__ void finish_board4(const Lane4& w, const Lane4& wr, const Args4& a, Slot4& b, Cells4& c,
                                              int st) {
    if (DN) {
        SlotDn* pd = s_dn4 + w.half * 2 + HI;
        const SlotDn d = *pd;
        if (d.rec != kDnNone) {       // a part of a donating board: bookkeeping after the step
            if (w.hl == 0) {
                const int k = w.half * 2 + HI;
                s_dnfin4[k] = DnFin{d.rec, d.part, st, b.maxd,
                                    (unsigned long long)(a.work_rounds == 1 ? (uint64_t)(a.iter - b.rstart) : b.nodes)};
                atomicOr(&s_dnpend4, 1u << k);
                *pd = SlotDn{kDnNone, kDnOwner, 0u, 0u};
            }
            next_board4<HI, kFresh4Round && !DN>(w, wr, a, b, c);
            return;
        }
    }
    // an exhaustive donation launch re-solves its undecided boards in LEX (see dn_finalize4)
    if (DN && a.order != ORDER_LEX && st == -2) st = kDnRetryLex;
    uint8_t* dst = a.out + (uint64_t)b.bidx * 81;
    if (a.count_mode && w.hl == 0 && st != -2 && b.count)
        atomicAdd(&s_count4, (unsigned long long)b.count);
    if (st != 1 && w.act && a.out && !SDK_SOLVE4_NO_OUTPUT) {  // the reference restores the grid (DHT_Node.py:535)
        const uint8_t* sin = w.s_in + HI * 81;
        dst[w.c0] = sin[w.c0];
        dst[w.c0 + 27] = sin[w.c0 + 27];
        dst[w.c0 + 54] = sin[w.c0 + 54];
    }
    if (FS && w.hl == 0 && (st == 1 || st == -2))   // boards above this one cannot matter any more
        atomicMin(s_found4, (long long)(a.in_first + (uint64_t)b.bidx * a.in_step));
    if (w.hl == 0) {
        a.status[b.bidx] = (int8_t)st;
        if (a.work)
            a.work[b.bidx] = a.work_rounds == 1 ? (uint64_t)(a.iter - b.rstart)
                                                : (a.work_rounds == 2 ? (uint64_t)b.maxd : b.nodes);
        if (DN) atomicAdd(&a.dn->x[blockIdx.x % kDnXcds].done, 1u);   // a board that never donated
    }
    next_board4<HI, kFresh4Round && !DN>(w, wr, a, b, c);
}

__device__ __forceinline__ uint32_t branch_key4(uint32_t x, uint32_t s, int cell, int order) {
    if (x == 0u) return ~0u;
    const uint32_t base = ((uint32_t)cell << 9) | x;
    return order == ORDER_LEX ? base : (((uint32_t)__popc(x)) << 16) | base;
}

// LEX branch cell of each half without a cross-lane reduction: lane j < 27 owns
// cells j, j + 27, j + 54, so the lowest open cell is the first lane whose first
// cell is open, else the first whose second is, else the first whose third is --
// three ballots and scalar bit scans; its candidates come back by v_readlane.
// (Spare lanes' cells are never open.)  Out: the cell and its candidate mask for
// the lane's half; a half outside EXEC gets junk nobody reads.
__device__ __forceinline__ void lex_pick4(const Lane4& w, uint32_t x0, uint32_t x1, uint32_t x2, int& cell,
                                          uint32_t& m) {
    const uint64_t o0 = __builtin_amdgcn_ballot_w64(x0 != 0u);
    const uint64_t o1 = __builtin_amdgcn_ballot_w64(x1 != 0u);
    const uint64_t o2 = __builtin_amdgcn_ballot_w64(x2 != 0u);
    uint32_t cl[2], ml[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        uint32_t a0 = (uint32_t)(o0 >> (32 * h)), a1 = (uint32_t)(o1 >> (32 * h)), a2 = (uint32_t)(o2 >> (32 * h));
        // keep the halves 32-bit scalars: left alone, clang tests "high half != 0" as a 64-bit
        // VALU compare against a constant it then holds in a VGPR pair for the whole kernel
        asm("" : "+s"(a0), "+s"(a1), "+s"(a2));
        if (a0 != 0u) {
            const uint32_t l = __builtin_ctz(a0);
            cl[h] = l;
            ml[h] = __builtin_amdgcn_readlane(x0, 32 * h + l);
        } else if (a1 != 0u) {
            const uint32_t l = __builtin_ctz(a1);
            cl[h] = 27 + l;
            ml[h] = __builtin_amdgcn_readlane(x1, 32 * h + l);
        } else {
            const uint32_t l = a2 != 0u ? __builtin_ctz(a2) : 0u;
            cl[h] = 54 + l;
            ml[h] = __builtin_amdgcn_readlane(x2, 32 * h + l);
        }
    }
    cell = (int)(w.half ? cl[1] : cl[0]);
    m = w.half ? ml[1] : ml[0];
}

// branch-free (selects): see solve2's set_cell2 on guarded updates of the three cells
template <int HI>
__device__ __forceinline__ void set_cell4(const Lane4& w, Cells4& c, int cell, uint32_t d) {
    const bool k0 = w.act && cell == w.c0, k1 = w.act && cell == w.c0 + 27, k2 = w.act && cell == w.c0 + 54;
    c.x0 = k0 ? setfld<HI>(c.x0, 0u) : c.x0;
    c.s0 = k0 ? setfld<HI>(c.s0, d) : c.s0;
    c.x1 = k1 ? setfld<HI>(c.x1, 0u) : c.x1;
    c.s1 = k1 ? setfld<HI>(c.s1, d) : c.s1;
    c.x2 = k2 ? setfld<HI>(c.x2, 0u) : c.x2;
    c.s2 = k2 ? setfld<HI>(c.s2, d) : c.s2;
}

// Split phase of a phased solve: a board that reaches the split budget leaves its DFS stack
// (levels 0..depth-1, its half's 32 lane words each) for the donation phase, which resumes
// it (see DnSeed).  Only boards the donation kernel could split (every unit exact), searched
// in the launch's own order, with no completion met yet and at most kSaveLv levels; the
// others restart there.
template <int HI>
__device__ __forceinline__ void split_save4(const Lane4& w, const Args4& a, const Slot4& b, const Cells4& c,
                                            const uint2* g_stk) {
    if (kLds4Levels != 0 || b.count != 0u || b.depth == 0u || b.depth > kSaveLv) return;
    if (b.order != (a.order == ORDER_LEX ? (uint32_t)ORDER_LEX : (uint32_t)ORDER_MRV)) return;
    if (half_any4(w, w.act && fld<HI>(c.E) == 0u)) return;
    SplitSave* sv = s_save4.save;
    uint32_t e = 0;
    if (w.hl == 0) e = atomicAdd(&sv->count, 1u);
    e = half_first4(w, e);
    if (e >= kSaveCap) return;
#pragma unroll
    for (uint32_t l = 0; l < kSaveLv; ++l)
        if (l < b.depth) sv->lv[e][l][w.hl] = g_stk[(l * 2 + HI) * 64 + w.lane];
    if (w.hl == 0) {
        sv->hdr[e] = make_uint2(b.bidx, b.depth);
        s_save4.save_idx[b.bidx] = e;
    }
}

// the search step of the board in slot HI after its round ended (bad: contradiction)
// DFS level record: every lane keeps the level's branch record -- cell | untried
// digits << 7, uniform in the half -- in the free upper 16 bits of its own snapshot
// word y, so a level is one 8-byte word per lane and needs no shared record array.
template <bool DN, int HI, bool SV = false, bool FS = false>
__device__ __forceinline__ void step4_body(const Lane4& w, const Lane4& wr, const Args4& a, Slot4& b, Cells4& c, bool bad,
                                           uint2 (*s_stk)[2][64], uint2* g_stk) {
    ++b.nodes;
    SlotDn dd = SlotDn{kDnNone, kDnOwner, 0u, 0u};
    if (DN) {
        dd = s_dn4[w.half * 2 + HI];
        if (dd.plen & kDnAbort) {     // pruned by dn_check4
            PROF4(3, finish_board4<DN, HI, FS>(w, wr, a, b, c, kDnPruned));
            return;
        }
        // every kDnEvery nodes of a LEX solve: prune / donate check after the step (dn_check4)
        if ((b.nodes & (kDnEvery - 1u)) == 0u && b.order == (a.order == ORDER_LEX ? ORDER_LEX : ORDER_MRV) &&
            !a.count_mode && w.hl == 0)
            atomicOr(&s_dnpend4, 16u << (w.half * 2 + HI));
    }
    if (FS && (b.nodes & (kFsEvery - 1u)) == 1u) {
        // first-solution scan: stop a board that lies above the lowest hit of the launch (an
        // agent-scope load: the found word is lowered by atomics from every XCD)
        bool above = false;
        if (w.hl == 0)
            above = (long long)(a.in_first + (uint64_t)b.bidx * a.in_step) >
                    __hip_atomic_load(s_found4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (half_any4(w, above)) {
            PROF4(3, finish_board4<DN, HI, FS>(w, wr, a, b, c, kStCancelled));
            return;
        }
    }
    const uint32_t x0 = fld<HI>(c.x0), x1 = fld<HI>(c.x1), x2 = fld<HI>(c.x2);
    const uint32_t s0 = fld<HI>(c.s0), s1 = fld<HI>(c.s1), s2 = fld<HI>(c.s2);
    int r = bad ? P_CONTRA
                : (half_any4(w, w.act && (x0 | x1 | x2) != 0u) ? P_OPEN : P_SOLVED);
    if (a.budget && b.nodes > a.budget) {
        if (SV) split_save4<HI>(w, a, b, c, g_stk);
        PROF4(3, finish_board4<DN, HI, FS>(w, wr, a, b, c, -2));
        return;
    }
    if (r == P_SOLVED) {
        ++b.count;
        if (DN && dd.rec != kDnNone) {
            // a part of a donating board (exact: every closed cell holds a digit): its own
            // completion store, the board's answer is chosen when its last part ends
            DnRec* rr = dn_recs4(a) + dd.rec;
            if (b.count == 1 && w.act) {
                uint8_t* dst = const_cast<uint8_t*>(dn_sol4(a, rr, dd.part));
                dst[w.c0] = (uint8_t)__ffs(s0);
                dst[w.c0 + 27] = (uint8_t)__ffs(s1);
                dst[w.c0 + 54] = (uint8_t)__ffs(s2);
            }
            if (b.order == ORDER_MRV) {
                // exhaustive mode: the board's completions are summed over its parts
                uint32_t old = 0;
                if (w.hl == 0) {
                    old = atomicAdd(&rr->total, 1u);
                    if (old == 0u) __hip_atomic_store(&rr->first, dd.part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                old = half_first4(w, old);
                if (old == 0u) {
                    r = P_CONTRA;             // the first: search on for a second one
                    goto backtrack;
                }
            }
            PROF4(3, finish_board4<DN, HI, FS>(w, wr, a, b, c, 1));   // LEX: the region's first
            return;
        } else if (b.count == 1 && w.act && a.out && !SDK_SOLVE4_NO_OUTPUT) {
            uint8_t* dst = a.out + (uint64_t)b.bidx * 81;
            const uint8_t* sin = w.s_in + HI * 81;
            const uint32_t i0 = sin[w.c0], i1 = sin[w.c0 + 27], i2 = sin[w.c0 + 54];
            dst[w.c0] = (uint8_t)(i0 == 0 ? (uint32_t)__ffs(s0) : i0);
            dst[w.c0 + 27] = (uint8_t)(i1 == 0 ? (uint32_t)__ffs(s1) : i1);
            dst[w.c0 + 54] = (uint8_t)(i2 == 0 ? (uint32_t)__ffs(s2) : i2);
        }
        if (b.count >= b.lim && a.count_mode && !a.count_stop) {
            // 2^31 completions on one board: move all but one to the total and go on
            if (w.hl == 0) atomicAdd(&s_count4, (unsigned long long)(b.count - 1u));
            b.count = 1;
        } else if (b.count >= b.lim) {
            if (b.order == ORDER_MRV && !a.count_mode) {      // >= 2 completions: lex re-search
                b.order = ORDER_LEX;
                b.lim = 1;
                start_board4<HI>(w, a, b, c, false);
            } else {                                           // found, or the count limit
                PROF4(3, finish_board4<DN, HI, FS>(w, wr, a, b, c, 1));
            }
            return;
        }
        r = P_CONTRA;
    }
    if (r == P_OPEN) {
        bool lc = false;
        if (a.locked == 2 || (a.locked == 1 && b.depth == 0)) PROF4(4, lc = lc4<HI>(w, c));
        if (lc) {                           // candidates removed: same node, propagate again
            --b.nodes;
            return;
        }
#if SDK_SOLVE4_PROFILE
        const uint64_t tb_ = __builtin_amdgcn_s_memtime();
#endif
        int cell;
        uint32_t m;
        if (b.order == ORDER_LEX) {
            lex_pick4(w, x0, x1, x2, cell, m);
        } else {
            uint32_t key = ~0u;
            if (w.act)
                key = min(branch_key4(x0, s0, w.c0, b.order),
                          min(branch_key4(x1, s1, w.c0 + 27, b.order), branch_key4(x2, s2, w.c0 + 54, b.order)));
            key = half_min(key);
            cell = (int)((key >> 9) & 0x7Fu);
            m = key & kCands;
        }
        const uint32_t d = m & (0u - m);
        const uint2 snap = make_uint2(snap4(x0, s0) | (snap4(x1, s1) << 16),
                                      snap4(x2, s2) | (((uint32_t)cell | ((m ^ d) << 7)) << 16));
        if (b.depth < kLds4Levels) s_stk[b.depth][HI][w.lane] = snap;
        else g_stk[(b.depth * 2 + HI) * 64 + w.lane] = snap;
        ++b.depth;
        b.maxd = max(b.maxd, b.depth);
        set_cell4<HI>(w, c, cell, d);
#if SDK_SOLVE4_PROFILE
        prof4_add(6, __builtin_amdgcn_s_memtime() - tb_);
#endif
        return;
    }
backtrack:
    // contradiction: resume the deepest level with untried digits (a donating part: levels
    // below its first live one were given away)
    if (b.depth == (DN ? dd.base : 0u)) {
        PROF4(3, finish_board4<DN, HI, FS>(w, wr, a, b, c, b.count > 0 ? 1 : 0));
        return;
    }
#if SDK_SOLVE4_PROFILE
    const uint64_t tk_ = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t lvl = b.depth - 1;
    const uint2 snap = lvl < kLds4Levels ? s_stk[lvl][HI][w.lane] : g_stk[(lvl * 2 + HI) * 64 + w.lane];
    const uint32_t rec = snap.y >> 16;
    const int cell = (int)(rec & 0x7Fu);
    uint32_t rest = rec >> 7;
    const uint32_t d = rest & (0u - rest);
    rest ^= d;
    const uint32_t y0 = snap.x & 0xFFFFu, y1 = snap.x >> 16, y2 = snap.y & 0xFFFFu;
    c.x0 = setfld<HI>(c.x0, snap_x4(y0));
    c.x1 = setfld<HI>(c.x1, snap_x4(y1));
    c.x2 = setfld<HI>(c.x2, snap_x4(y2));
    c.s0 = setfld<HI>(c.s0, snap_s4(y0));
    c.s1 = setfld<HI>(c.s1, snap_s4(y1));
    c.s2 = setfld<HI>(c.s2, snap_s4(y2));
    if (rest == 0) {
        --b.depth;
    } else {
        const uint32_t y = y2 | (((uint32_t)cell | (rest << 7)) << 16);
        if (lvl < kLds4Levels) s_stk[lvl][HI][w.lane].y = y;
        else g_stk[(lvl * 2 + HI) * 64 + w.lane].y = y;
    }
    set_cell4<HI>(w, c, cell, d);
#if SDK_SOLVE4_PROFILE
    prof4_add(5, __builtin_amdgcn_s_memtime() - tk_);
#endif
}

// step of slot HI: its state comes from and returns to LDS; returns whether the slot is active
template <bool DN, int HI, bool SV = false, bool FS = false>
__device__ __forceinline__ bool step4(const Lane4& wr, const Args4& a, Cells4& c, bool bad, uint2 (*s_stk)[2][64],
                                      uint2* g_stk_all, Slot4* s_slot, uint2* s_region, uint8_t* s_in) {
    const Lane4 w = lane4_fresh(s_region, s_in);
    uint2* g_stk = g_stk_all + (size_t)blockIdx.x * (kMaxDepth * 2 * 64);
    Slot4* p = s_slot + w.half * 2 + HI;
    Slot4 b;
    PROF4(1 + HI, b = *p; step4_body<DN, HI, SV, FS>(w, wr, a, b, c, bad, s_stk, g_stk); if (w.hl == 0) *p = b);
    return (b.active & 1u) != 0u;
}

// first board of slot HI (all lanes)
template <bool DN, int HI>
__device__ __forceinline__ bool first_board4(const Lane4& w, const Args4& a, Cells4& c, Slot4* s_slot) {
    Slot4 b;
    b.bidx = 0xFFFFFFFFu;   // ++ -> 0 >= bend = 0: first dequeue
    b.bend = 0;
    b.active = 0;
    b.depth = 0;
    b.count = 0;
    next_board4<HI, kFresh4Round && !DN>(w, w, a, b, c);
    if (w.hl == 0) s_slot[w.half * 2 + HI] = b;
    return (b.active & 1u) != 0u;
}

#ifdef SDK_DEFINE_SOLVE4_KERNEL   // defined in solve4_launch.hip only
// DN: subtree donation (see "subtree donation" above); solve4_kernel<false> is the plain kernel
#ifndef SDK_SOLVE4_DN_WAVES_PER_EU
// the donation kernel runs only the launch tail (few boards, mostly idle helper waves): 96
// VGPRs at 5 waves per SIMD keep its round free of scratch reloads (at 6: 48 B/lane spilled)
#define SDK_SOLVE4_DN_WAVES_PER_EU 5
#endif
// SV: the split phase of a phased solve (split_save4); FS: a first-solution scan of a lex frontier
// (boards above the lowest hit are cancelled, see s_found4)
template <bool DN, bool SV = false, bool FS = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DN ? SDK_SOLVE4_DN_WAVES_PER_EU : SDK_SOLVE4_WAVES_PER_EU))) void solve4_kernel(SolveArgs args) {
    // the donation phases are enqueued without the host: their board count comes from the
    // device (the list the previous phase left), and the launch is the full resident grid, of
    // which 64 + SDK_OPT_DONATE_HELPERS (default 2) waves per board take part (a few tail boards do not need thousands of
    // idle waves registering and polling; none when nothing was listed)
    // dn_donate4 reads and rewrites a donated level in the global stack
    static_assert(!DN || kLds4Levels == 0, "subtree donation needs every DFS level in the global stack");
    uint64_t n = args.n;
    uint32_t grid = gridDim.x;
    uint32_t resumed = 0;
    if constexpr (DN) {
        // boards to restart (the list) and resumed boards (seeded before the launch)
        DnCtl* dn = static_cast<DnCtl*>(args.donate);
        if (args.n_dev) n = min<uint64_t>(*args.n_dev, args.n);
        resumed = ld_agent(&dn->seed.boards);
        // the waves the boards fill (four per wave) and the helpers: SDK_OPT_DONATE_HELPERS per board
        // for the first kDnHelpCap boards (a long list is mostly light boards: more idle waves only
        // slow the donors with their polls)
        const uint64_t nb = n + resumed;
        grid = (uint32_t)min<uint64_t>(gridDim.x, (nb + 3) / 4 + 64ull +
                                                      (uint64_t)ld_agent(&dn->helpers) * min<uint64_t>(nb, kDnHelpCap));
        if (n + resumed == 0 || blockIdx.x >= grid) return;
    } else if (args.n_dev) {
        // a prop32 fallback batch: its length is the list the propagation pass left
        n = min<uint64_t>(*args.n_dev, args.n);
        if (n == 0) return;
    }
    const uint64_t budget = (args.budget_big && n > kBudgetBigBoards) ? args.budget_big : args.budget;
    __shared__ uint2 s_region[2 * kRegion4];
    __shared__ uint8_t s_in[2 * 2 * 81];
    __shared__ uint2 s_stk[kLds4Levels > 0 ? kLds4Levels : 1][2][64];   // unused when kLds4Levels = 0
    Slot4* const s_slot = s_slot4;
    Lane4 w;
    init_lane4(w, s_region, s_in);
    if (threadIdx.x == 0) {
        s_deq4 = 0u;
        s_count4 = 0ull;
    }
#if SDK_SOLVE4_PROFILE
    if (threadIdx.x < 10) s_prof4[threadIdx.x] = 0;
    __syncthreads();
#endif
    uint2* g_stk = reinterpret_cast<uint2*>(args.stack);   // the steps add this workgroup's offset
    Args4 a;
    a.in = args.in;
    a.in_first = args.in_first;
    a.in_step = args.in_step;
    a.mask = args.mask;
    a.next = args.next;
    a.chunk = args.chunk;
    a.n = n;
    a.order = args.order;
    a.out = args.out;
    a.status = args.status;
    a.work = args.work;
    a.work_rounds = args.work_rounds;
    a.budget = budget;
    a.iter = 0;
    a.locked = args.locked;
    a.heads = args.heads;
    a.count_mode = args.count_mode;
    a.count_stop = args.count_mode && args.limit && args.limit < 0x80000000ull;
    a.count_lim = a.count_stop ? (uint32_t)args.limit : 0x80000000u;
    a.count = args.count;
    a.dn = static_cast<DnCtl*>(args.donate);
    if (DN && threadIdx.x < 4) s_dn4[threadIdx.x] = SlotDn{kDnNone, kDnOwner, 0u, 0u};
    if (DN && threadIdx.x == 0) {
        s_dnpend4 = 0u;
        s_dnseedn4 = ld_agent(&a.dn->seed.total);
        s_dnwave4 = s_dnseedn4 == 0u ? 4u : 0u;
        s_dntarget4 = (uint32_t)n + resumed;
        s_dnepoch4 = ld_agent(&a.dn->epoch);
        s_dnfault4 = ld_agent(&a.dn->fault);
        s_dngrid4 = grid;
        if (blockIdx.x == 0) a.dn->started = grid;    // diagnostics: the waves taking part
    }
    {   // segments share the first n - n/128 boards (rounded to whole chunks); the rest is the tail
        a.tail_chunk = max(1u, args.chunk / SDK_SOLVE4_TAIL_CHUNK_DIV);
        const uint64_t tail = ((n / SDK_SOLVE4_TAIL_DIV + args.chunk - 1) / args.chunk) * args.chunk;
        a.tail0 = (uint32_t)(n - min<uint64_t>(tail, n));
        // every segment needs a workgroup that drains it: fewer segments on a small grid
        a.nseg = min<uint32_t>(kHeads, grid);
        a.seg_size = (a.tail0 + a.nseg - 1) / a.nseg;
        if (SV && threadIdx.x == 0) s_save4 = SaveP4{static_cast<SplitSave*>(args.save), args.save_idx};
        if (FS && threadIdx.x == 0) s_found4 = args.found;
    }

    Cells4 c;
    c.x0 = c.x1 = c.x2 = 0u;
    c.s0 = c.s1 = c.s2 = kInert4x2;
    c.D = kC2;
    c.E = 0;
    if (threadIdx.x == 0) TL4(0);
    const bool act0 = first_board4<DN, 0>(w, a, c, s_slot);
    const bool act1 = first_board4<DN, 1>(w, a, c, s_slot);
    if (threadIdx.x == 0) TL4(1);

    // Event detection in scalar registers: one ballot per (flag, slot), each spread
    // to the 32 lanes of the half it came from; a slot's board takes its search step
    // when it contradicted (B) or nothing changed (no C) in its half.  A* = halves
    // whose slot still has a board.
    uint64_t A0 = __builtin_amdgcn_ballot_w64(act0), A1 = __builtin_amdgcn_ballot_w64(act1);
#if SDK_SOLVE4_PROFILE
    const uint64_t tl_ = __builtin_amdgcn_s_memtime();
#endif
    for (;;) {
        if ((A0 | A1) == 0) {
            if (!DN) break;
            // every slot idle: take a donated item, or leave once the whole grid is idle
            const int r = dn_idle4(lane4_fresh(s_region, s_in), a, c, A0, s_slot);
            if (r == 0) break;
            if (r == 1) continue;
        }
        uint32_t badw, chg;
        // every board of the wave exact (an inactive slot is not): the shorter round
        if (a.locked && __builtin_amdgcn_ballot_w64(c.E != kC2) == 0)
            PROF4(0, round4<true>(w, c, badw, chg));
        else   // kFresh4Round: also the rounds of waves with a board that just started
            PROF4(0, (round4<false, kFresh4Round && !DN>(w, c, badw, chg)));
        ++a.iter;
        const uint64_t B0 = spread_halves(__builtin_amdgcn_ballot_w64((badw & 0xFFFFu) != 0u));
        const uint64_t B1 = spread_halves(__builtin_amdgcn_ballot_w64(badw > 0xFFFFu));
        const uint64_t C0 = spread_halves(__builtin_amdgcn_ballot_w64((chg & 0xFFFFu) != 0u));
        const uint64_t C1 = spread_halves(__builtin_amdgcn_ballot_w64(chg > 0xFFFFu));
        const uint64_t E0 = A0 & (B0 | ~C0), E1 = A1 & (B1 | ~C1);
        if (E0 != 0) {
            bool r = false;
            if (__builtin_amdgcn_inverse_ballot_w64(E0))
                r = step4<DN, 0, SV, FS>(w, a, c, __builtin_amdgcn_inverse_ballot_w64(B0), s_stk, g_stk, s_slot, s_region, s_in);
            A0 = (A0 & ~E0) | (__builtin_amdgcn_ballot_w64(r) & E0);
        }
        if (E1 != 0) {
            bool r = false;
            if (__builtin_amdgcn_inverse_ballot_w64(E1))
                r = step4<DN, 1, SV, FS>(w, a, c, __builtin_amdgcn_inverse_ballot_w64(B1), s_stk, g_stk, s_slot, s_region, s_in);
            A1 = (A1 & ~E1) | (__builtin_amdgcn_ballot_w64(r) & E1);
        }
        if (DN && (E0 | E1) != 0) {
            // after the steps: bookkeeping of parts that ended, donation / pruning checks
            const uint32_t pend = __builtin_amdgcn_readfirstlane(s_dnpend4);
            if (pend != 0u) {
                const Lane4 wf = lane4_fresh(s_region, s_in);
                uint2* g_wg = g_stk + (size_t)blockIdx.x * (kMaxDepth * 2 * 64);
#pragma nounroll
                for (uint32_t k = 0; k < 4; ++k) {
                    if (!((pend >> k) & 0x11u)) continue;
                    if (wf.half == (int)(k >> 1)) {
                        if ((pend >> k) & 1u) dn_finish_part4(wf, a, s_dnfin4[k]);
                        if ((pend >> (4 + k)) & 1u) dn_check4(wf, a, c, k, s_slot, g_wg);
                    }
                }
                if (threadIdx.x == 0) s_dnpend4 = 0u;
            }
        }
    }
    if (a.count_mode && threadIdx.x == 0) {
        const unsigned long long n = s_count4;
        if (n) atomicAdd(a.count, n);
    }
#if SDK_SOLVE4_PROFILE
    prof4_add(8, __builtin_amdgcn_s_memtime() - tl_);
    prof4_add(9, a.iter);
    __syncthreads();
    if (threadIdx.x < 10) atomicAdd(&g_prof4[threadIdx.x], s_prof4[threadIdx.x]);
#endif
    if (threadIdx.x == 0) TL4(3);
}
#endif  // SDK_DEFINE_SOLVE4_KERNEL

}  // namespace sdk
