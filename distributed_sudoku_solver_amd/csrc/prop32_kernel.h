// prop32_kernel.h -- root propagation of 32 boards per half-wave, bit-sliced: the QUAD solver's
// first pass over a batch ("prop32").
//
// What it decides.  The reference solves every board by depth-first search (DHT_Node.py:512-535,
// `solve_sudoku`); a board whose constraint propagation alone -- naked and hidden singles, pointing
// and claiming (locked candidates) -- fills every cell has exactly one completion, so every
// search order returns it: status 1 and that grid.  One that propagation refutes has none: status 0
// and the input grid back (DHT_Node.py:535).  Everything else -- a board propagation leaves open,
// a board with a duplicated or out-of-domain given (whose units are not "exact", see solve4_kernel.h
// unit4x), a board still changing after max_steps -- is left undecided (kStUndecided): it goes to
// the fallback list -- with its propagated grid when the caller set no node budget (handover), else
// its input -- solve4_kernel searches it, and its answer is scattered back (sudoku_hip.hip,
// launch_prop32_solve).  On the 17-clue workload of the headline metric
// every board is decided here (tools/lockstep_model.py: all of 2,048 solved by propagation).
//
// Layout.  Bit b of a 32-bit word is board b of the half's group of 32 (board base + 32 * half + b).
// Lane hl < 27 of a half owns row triad hl -- cells 3 hl .. 3 hl + 2, one row, one box -- with nine
// candidate words per cell (c[k][d], bit b set: digit d + 1 is still possible in that cell of board
// b) and unit hl (rows 0-8, columns 9-17, boxes 18-26).  A triad's cells share their row and box, so
// the cell update reads five unit records, not seven, and the locked-candidates pass has the
// presence and eliminations of the lane's own row triad in registers.  A cell is closed when exactly
// one candidate is left (its single word s[k]); no separate closed state.  Lanes 27..31 run the same
// code on spare slots (their results are masked out).
//
// One step for all 32 boards of a half:
//   singles:  s = exactly-one over the nine words, empty = no candidate, and the cell records
//             (9 candidate words + s) written to LDS;
//   unit:     the lane's unit over its nine cell records -- T (digits of its closed cells),
//             twos (digits in two or more cells), missing digits (contradiction) -- written as
//             (T_d, twos_d) pairs;
//   cells:    each cell loses the T of its three units unless closed, takes a hidden single
//             (a remaining candidate not in some unit's twos: the cell itself holds it, so that
//             unit holds it once), and "changed" is accumulated.
// After every lc_every-th step the next step's unit/cell phases are replaced by one
// locked-candidates pass over the 54 box-line triads:
//   presence P(triad) = OR of its three cells' words (closed cells included, so the pass is sound at
//   any state); claim(L,B) = P(L,B) & ~P(L,B1) & ~P(L,B2); point(L,B) = P(L,B) & ~P(L1,B) & ~P(L2,B);
//   a triad's open cells lose claim(L1,B) | claim(L2,B) | point(L,B1) | point(L,B2).
// A board whose last singles step changed nothing and whose locked-candidates pass removes nothing
// is stuck: undecided.
//
// The two halves run their groups in lock step (one instruction stream, no divergence): a wave
// takes 64 boards per dequeue and steps until no board of either half is live.
//
// The exact-unit argument of solve4_kernel.h unit4x carries over: with no duplicated and no
// out-of-domain given, a digit taken twice in a unit leaves another digit of the unit without a
// cell, so the missing-digit test refutes every such state -- a board is declared solved only when
// every cell is closed and no unit misses a digit (then each unit holds each digit once).
#pragma once
#include "solve_kernel.h"

namespace sdk {

// status of a board the propagation pass left to the search (never returned to callers)
constexpr int kStUndecided = -4;

constexpr uint32_t kP32Rec = 40;         // bytes per cell record: 9 candidate words, the single word
constexpr uint32_t kP32URec = 72;        // bytes per unit record: (T_d, twos_d), d = 0..8
constexpr uint32_t kP32TRec = 40;        // bytes per triad record: 9 words + pad
constexpr uint32_t kP32ColTri = 1280;    // the column triads' records (32 row-triad slots before)
constexpr uint32_t kP32Region = 3456;    // bytes per half: 81 cell records + the spare lanes' record 81
constexpr uint32_t kP32Table = 2 * kP32Region;   // p32_unit's read order, 40 B per lane (p32_order_table)
constexpr uint32_t kP32Lds = kP32Table + 64 * 40;
constexpr uint32_t kP32Stage = 2592;     // bytes per half of the group's boards (32 x 81)
constexpr uint32_t kP32Heads = 8;        // dequeue counters, one per XCD segment of the groups
constexpr uint32_t kP32HeadStride = 32;  // words between counters (own cache lines)

struct Prop32Args {
    const uint8_t* in;       // boards [n][81]; 16-byte aligned
    uint8_t* out;            // [n][81]; 16-byte aligned
    int8_t* status;          // [n]: 1 solved, 0 no completion, kStUndecided
    uint64_t n;
    uint32_t* heads;         // kP32Heads counters kP32HeadStride words apart (zeroed)
    uint32_t* list;          // [0] undecided boards, then their indices (list[0] zeroed)
    uint8_t* list_in;        // the undecided boards' inputs, dense, in list order
    uint32_t lc_every;       // a locked-candidates pass after step lc_first, then every lc_every-th
    uint32_t lc_first;       // step (lc_first = lc_every: after every lc_every-th step)
    uint32_t max_steps;      // boards still live after this many steps are undecided
    int handover;            // the list gets an undecided board's propagated grid (its closed cells
                             // filled in: the same completions) instead of its input; not for
                             // boards with a duplicated or out-of-domain given
    uint32_t tail_live;      // handover: from step tail_step on, a group with at most this many
    uint32_t tail_step;      // live boards hands them to the search and ends (0 = never)
};

// OR / AND over the 32 lanes of each half, result in every lane of the half: rotations inside
// each row of 16 (DPP), then the two rows of each half combined -- v_permlane16_swap (gfx950: the
// odd rows of one register trade places with the even rows of another; on two copies of x the OR
// of both is row 0 | row 1 in each half), a VALU op, where the ds_swizzle it replaces (lane ^ 16)
// went through the LDS pipe that bounds the kernel.  Every lane of the wave must be active.
#ifndef SDK_PROP32_PERMLANE
#define SDK_PROP32_PERMLANE 1
#endif
__device__ __forceinline__ uint32_t p32_half_or(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x121, 0xF, 0xF, false);   // row_ror:1
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x122, 0xF, 0xF, false);   // row_ror:2
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, false);   // row_ror:4
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);   // row_ror:8
#if SDK_PROP32_PERMLANE
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return r[0] | r[1];
#else
    x |= (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);
    return x;
#endif
}
__device__ __forceinline__ uint32_t p32_half_and(uint32_t x) { return ~p32_half_or(~x); }

// one v_bitop3_b32 with truth table TT over (S0 = a, S1 = b, S2 = c).  Left to itself the compiler
// forms three-input ORs as v_or3_b32, which issues at ~0.6x the rate of v_bitop3_b32
// (solve_kernel.h SDK_OR3); the locked-candidates pass states its algebra through this.
template <unsigned TT>
__device__ __forceinline__ uint32_t p32_b3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(b), "v"(c), "i"(TT));
    return r;
}
constexpr unsigned kB3Or3 = 0xFEu;       // S0 | S1 | S2
constexpr unsigned kB3AndNor = 0x10u;    // S0 & ~(S1 | S2)

// LDS access through address-space-3 pointers (ds_* instructions); loads are volatile so the
// compiler keeps them single ds_read_b64 (a ds_read2_b64 pair costs 8 LDS-array cycles against
// 2 x 2, MI355X_MICROARCH.md LDS table)
typedef __attribute__((address_space(3))) uint8_t p32_lds_t;
typedef unsigned int p32_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 p32_ld(p32_lds_t* base, uint32_t off) {
    const uint64_t v = *(const volatile __attribute__((address_space(3))) uint64_t*)(base + off);
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
__device__ __forceinline__ uint2 p32_lda(uint32_t addr) {   // an absolute LDS address
    const uint64_t v = *(const volatile __attribute__((address_space(3))) uint64_t*)(uintptr_t)addr;
    return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
// stores volatile too: merged pairs become ds_write2_b64, 13 cycles against 2 x 6 (same table)
// The unit phase's per-lane read-order table (p32_order_table): SDK_PROP32_TABLE16 keeps the nine
// record addresses as 16-bit halves (three ds_read_b64 per step, halves split by VOP2 shifts and
// masks) instead of 32-bit words (five reads) -- two LDS instructions fewer per step on the pipe
// that bounds the kernel, for nine pairing VALU ops
#ifndef SDK_PROP32_TABLE16
#define SDK_PROP32_TABLE16 1
#endif
__device__ __forceinline__ uint64_t p32_tab64(const p32_lds_t* lds, uint32_t off) {
    return *(const volatile __attribute__((address_space(3))) uint64_t*)(lds + off);
}
// 16-bit field k (0..3) of a table word
__device__ __forceinline__ uint32_t p32_tab_field(uint64_t v, int k) {
    const uint32_t w = k < 2 ? (uint32_t)v : (uint32_t)(v >> 32);
    return (k & 1) ? w >> 16 : w & 0xFFFFu;
}
__device__ __forceinline__ void p32_st(p32_lds_t* base, uint32_t off, uint32_t x, uint32_t y) {
    *(volatile __attribute__((address_space(3))) uint64_t*)(base + off) = (uint64_t)x | ((uint64_t)y << 32);
}

// a copy of v the compiler cannot see through: per-lane addresses derived from it are computed
// where they are used instead of being hoisted out of the step loop (where they would hold ~20
// VGPRs for the whole kernel)
__device__ __forceinline__ uint32_t p32_opq(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

struct P32Lane {
    uint32_t half, hl;
    bool act;
    p32_lds_t* reg;        // the half's LDS region
};

struct P32Cells {
    uint32_t c[3][9];
    uint32_t s[3];
};

// singles: s = exactly one candidate, empty = none; the cell records of the real lanes (cell j at
// 40j: cells 3 hl + k at 120 hl + 40k)
__device__ __forceinline__ void p32_singles(const P32Lane& w, P32Cells& x, uint32_t& empty, uint32_t& alls) {
    empty = 0u;
    alls = ~0u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        // exactly one of nine words: "in two or more" by majorities, three words then pairs (10
        // instructions instead of the 17 of a one-word-at-a-time chain)
        const uint32_t* c = x.c[k];
        uint32_t o, w2, t1, t2, t3;
        asm(SDK_OR3("%[o]", "%[c0]", "%[c1]", "%[c2]")
            "v_bitop3_b32 %[w], %[c0], %[c1], %[c2] bitop3:0xe8\n\t"
            "v_bitop3_b32 %[t1], %[o], %[c3], %[c4] bitop3:0xe8\n\t"
            SDK_OR3("%[o]", "%[o]", "%[c3]", "%[c4]")
            "v_bitop3_b32 %[t2], %[o], %[c5], %[c6] bitop3:0xe8\n\t"
            SDK_OR3("%[o]", "%[o]", "%[c5]", "%[c6]")
            "v_bitop3_b32 %[t3], %[o], %[c7], %[c8] bitop3:0xe8\n\t"
            SDK_OR3("%[o]", "%[o]", "%[c7]", "%[c8]")
            SDK_OR3("%[w]", "%[w]", "%[t1]", "%[t2]")
            : [o] "=&v"(o), [w] "=&v"(w2), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
            : [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]), [c5] "v"(c[5]),
              [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]));
        x.s[k] = o & ~(w2 | t3);
        empty |= ~o;
        alls &= x.s[k];
    }
    // spare lanes store into record 81 (no branch: a divergent region inside the step loop cost the
    // cell words a second register home); their unit reads return whatever is there
    const uint32_t rec = kP32Rec * p32_opq(w.hl);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t o = w.act ? 3u * rec + kP32Rec * k : 81u * kP32Rec;
        p32_st(w.reg, o, x.c[k][0], x.c[k][1]);
        p32_st(w.reg, o + 8, x.c[k][2], x.c[k][3]);
        p32_st(w.reg, o + 16, x.c[k][4], x.c[k][5]);
        p32_st(w.reg, o + 24, x.c[k][6], x.c[k][7]);
        p32_st(w.reg, o + 32, x.c[k][8], x.s[k]);
    }
}

// Exact instruction sequences for the step's bit algebra (v_bitop3_b32 truth tables over S0 = 0xF0,
// S1 = 0xCC, S2 = 0xAA): left to itself the compiler splits the majority and the and-or forms into
// 3-instruction chains (7 instead of 5 per pair and digit in the unit summary).
//   unit, first three cells:  ones = a | b | c, twos = maj(a, b, c) (0xE8), T = a&sa | b&sb | c&sc
//   unit, a pair:             twos |= maj(ones, a, b), ones |= a | b, T |= a&sa | b&sb (0xF8: S0 | S1&S2)
__device__ __forceinline__ void p32_unit3(uint32_t& ones, uint32_t& twos, uint32_t& T, uint32_t a, uint32_t b,
                                          uint32_t c, uint32_t sa, uint32_t sb, uint32_t sc) {
    asm(SDK_OR3("%[o]", "%[a]", "%[b]", "%[c]")
        "v_bitop3_b32 %[w], %[a], %[b], %[c] bitop3:0xe8\n\t"
        "v_and_b32 %[t], %[a], %[sa]\n\t"
        "v_bitop3_b32 %[t], %[t], %[b], %[sb] bitop3:0xf8\n\t"
        "v_bitop3_b32 %[t], %[t], %[c], %[sc] bitop3:0xf8"
        : [o] "=&v"(ones), [w] "=&v"(twos), [t] "=&v"(T)
        : [a] "v"(a), [b] "v"(b), [c] "v"(c), [sa] "v"(sa), [sb] "v"(sb), [sc] "v"(sc));
}
__device__ __forceinline__ void p32_unit2(uint32_t& ones, uint32_t& twos, uint32_t& T, uint32_t a, uint32_t b,
                                          uint32_t sa, uint32_t sb) {
    uint32_t t;
    asm("v_bitop3_b32 %[t], %[o], %[a], %[b] bitop3:0xe8\n\t"
        SDK_OR3("%[o]", "%[o]", "%[a]", "%[b]")
        "v_or_b32 %[w], %[w], %[t]\n\t"
        "v_bitop3_b32 %[T], %[T], %[a], %[sa] bitop3:0xf8\n\t"
        "v_bitop3_b32 %[T], %[T], %[b], %[sb] bitop3:0xf8"
        : [t] "=&v"(t), [o] "+v"(ones), [w] "+v"(twos), [T] "+v"(T)
        : [a] "v"(a), [b] "v"(b), [sa] "v"(sa), [sb] "v"(sb));
}
// cell update, first pass for digit d:  U = cT|rT|bT, H = ~(cW & rW & bW) (0x7F; W = twos: a candidate of
// the cell outside some unit's twos is that unit's hidden single), c &= ~U | s (0xB0: S0 & (~S1 | S2)),
// anyh |= c & H (0xF8); with CHG, chg |= c_old & ~c_new (0xF4: S0 | S1 & ~S2)
template <bool CHG>
__device__ __forceinline__ void p32_upd1(uint32_t& c, uint32_t& H, uint32_t& anyh, uint32_t& chg, uint32_t s,
                                         uint32_t cT, uint32_t rT, uint32_t bT, uint32_t cH, uint32_t rH, uint32_t bH) {
    uint32_t U, v;
    if (CHG)
        asm(SDK_OR3("%[u]", "%[ct]", "%[rt]", "%[bt]")
            "v_bitop3_b32 %[h], %[ch], %[rh], %[bh] bitop3:0x7f\n\t"
            "v_bitop3_b32 %[v], %[c], %[u], %[s] bitop3:0xb0\n\t"
            "v_bitop3_b32 %[g], %[g], %[c], %[v] bitop3:0xf4\n\t"
            "v_bitop3_b32 %[a], %[a], %[v], %[h] bitop3:0xf8"
            : [u] "=&v"(U), [h] "=&v"(H), [v] "=&v"(v), [g] "+v"(chg), [a] "+v"(anyh)
            : [c] "v"(c), [s] "v"(s), [ct] "v"(cT), [rt] "v"(rT), [bt] "v"(bT), [ch] "v"(cH), [rh] "v"(rH),
              [bh] "v"(bH));
    else
        asm(SDK_OR3("%[u]", "%[ct]", "%[rt]", "%[bt]")
            "v_bitop3_b32 %[h], %[ch], %[rh], %[bh] bitop3:0x7f\n\t"
            "v_bitop3_b32 %[v], %[c], %[u], %[s] bitop3:0xb0\n\t"
            "v_bitop3_b32 %[a], %[a], %[v], %[h] bitop3:0xf8"
            : [u] "=&v"(U), [h] "=&v"(H), [v] "=&v"(v), [a] "+v"(anyh)
            : [c] "v"(c), [s] "v"(s), [ct] "v"(cT), [rt] "v"(rT), [bt] "v"(bT), [ch] "v"(cH), [rh] "v"(rH),
              [bh] "v"(bH));
    c = v;
}
// second pass: the hidden single, c &= H | ~anyh (0xD0: S0 & (S1 | ~S2)); with CHG the change bits
template <bool CHG>
__device__ __forceinline__ void p32_upd2(uint32_t& c, uint32_t H, uint32_t anyh, uint32_t& chg) {
    uint32_t v;
    if (CHG)
        asm("v_bitop3_b32 %[v], %[c], %[h], %[a] bitop3:0xd0\n\t"
            "v_bitop3_b32 %[g], %[g], %[c], %[v] bitop3:0xf4"
            : [v] "=&v"(v), [g] "+v"(chg)
            : [c] "v"(c), [h] "v"(H), [a] "v"(anyh));
    else
        asm("v_bitop3_b32 %[v], %[c], %[h], %[a] bitop3:0xd0" : [v] "=v"(v) : [c] "v"(c), [h] "v"(H), [a] "v"(anyh));
    c = v;
}

// the record offsets of unit j's cells (rows 0-8, columns 9-17, boxes 18-26): cell q at
// u0 + (q % 3) ua + (q / 3) ub (p32_order_table; j < 27)
__device__ __forceinline__ void p32_unit_cells(uint32_t j, uint32_t& u0, uint32_t& ua, uint32_t& ub) {
    if (j < 9) {                           // row j: cells 9j + q
        u0 = kP32Rec * 9 * j; ua = kP32Rec; ub = 3 * kP32Rec;
    } else if (j < 18) {                   // column j - 9: cells 9q + (j - 9)
        u0 = kP32Rec * (j - 9); ua = 9 * kP32Rec; ub = 27 * kP32Rec;
    } else {                               // box b: rows 3 (b / 3) + q / 3, columns 3 (b % 3) + q % 3
        const uint32_t b = j - 18;
        u0 = kP32Rec * (27 * (b / 3) + 3 * (b % 3)); ua = kP32Rec; ub = 9 * kP32Rec;
    }
}

// digits given twice in the lane's unit (a group's first step, before p32_unit: its closed cells are
// the givens); such a board is not exact and goes to the search
__device__ __forceinline__ uint32_t p32_dups(const P32Lane& w, const p32_lds_t* lds) {
    // the unit's cells from p32_unit's order table (any order will do; no lane-dependent branch)
    const uint32_t tb = kP32Table + 40u * p32_opq(threadIdx.x);
    uint32_t T[9], dup = 0u;
#if SDK_PROP32_TABLE16
    uint64_t tw = 0ull;
#endif
#pragma unroll
    for (int q = 0; q < 9; ++q) {
#if SDK_PROP32_TABLE16
        if (q % 4 == 0) tw = p32_tab64(lds, tb + 2u * q);
        const uint32_t o = p32_tab_field(tw, q % 4);
#else
        const uint32_t o = *(const volatile __attribute__((address_space(3))) uint32_t*)(lds + tb + 4u * (q < 3 ? q : q + 1));
#endif
        const uint2 r0 = p32_lda(o), r1 = p32_lda(o + 8), r2 = p32_lda(o + 16), r3 = p32_lda(o + 24),
                    r4 = p32_lda(o + 32);
        const uint32_t a[9] = {r0.x, r0.y, r1.x, r1.y, r2.x, r2.y, r3.x, r3.y, r4.x};
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            const uint32_t t = a[d] & r4.y;
            if (q == 0) {
                T[d] = t;
            } else {
                dup |= T[d] & t;
                T[d] |= t;
            }
        }
        // one cell's loads at a time (see p32_unit)
        asm volatile("" : "+v"(T[0]), "+v"(T[1]), "+v"(T[2]), "+v"(T[3]), "+v"(T[4]), "+v"(T[5]), "+v"(T[6]),
                     "+v"(T[7]), "+v"(T[8]), "+v"(dup)::"memory");
    }
    return dup;
}

// The unit summary: "in two or more cells" is accumulated two cells at a time after the first
// three -- a bit is in at least two of (ones, a, b) exactly when it is in their majority (bitop3
// 0xE8), as in solve4's unit4.
// The unit phase's read order.  Step t of every unit lane reads the cell of its unit where the fixed
// grid kP32Order holds t: kP32Order is a valid Sudoku solution, so at each step the 27 lanes read the
// same nine cells (one per row, column and box -- each by three lanes, a broadcast), and it is chosen
// so that those nine cells' records (40 B apart) fall in nine different bank pairs (cell index mod 32
// distinct in every digit class; found by a search over relabelled and permuted pattern grids).  The
// natural order met two addresses per bank pair on every read (15-16 % of the launch's LDS cycles
// were bank conflicts).  The per-lane offsets are a table in LDS (40 B per lane; SDK_PROP32_TABLE16 above).
// kDups (a group's first step): also the digits given twice in the unit (p32_dups) from the same
// loaded records -- a digit closed in at least two of the unit's cells: the majority of three closed
// terms over the first three cells, then of (closed so far, the pair's two closed terms) -- instead of
// a second pass over the nine records
template <bool kDups>
__device__ __forceinline__ void p32_unit(const P32Lane& w, const p32_lds_t* lds, uint32_t& miss, uint32_t& dup) {
    const uint32_t j = p32_opq(w.hl);   // the unit record written below
    const uint32_t tb = kP32Table + 40u * p32_opq(threadIdx.x);
    uint32_t ones[9], twos[9], T[9];
#if SDK_PROP32_TABLE16
    uint64_t tA, tB = 0ull;   // table words: steps 0-3, 4-7 (step 8: its own read)
#endif
    // cells 0, 1, 2
    {
        uint32_t a[3][9], s[3];
#if SDK_PROP32_TABLE16
        tA = p32_tab64(lds, tb);
#else
        const uint64_t o01 = *(const volatile __attribute__((address_space(3))) uint64_t*)(lds + tb);
        const uint32_t o2 = *(const volatile __attribute__((address_space(3))) uint32_t*)(lds + tb + 8u);
#endif
#pragma unroll
        for (int q = 0; q < 3; ++q) {
#if SDK_PROP32_TABLE16
            const uint32_t o = p32_tab_field(tA, q);
#else
            const uint32_t o = q == 0 ? (uint32_t)o01 : q == 1 ? (uint32_t)(o01 >> 32) : o2;
#endif
            const uint2 r0 = p32_lda(o), r1 = p32_lda(o + 8), r2 = p32_lda(o + 16), r3 = p32_lda(o + 24),
                        r4 = p32_lda(o + 32);
            a[q][0] = r0.x; a[q][1] = r0.y; a[q][2] = r1.x; a[q][3] = r1.y; a[q][4] = r2.x;
            a[q][5] = r2.y; a[q][6] = r3.x; a[q][7] = r3.y; a[q][8] = r4.x;
            s[q] = r4.y;
        }
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            if (kDups) dup |= p32_b3<0xE8u>(a[0][d] & s[0], a[1][d] & s[1], a[2][d] & s[2]);
            p32_unit3(ones[d], twos[d], T[d], a[0][d], a[1][d], a[2][d], s[0], s[1], s[2]);
        }
    }
    // cells (3, 4), (5, 6), (7, 8): one pair's reads at a time -- the accumulators pass through the
    // empty asm after each pair, so the next pair's loads are not hoisted above this pair's
    // arithmetic (left alone the scheduler issues every load first and spills)
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        asm volatile("" : "+v"(ones[0]), "+v"(ones[1]), "+v"(ones[2]), "+v"(ones[3]), "+v"(ones[4]), "+v"(ones[5]),
                     "+v"(ones[6]), "+v"(ones[7]), "+v"(ones[8]), "+v"(twos[0]), "+v"(twos[1]), "+v"(twos[2]),
                     "+v"(twos[3]), "+v"(twos[4]), "+v"(twos[5]), "+v"(twos[6]), "+v"(twos[7]), "+v"(twos[8]),
                     "+v"(T[0]), "+v"(T[1]), "+v"(T[2]), "+v"(T[3]), "+v"(T[4]), "+v"(T[5]), "+v"(T[6]),
                     "+v"(T[7]), "+v"(T[8])::"memory");
        uint32_t a[2][9], s[2];
#if SDK_PROP32_TABLE16
        // steps 3 + 2p, 4 + 2p: (3, 4) from words A and B, (5, 6) from B, (7, 8) from B and C
        uint32_t oo[2];
        if (p == 0) {
            tB = p32_tab64(lds, tb + 8u);
            oo[0] = p32_tab_field(tA, 3);
            oo[1] = p32_tab_field(tB, 0);
        } else if (p == 1) {
            oo[0] = p32_tab_field(tB, 1);
            oo[1] = p32_tab_field(tB, 2);
        } else {
            oo[0] = p32_tab_field(tB, 3);
            oo[1] = p32_tab_field(p32_tab64(lds, tb + 16u), 0);
        }
#else
        const uint64_t op = *(const volatile __attribute__((address_space(3))) uint64_t*)(lds + tb + 16u + 8u * p);
#endif
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#if SDK_PROP32_TABLE16
            const uint32_t o = oo[h];
#else
            const uint32_t o = h == 0 ? (uint32_t)op : (uint32_t)(op >> 32);
#endif
            const uint2 r0 = p32_lda(o), r1 = p32_lda(o + 8), r2 = p32_lda(o + 16), r3 = p32_lda(o + 24),
                        r4 = p32_lda(o + 32);
            a[h][0] = r0.x; a[h][1] = r0.y; a[h][2] = r1.x; a[h][3] = r1.y; a[h][4] = r2.x;
            a[h][5] = r2.y; a[h][6] = r3.x; a[h][7] = r3.y; a[h][8] = r4.x;
            s[h] = r4.y;
        }
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            if (kDups) dup |= p32_b3<0xE8u>(T[d], a[0][d] & s[0], a[1][d] & s[1]);   // T: closed so far
            p32_unit2(ones[d], twos[d], T[d], a[0][d], a[1][d], s[0], s[1]);
        }
    }
    // a digit with no cell: the complement of the and of the nine "in some cell" words (and3 chains)
    uint32_t all;
    asm("v_bitop3_b32 %[m], %[o0], %[o1], %[o2] bitop3:0x80\n\t"
        "v_bitop3_b32 %[m], %[m], %[o3], %[o4] bitop3:0x80\n\t"
        "v_bitop3_b32 %[m], %[m], %[o5], %[o6] bitop3:0x80\n\t"
        "v_bitop3_b32 %[m], %[m], %[o7], %[o8] bitop3:0x80"
        : [m] "=&v"(all)
        : [o0] "v"(ones[0]), [o1] "v"(ones[1]), [o2] "v"(ones[2]), [o3] "v"(ones[3]), [o4] "v"(ones[4]),
          [o5] "v"(ones[5]), [o6] "v"(ones[6]), [o7] "v"(ones[7]), [o8] "v"(ones[8]));
    miss = ~all;
    __builtin_amdgcn_wave_barrier();   // every lane's reads before the records are overwritten
    const uint32_t urec = kP32URec * j;   // spare lanes: unit slots 27..31
#pragma unroll
    for (int d = 0; d < 9; ++d) p32_st(w.reg, urec + 8 * d, T[d], twos[d]);
}

// the cell update of one step; CHG: also returns the change bits of the lane's three cells (only the
// step before a locked-candidates pass needs them: a board unchanged by it and by the pass is stuck).
// The lane's cells 3j + k share row j / 3 and box 3 (j / 9) + j % 3: those two records are read once
// (36 registers for the phase), each cell's column record beside its update.
template <bool CHG>
__device__ __forceinline__ uint32_t p32_cells(const P32Lane& w, P32Cells& x) {
    const uint32_t j = p32_opq(w.hl);
    const uint32_t r = j / 3, bc = j - 3 * r;          // row r, box column bc: columns 3 bc + k
    const uint32_t rowrec = kP32URec * r, boxrec = kP32URec * (18 + 3 * (r / 3) + bc),
                   colrec = kP32URec * (9 + 3 * bc);
    uint32_t rT[9], rW[9], bT[9], bW[9];
#pragma unroll
    for (int d = 0; d < 9; ++d) {
        const uint2 v = p32_ld(w.reg, rowrec + 8 * d), u = p32_ld(w.reg, boxrec + 8 * d);
        rT[d] = v.x;
        rW[d] = v.y;
        bT[d] = u.x;
        bW[d] = u.y;
    }
    uint32_t chg = 0u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        uint32_t H[9], anyh = 0u;
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            const uint2 c = p32_ld(w.reg, colrec + kP32URec * k + 8 * d);   // column 3 bc + k
            p32_upd1<CHG>(x.c[k][d], H[d], anyh, chg, x.s[k], c.x, rT[d], bT[d], c.y, rW[d], bW[d]);
        }
#pragma unroll
        for (int d = 0; d < 9; ++d) p32_upd2<CHG>(x.c[k][d], H[d], anyh, chg);
    }
    return chg;
}

// the eliminations into the lane's triad (line tl, box index tb along the line) of one kind
// (base: the row or column triads' records): lines L1, L2 of the band / stack, boxes B1, B2
__device__ __forceinline__ void p32_elim(const P32Lane& w, uint32_t tl, uint32_t tb, uint32_t base,
                                         uint32_t (&e)[9]) {
    const uint32_t L0 = tl - tl % 3;
    const uint32_t L1 = L0 + (tl - L0 + 1) % 3, L2 = L0 + (tl - L0 + 2) % 3;
    const uint32_t B1 = (tb + 1) % 3, B2 = (tb + 2) % 3;
    const uint32_t oL1B = base + kP32TRec * (3 * L1 + tb), oL1B1 = base + kP32TRec * (3 * L1 + B1),
                   oL1B2 = base + kP32TRec * (3 * L1 + B2), oL2B = base + kP32TRec * (3 * L2 + tb),
                   oL2B1 = base + kP32TRec * (3 * L2 + B1), oL2B2 = base + kP32TRec * (3 * L2 + B2),
                   oLB1 = base + kP32TRec * (3 * tl + B1), oLB2 = base + kP32TRec * (3 * tl + B2);
#pragma unroll
    for (int h = 0; h < 5; ++h) {
        const uint2 l1b = p32_ld(w.reg, oL1B + 8 * h), l1b1 = p32_ld(w.reg, oL1B1 + 8 * h),
                    l1b2 = p32_ld(w.reg, oL1B2 + 8 * h), l2b = p32_ld(w.reg, oL2B + 8 * h),
                    l2b1 = p32_ld(w.reg, oL2B1 + 8 * h), l2b2 = p32_ld(w.reg, oL2B2 + 8 * h),
                    lb1 = p32_ld(w.reg, oLB1 + 8 * h), lb2 = p32_ld(w.reg, oLB2 + 8 * h);
        e[2 * h] = p32_b3<kB3Or3>(p32_b3<kB3AndNor>(l1b.x, l1b1.x, l1b2.x), p32_b3<kB3AndNor>(l2b.x, l2b1.x, l2b2.x),
                                  p32_b3<kB3AndNor>(lb1.x, l1b1.x, l2b1.x)) |
                   p32_b3<kB3AndNor>(lb2.x, l1b2.x, l2b2.x);
        if (h < 4)
            e[2 * h + 1] = p32_b3<kB3Or3>(p32_b3<kB3AndNor>(l1b.y, l1b1.y, l1b2.y),
                                          p32_b3<kB3AndNor>(l2b.y, l2b1.y, l2b2.y),
                                          p32_b3<kB3AndNor>(lb1.y, l1b1.y, l2b1.y)) |
                           p32_b3<kB3AndNor>(lb2.y, l1b2.y, l2b2.y);
    }
}

// one locked-candidates pass (the cell records of this step are in LDS); returns the change bits.
// Lane j < 27 owns row triad j (row j / 3, box column j % 3) -- its own three cells -- and column
// triad j (column j / 3, box row j % 3); spare lanes read triad 26's column and write their own
// slots 27..31.
__device__ __forceinline__ uint32_t p32_locked(const P32Lane& w, P32Cells& x) {
    const uint32_t j = p32_opq(w.hl), jt = min(j, 26u);
    const uint32_t tl = jt / 3, tb = jt - 3 * tl;
    const uint32_t ctri = kP32Rec * (27 * tb + tl);
    const uint32_t rtrec = kP32TRec * j, ctrec = kP32ColTri + kP32TRec * j;
    // presence of the lane's row triad (its own cells, closed ones included) and column triad
    uint32_t pr[9], pc[9];
#pragma unroll
    for (int d = 0; d < 9; ++d) pr[d] = p32_b3<kB3Or3>(x.c[0][d], x.c[1][d], x.c[2][d]);
#pragma unroll
    for (int h = 0; h < 5; ++h) {
        const uint2 b0 = p32_ld(w.reg, ctri + 8 * h), b1 = p32_ld(w.reg, ctri + 360 + 8 * h),
                    b2 = p32_ld(w.reg, ctri + 720 + 8 * h);
        pc[2 * h] = p32_b3<kB3Or3>(b0.x, b1.x, b2.x);
        if (h < 4) pc[2 * h + 1] = p32_b3<kB3Or3>(b0.y, b1.y, b2.y);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int h = 0; h < 5; ++h) {
        p32_st(w.reg, rtrec + 8 * h, pr[2 * h], h < 4 ? pr[2 * h + 1] : 0u);
        p32_st(w.reg, ctrec + 8 * h, pc[2 * h], h < 4 ? pc[2 * h + 1] : 0u);
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t er[9], ec[9];
    p32_elim(w, tl, tb, 0u, er);
    p32_elim(w, tl, tb, kP32ColTri, ec);
    __builtin_amdgcn_wave_barrier();
    // the column triads' eliminations to LDS (the row triad's are this lane's own cells')
#pragma unroll
    for (int h = 0; h < 5; ++h) p32_st(w.reg, ctrec + 8 * h, ec[2 * h], h < 4 ? ec[2 * h + 1] : 0u);
    __builtin_amdgcn_wave_barrier();
    // apply to the lane's open cells: cell 3j + k lies in column 3 (j % 3) + k, box row j / 9, so in
    // column triad 9 (j % 3) + 3k + j / 9
    const uint32_t at_c = kP32ColTri + kP32TRec * (9 * (j % 3) + j / 9);
    uint32_t chg = 0u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int h = 0; h < 5; ++h) {
            const uint2 c = p32_ld(w.reg, at_c + 3 * kP32TRec * k + 8 * h);
            {
                const uint32_t rm = (er[2 * h] | c.x) & x.c[k][2 * h] & ~x.s[k];
                chg |= rm;
                x.c[k][2 * h] ^= rm;
            }
            if (h < 4) {
                const uint32_t rm = (er[2 * h + 1] | c.y) & x.c[k][2 * h + 1] & ~x.s[k];
                chg |= rm;
                x.c[k][2 * h + 1] ^= rm;
            }
        }
    }
    return chg;
}

// One cell of the half's 32 boards, from the staging (byte of board b at col[81 b]) to its nine
// candidate words.  Per 8 boards: the 8 bytes as a 64-bit word (byte r = board r), an 8 x 8 bit
// transpose (three swap stages; Hacker's Delight 7-3) makes byte i the bit-i plane of the 8 boards,
// v_perm gathers the planes of the 32 boards, and each digit's word is its minterm over the low
// four planes (values > 9 are the inert boards, decided elsewhere), or'd with the empty cells.
__device__ __forceinline__ void p32_convert(const p32_lds_t* col, uint32_t (&c)[9]) {
    uint32_t lo[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        uint32_t l = col[81u * (8 * m)], h = col[81u * (8 * m + 4)];
#pragma unroll
        for (int r = 1; r < 4; ++r) {
            l |= (uint32_t)col[81u * (8 * m + r)] << (8 * r);
            h |= (uint32_t)col[81u * (8 * m + 4 + r)] << (8 * r);
        }
        uint32_t t;
        t = (l ^ (l >> 7)) & 0x00AA00AAu;  l ^= t ^ (t << 7);
        t = (h ^ (h >> 7)) & 0x00AA00AAu;  h ^= t ^ (t << 7);
        t = (l ^ (l >> 14)) & 0x0000CCCCu; l ^= t ^ (t << 14);
        t = (h ^ (h >> 14)) & 0x0000CCCCu; h ^= t ^ (t << 14);
        t = (l ^ (h << 4)) & 0xF0F0F0F0u;  l ^= t;       // the high word is not needed after this
        lo[m] = l;                         // byte i: plane i of boards 8m .. 8m + 7
    }
    uint32_t P[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // bytes (lo[0].i, lo[1].i) and (lo[2].i, lo[3].i); selector 0x0C = a zero byte
        const uint32_t a = __builtin_amdgcn_perm(lo[1], lo[0], 0x0C0C0400u + 0x0101u * (uint32_t)i);
        const uint32_t b = __builtin_amdgcn_perm(lo[3], lo[2], 0x04000C0Cu + 0x01010000u * (uint32_t)i);
        P[i] = a | b;
    }
    const uint32_t e = ~(P[0] | P[1] | P[2] | P[3]);        // empty cells: every digit
    const uint32_t n3 = ~P[3];
    c[0] = (P[0] & ~P[1] & ~P[2] & n3) | e;                 // 1 = 0001
    c[1] = (~P[0] & P[1] & ~P[2] & n3) | e;                 // 2 = 0010
    c[2] = (P[0] & P[1] & ~P[2] & n3) | e;                  // 3 = 0011
    c[3] = (~P[0] & ~P[1] & P[2] & n3) | e;                 // 4 = 0100
    c[4] = (P[0] & ~P[1] & P[2] & n3) | e;                  // 5 = 0101
    c[5] = (~P[0] & P[1] & P[2] & n3) | e;                  // 6 = 0110
    c[6] = (P[0] & P[1] & P[2] & n3) | e;                   // 7 = 0111
    c[7] = (P[3] & ~P[0]) | e;                              // 8 = 1000 (9 < v < 16: inert)
    c[8] = (P[3] & P[0]) | e;                               // 9 = 1001
}

// The inverse of p32_convert for one cell: the digit of each of the 32 boards (the binary planes of
// its one-hot words, gathered 8 boards at a time and bit-transposed back into bytes) into the
// staging, byte of board b at col[81 b]; 0 where the cell is open.  (Boards with a contradiction or
// an inert given get meaningless bytes.)
__device__ __forceinline__ void p32_digits(const uint32_t (&c)[9], uint32_t single, p32_lds_t* col) {
    // open cells (more than one candidate left) come out as 0
    const uint32_t Q[4] = {(c[0] | c[2] | c[4] | c[6] | c[8]) & single, (c[1] | c[2] | c[5] | c[6]) & single,
                           (c[3] | c[4] | c[5] | c[6]) & single, (c[7] | c[8]) & single};
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        // byte i: plane i of boards 8m .. 8m + 7 (the high word, planes 4..7, is zero)
        const uint32_t a = __builtin_amdgcn_perm(Q[1], Q[0], 0x0C0C0400u + 0x0101u * (uint32_t)m);
        const uint32_t b = __builtin_amdgcn_perm(Q[3], Q[2], 0x04000C0Cu + 0x01010000u * (uint32_t)m);
        uint32_t l = a | b, t;
        t = (l ^ (l >> 7)) & 0x00AA00AAu;  l ^= t ^ (t << 7);
        t = (l ^ (l >> 14)) & 0x0000CCCCu; l ^= t ^ (t << 14);
        const uint32_t h = (l >> 4) & 0x0F0F0F0Fu;   // boards 8m + 4 .. 8m + 7
        l &= 0x0F0F0F0Fu;                             // boards 8m .. 8m + 3
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            col[81u * (8 * m + r)] = (uint8_t)(l >> (8 * r));
            col[81u * (8 * m + 4 + r)] = (uint8_t)(h >> (8 * r));
        }
    }
}

// the 64-bit board mask of a half-reduced word (lane 0: boards 0..31, lane 32: boards 32..63)
__device__ __forceinline__ uint64_t p32_mask64(uint32_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// the next group of 64 boards: the home segment's counter (blockIdx % kP32Heads, one XCD), then
// the others in turn.  Returns the group index or ~0u.
__device__ __forceinline__ uint32_t p32_dequeue(const Prop32Args& a, uint32_t groups, uint32_t& seg) {
    const uint32_t per = (groups + kP32Heads - 1) / kP32Heads;
    for (uint32_t t = 0; t < kP32Heads; ++t) {
        const uint32_t sg = (seg + t) % kP32Heads;
        const uint32_t lo = sg * per, hi = min(lo + per, groups);
        if (lo >= hi) continue;
        uint32_t g = 0;
        if (threadIdx.x == 0) {
            // a drained segment: one plain read instead of an atomic that only counts further
            g = __hip_atomic_load(a.heads + sg * kP32HeadStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (lo + g < hi) g = atomicAdd(a.heads + sg * kP32HeadStride, 1u);
        }
        g = lo + (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
        if (g < hi) {
            seg = sg;
            return g;
        }
    }
    return ~0u;
}

// SDK_PROP32_STATS (profiling builds only): per group, histograms of the steps it ran, of the step at
// which at most 4 / at most 1 of its boards were still live, and the locked-candidates passes
#ifndef SDK_PROP32_STATS
#define SDK_PROP32_STATS 0
#endif
#if SDK_PROP32_STATS
__device__ unsigned long long g_p32_stats[4][128];
#define P32_STAT(k, v) atomicAdd(&g_p32_stats[k][min((uint32_t)(v), 127u)], 1ull)
#else
#define P32_STAT(k, v) ((void)0)
#endif

#ifdef SDK_DEFINE_PROP32_KERNEL
// The fallback's answers back into the batch: listed board i is board list[1 + i]; a board the search
// did not solve gets its own input back (DHT_Node.py:535), not the propagated grid it was searched from.
// One thread per 4 bytes of the dense answers (one dword load; 32-bit index math: the list holds at most
// 2^24 boards), grid-stride over the whole list.
__global__ void p32_scatter_kernel(const uint32_t* list, const uint8_t* sub_out, const int8_t* sub_st,
                                   const uint8_t* in, uint8_t* out, int8_t* status) {
    const uint32_t total = list[0] * 81u;
    for (uint32_t e0 = 4u * (blockIdx.x * blockDim.x + threadIdx.x); e0 < total; e0 += 4u * gridDim.x * blockDim.x) {
        uint32_t word;
        if (e0 + 4u <= total) {
            word = *reinterpret_cast<const uint32_t*>(sub_out + e0);
        } else {
            word = 0u;
            for (uint32_t b = 0; e0 + b < total; ++b) word |= (uint32_t)sub_out[e0 + b] << (8 * b);
        }
#pragma unroll
        for (uint32_t b = 0; b < 4u; ++b) {
            const uint32_t e = e0 + b;
            if (e >= total) break;
            const uint32_t i = e / 81u, c = e - 81u * i;
            const uint32_t j = list[1 + i];
            const int8_t st = sub_st[i];
            const uint64_t o = (uint64_t)j * 81u + c;
            out[o] = st == 1 ? (uint8_t)(word >> (8 * b)) : in[o];
            if (c == 0) status[j] = st;
        }
    }
}

// kP32Order (see p32_unit): digit class t of a Sudoku solution with cell indices distinct mod 32
// in every class
__constant__ uint8_t kP32Order[81] = {2, 5, 8, 1, 4, 7, 3, 0, 6, 1, 4, 7, 0, 3, 6, 2, 8, 5, 0, 3, 6, 8, 2, 5, 1,
                                      7, 4, 8, 2, 5, 7, 1, 4, 0, 6, 3, 7, 1, 4, 6, 0, 3, 8, 5, 2, 6, 0, 3, 5, 8,
                                      2, 7, 4, 1, 5, 8, 2, 4, 7, 1, 6, 3, 0, 4, 7, 1, 3, 6, 0, 5, 2, 8, 3, 6, 0,
                                      2, 5, 8, 4, 1, 7};

// p32_unit's per-lane read order, lane L (half L / 32, unit L % 32) at kP32Table + 40 L: word t = the
// LDS address of the cell of the unit whose kP32Order entry is t, in the lane's half (no per-read
// address add).  Spare lanes take unit 0's (one more reader of each address).  Written once per
// workgroup.
__device__ __forceinline__ void p32_order_table(p32_lds_t* lds) {
    const uint32_t hl = threadIdx.x & 31u;
    uint32_t u0, ua, ub;
    p32_unit_cells(hl < 27 ? hl : 0u, u0, ua, ub);
    __attribute__((address_space(3))) uint32_t* tab =
        (__attribute__((address_space(3))) uint32_t*)(lds + kP32Table + 40u * threadIdx.x);
    const uint32_t region = (uint32_t)(uintptr_t)lds + (threadIdx.x >> 5) * kP32Region;
    for (uint32_t q = 0; q < 9; ++q) {
        const uint32_t o = u0 + (q % 3) * ua + (q / 3) * ub;
        const uint32_t t = kP32Order[o / kP32Rec];
#if SDK_PROP32_TABLE16
        static_assert(kP32Lds <= 65536u, "16-bit table entries");
        ((__attribute__((address_space(3))) uint16_t*)tab)[t] = (uint16_t)(region + o);   // halves 0-8
#else
        tab[t < 3u ? t : t + 1u] = region + o;   // words 0-2, then the pairs (3, 4) .. (7, 8) 8-byte aligned
#endif
    }
}

#ifndef SDK_PROP32_WAVES_PER_EU
#define SDK_PROP32_WAVES_PER_EU 4
#endif
// The kernel body; kStamp (prop32_clock_kernel, a diagnostic twin: the timed kernel runs no stamp)
// writes s_memtime (shader clock) and s_memrealtime (100 MHz) at a workgroup's entry and exit to
// stamps[4 blockIdx.x ..], a buffer nothing else reads: the in-kernel clock of a launch is
// their ratio (MI355X_MICROARCH.md, "DVFS give-back" item 6), the clock the VALU roofline prices
template <bool kStamp>
__device__ __forceinline__ void prop32_body(Prop32Args a, uint64_t* stamps) {
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[kP32Lds];
    p32_lds_t* const lds = (p32_lds_t*)s_lds;
    if (kStamp && threadIdx.x == 0) {    // (stored at once: no register holds them through the loop)
        uint64_t* o = stamps + 4u * blockIdx.x;
        o[0] = __builtin_amdgcn_s_memtime();
        o[1] = __builtin_amdgcn_s_memrealtime();
    }
    p32_order_table(lds);
    __builtin_amdgcn_wave_barrier();
    P32Lane w;
    w.half = threadIdx.x >> 5;
    w.hl = threadIdx.x & 31;
    w.act = w.hl < 27;
    w.reg = lds + w.half * kP32Region;
    const uint32_t groups = (uint32_t)((a.n + 63) / 64);
    uint32_t seg = blockIdx.x % kP32Heads;
    for (;;) {
        const uint32_t g = p32_dequeue(a, groups, seg);
        if (g == ~0u) break;
        const uint64_t base = (uint64_t)g * 64;
        const uint32_t nb = (uint32_t)min<uint64_t>(64, a.n - base);
        // the group's boards into the staging (row-major, 81 bytes each; half h: boards 32h..)
        const uint8_t* src = a.in + base * 81;
        bool hi_given = true;      // a byte > 9 may be in the group: find the inert boards one by one
        if (nb == 64) {
            // 324 pieces of 16 B: 5 per lane, 4 lanes a sixth; piece q of the group to the staging of
            // half q / 162.  Every byte is also tested for > 9 (bytewise, exact: the high bit of
            // (b & 0x7F) + 0x76, or of b itself)
            const uint32_t t = p32_opq(threadIdx.x);
            p32_u4 v[6];
#pragma unroll
            for (int i = 0; i < 6; ++i)
                if (i < 5 || t < 4u) v[i] = reinterpret_cast<const p32_u4*>(src)[t + 64u * i];
            uint32_t hi = 0u;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const uint32_t q = t + 64u * i, h = q >= 162u ? 1u : 0u;
                if (i < 5 || t < 4u) {
                    *(__attribute__((address_space(3))) p32_u4*)(lds + h * (kP32Region - kP32Stage) + 16u * q) = v[i];
#pragma unroll
                    for (int e = 0; e < 4; ++e) hi |= ((v[i][e] & 0x7F7F7F7Fu) + 0x76767676u) | v[i][e];
                }
            }
            hi_given = __builtin_amdgcn_ballot_w64((hi & 0x80808080u) != 0u) != 0ull;
        } else {
            for (uint32_t o = threadIdx.x; o < nb * 81u; o += 64u) {
                const uint32_t h = o >= kP32Stage ? 1u : 0u;
                lds[h * kP32Region + o - h * kP32Stage] = src[o];
            }
        }
        __builtin_amdgcn_wave_barrier();
        // the boards with a given > 9 (inert cells, undecided here): lane L scans board L's row
        uint64_t inert64 = 0ull;
        if (hi_given) {
            bool bad = false;
            const uint32_t t = p32_opq(threadIdx.x);   // (per-lane values recomputed per group: hoisted
            if (t < nb) {                               // out of the group loop they were spilled)
                const p32_lds_t* row = lds + (t >> 5) * kP32Region + (t & 31u) * 81u;
                for (uint32_t c = 0; c < 81u; ++c) bad |= row[c] > 9u;
            }
            inert64 = __builtin_amdgcn_ballot_w64(bad);
        }
        // bit-sliced candidate words: digit v -> one word, 0 -> all nine (boards with a given > 9 are
        // undecided; their words do not matter)
        P32Cells x;
#pragma unroll
        for (int k = 0; k < 3; ++k) p32_convert(w.reg + 3u * w.hl + k, x.c[k]);
        // per-group bookkeeping as 64-bit board masks in scalar registers (bit 32h + b: board b of
        // half h)
        const uint64_t valid = nb >= 64u ? ~0ull : ((1ull << nb) - 1ull);
        uint64_t undec = inert64 & valid, inexact = undec;
        uint64_t live = valid & ~undec, solved = 0ull, contra = 0ull, fixw = 0ull;
        bool lc = false;
        uint32_t next_lc = a.lc_first;     // the step after which the next locked-candidates pass runs
#if SDK_PROP32_STATS
        uint32_t st_lc = 0, st_t4 = ~0u, st_t1 = ~0u;
#endif
        uint32_t it = 0;
        // One exit, at the head: a group that ends in a step still runs that step's cells phase (sound
        // propagation; it only tightens what a handed-over board carries), so every path through the
        // body ends in an update of the cell words and they keep one register home (with exits in the
        // middle of the step the register allocator gave the words a second home and copied all 27
        // out and back on every step)
        // one step (see above); the loop runs two per iteration, so the two copies' register homes of
        // the cell words can alternate instead of being copied back at every latch
        auto step = [&]() {
            uint32_t empty, alls;
            p32_singles(w, x, empty, alls);
            __builtin_amdgcn_wave_barrier();
            if (lc) {
#if SDK_PROP32_STATS
                ++st_lc;
#endif
                const uint32_t lc_own = p32_locked(w, x);
                const uint64_t lchg = p32_mask64(p32_half_or(w.act ? lc_own : 0u));
                const uint64_t stuck = fixw & ~lchg & live;
                undec |= stuck;
                live &= ~stuck;
                fixw = 0ull;
                lc = false;
                __builtin_amdgcn_wave_barrier();
                return;
            }
            uint32_t miss, dup = 0u;
            if (it == 0) {   // a digit given twice: not exact, to the search
                p32_unit<true>(w, lds, miss, dup);
                const uint64_t dupw = p32_mask64(p32_half_or(w.act ? dup : 0u)) & live;
                undec |= dupw;
                inexact |= dupw;
                live &= ~dupw;
            } else {
                p32_unit<false>(w, lds, miss, dup);
            }
            const uint64_t badw = p32_mask64(p32_half_or(w.act ? (miss | empty) : 0u));
            const uint64_t allw = p32_mask64(p32_half_and(w.act ? alls : ~0u));
            const uint64_t sv = allw & ~badw & live, ct = badw & live;
            solved |= sv;
            contra |= ct;
            live &= ~(sv | ct);
#if SDK_PROP32_STATS
            if (st_t4 == ~0u && __builtin_popcountll(live) <= 4) st_t4 = it;
            if (st_t1 == ~0u && __builtin_popcountll(live) <= 1) st_t1 = it;
#endif
            if (live != 0ull) {
                if (a.tail_live && it >= a.tail_step && (uint32_t)__builtin_popcountll(live) <= a.tail_live) {
                    undec |= live;   // the last few boards go to the search with their propagated grids
                    live = 0ull;
                } else if (++it >= a.max_steps) {
                    undec |= live;
                    live = 0ull;
                }
            }
            __builtin_amdgcn_wave_barrier();
            // step lc_first and every lc_every-th after it are followed by a locked-candidates pass;
            // that step also reports which boards it left unchanged (a board unchanged by it and by
            // the pass is stuck)
            lc = live != 0ull && it == next_lc;
            if (lc) next_lc += a.lc_every;
            if (lc) {
                const uint32_t chg_own = p32_cells<true>(w, x);
                fixw = live & ~p32_mask64(p32_half_or(w.act ? chg_own : 0u));
            } else {
                (void)p32_cells<false>(w, x);
            }
            __builtin_amdgcn_wave_barrier();
        };
        while (live != 0ull) {
            step();
            if (live == 0ull) break;
            step();
        }
#if SDK_PROP32_STATS
        if (threadIdx.x == 0) {
            P32_STAT(0, it);
            P32_STAT(1, st_t4);
            P32_STAT(2, st_t1);
            P32_STAT(3, st_lc);
        }
#endif
        __builtin_amdgcn_wave_barrier();
        // the answers, in the staging: solved boards' digits (binary planes of the one-hot words),
        // boards without a completion their input (DHT_Node.py:535); then out, for the whole group
        uint64_t handed = a.handover ? undec & ~inexact : 0ull;   // listed with their grids
        if (handed) {
            // a handed-over grid is searched as a board of its own: two closed cells with one digit
            // in a unit would be duplicated givens there (whose reference semantics differ), and they
            // are a contradiction here -- such a board has no completion
            uint32_t empty, alls;
            p32_singles(w, x, empty, alls);
            __builtin_amdgcn_wave_barrier();
            const uint64_t dupw = p32_mask64(p32_half_or(w.act ? p32_dups(w, lds) : 0u)) & handed;
            contra |= dupw;
            undec &= ~dupw;
            handed &= ~dupw;
            __builtin_amdgcn_wave_barrier();
        }
        if ((solved | handed) && w.act) {
#pragma unroll
            for (int k = 0; k < 3; ++k) p32_digits(x.c[k], x.s[k], w.reg + 3u * w.hl + k);
        }
        for (uint64_t m = contra; m; m &= m - 1ull) {     // rare: the 81 bytes by 64 lanes
            const uint32_t p = (uint32_t)__builtin_ctzll(m);
            const uint8_t* s = a.in + (base + p) * 81;
            p32_lds_t* d = lds + (p >> 5) * kP32Region + (p & 31u) * 81u;
            d[threadIdx.x] = s[threadIdx.x];
            if (threadIdx.x < 17u) d[64 + threadIdx.x] = s[64 + threadIdx.x];
        }
        __builtin_amdgcn_wave_barrier();
        if (solved | contra) {
            // undecided boards' rows get what the staging holds; the search's answers replace them
            uint8_t* dst = a.out + base * 81;
            if (nb == 64) {
                const uint32_t t = p32_opq(threadIdx.x);
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const uint32_t q = t + 64u * i, h = q >= 162u ? 1u : 0u;
                    if (i < 5 || t < 4u)
                        reinterpret_cast<p32_u4*>(dst)[q] =
                            *(const __attribute__((address_space(3))) p32_u4*)(lds + h * (kP32Region - kP32Stage) + 16u * q);
                }
            } else {
                for (uint32_t o = threadIdx.x; o < nb * 81u; o += 64u) {
                    const uint32_t h = o >= kP32Stage ? 1u : 0u;
                    dst[o] = lds[h * kP32Region + o - h * kP32Stage];
                }
            }
        }
        // statuses; the undecided boards are listed with their inputs for the search
        const uint32_t me = p32_opq(threadIdx.x);        // board me of the group (32 half + hl)
        if ((valid >> me) & 1ull)
            a.status[base + me] = (int8_t)(((solved >> me) & 1ull) ? 1 : (((contra >> me) & 1ull) ? 0 : kStUndecided));
        if (undec) {
            uint32_t k0 = 0;
            if (threadIdx.x == 0) k0 = atomicAdd(a.list, (uint32_t)__builtin_popcountll(undec));
            k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);
            if ((undec >> me) & 1ull)
                a.list[1 + k0 + (uint32_t)__builtin_popcountll(undec & ((1ull << me) - 1ull))] = (uint32_t)(base + me);
            uint32_t k = k0;
            for (uint64_t m = undec; m; m &= m - 1ull, ++k) {
                const uint32_t p = (uint32_t)__builtin_ctzll(m);
                uint8_t* d = a.list_in + (uint64_t)k * 81;
                if ((handed >> p) & 1ull) {      // the propagated grid, from the staging
                    const p32_lds_t* s = lds + (p >> 5) * kP32Region + (p & 31u) * 81u;
                    d[threadIdx.x] = s[threadIdx.x];
                    if (threadIdx.x < 17u) d[64 + threadIdx.x] = s[64 + threadIdx.x];
                } else {
                    const uint8_t* s = a.in + (base + p) * 81;
                    d[threadIdx.x] = s[threadIdx.x];
                    if (threadIdx.x < 17u) d[64 + threadIdx.x] = s[64 + threadIdx.x];
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (kStamp) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            uint64_t* o = stamps + 4u * blockIdx.x;
            o[2] = t1;
            o[3] = r1;
        }
    }
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SDK_PROP32_WAVES_PER_EU))) void prop32_kernel(
    Prop32Args a) {
    prop32_body<false>(a, nullptr);
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SDK_PROP32_WAVES_PER_EU))) void prop32_clock_kernel(
    Prop32Args a, uint64_t* stamps) {
    prop32_body<true>(a, stamps);
}
#endif

}  // namespace sdk
