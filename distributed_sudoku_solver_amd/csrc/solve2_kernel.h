// solve2_kernel.h -- DHTNode.solve_sudoku (DHT_Node.py:474-538) on gfx950, two
// boards per wavefront.
//
// Same search as solve_kernel.h (same constraint, same propagation rules, same
// branching orders, same lex-first argument), with a lane layout that keeps the
// SIMD busy: each 32-lane half of the wave owns one board, and lane j < 27 of a
// half owns the three cells j, j+27, j+54 (one column, one row per band) and the
// summary of unit j (rows 0..8, columns 9..17, boxes 18..26).  A propagation round
// is then 84% lane-efficient in all three phases (write contributions, summarise
// units, update cells) instead of 42-63% for one board per wave, and the two
// boards share every instruction of the round.
//
// The halves run independent searches.  Every loop iteration is one propagation
// round for both halves; a half whose round ended (contradiction or fixpoint)
// then takes its search step (count a completion, branch, backtrack, finish the
// board and dequeue the next) under an exec mask while the other half is idle
// for those few instructions.  Everything that is uniform per board (depth,
// completions, node count, board index) lives in VGPRs, identical across the
// half's lanes.
//
// Cell state = its contribution word.  solve_kernel keeps 16-bit states and
// converts each to the bit-sliced contribution word (solve_kernel.h contrib())
// before every LDS write; here the state IS that word, so the three writes of a
// round need no VALU work and only a cell that changes pays for the format:
//   [0..8]   candidates
//   [9..17]  the digit of a given (1..9)
//   [18..26] the digit of a solved non-given cell (set iff one candidate is left)
//   [27]     out-of-domain given (10..255): constrains nothing
// so  open (branchable) <=> state < 0x200 with >= 2 candidates, and a
// contradiction cell (no candidate) is the state 0.
//
// Bank-conflict-free unit reads: read k of a unit lane fetches the cell of its
// unit that holds digit k+1 in the fixed Sudoku solution
// G(r,c) = (3(r%3) + 2(r/3) + c) mod 9.  The 9 cells of one digit of a solution
// are one per row, column and box, so in every read the 27 lanes of a half
// fetch only 9 distinct words (each broadcast to its row, column and box lane),
// and for this G those 9 words sit in 9 distinct banks of ds_read_b32's
// 32-lane group (tools/lds_banks.py checks it).  Spare lanes 27..31 read what
// lane 0 of their half reads.
//
// DFS stack: one 8-byte snapshot (the lane's three cell states, packed to 16 bits) per lane
// per level; the first kLdsLevels levels are LDS-resident, deeper levels go to a
// per-workgroup HBM region (L2-resident).  Branch records (cell, untried digits)
// are in LDS.  Count mode (frontier counts) stays on solve_kernel.
#pragma once
#include "solve_kernel.h"

namespace sdk {

constexpr int kLdsLevels = 10;                     // 10 x 512 B per wave in LDS (24 waves/CU fit)
constexpr int kStack2WordsPerBlock = kMaxDepth * 64 * 2;

struct Lane2 {
    int lane, hl, half;
    bool act;                 // owns cells (hl < 27)
    int c0, c1, c2;           // cells hl, hl+27, hl+54
    int ucol, ur0, ur1, ur2, ub0, ub1, ub2;
    int ucell[9];             // cells of unit hl
    uint32_t* s_cell;         // this half's 81 contribution words
    uint32_t* s_unit;         // this half's 27 unit summaries
};

__device__ __forceinline__ void init_lane2(Lane2& w, uint32_t* s_cell_all, uint32_t* s_unit_all) {
    const int lane = threadIdx.x;
    w.lane = lane;
    w.hl = lane & 31;
    w.half = lane >> 5;
    w.act = w.hl < 27;
    const int j = w.act ? w.hl : 0;
    const int col = j % 9, r0 = j / 9;
    if (w.act) {
        w.c0 = j;
        w.c1 = j + 27;
        w.c2 = j + 54;
        w.ucol = 9 + col;
        w.ur0 = r0;
        w.ur1 = r0 + 3;
        w.ur2 = r0 + 6;
        w.ub0 = 18 + col / 3;
        w.ub1 = 21 + col / 3;
        w.ub2 = 24 + col / 3;
    } else {
        // lanes 27..31 run the same instructions on spare slots (cells 81..95, units
        // 27..31) with inert cells, so the round needs no exec-mask branches
        // (slot banks chosen so no write shares a bank with a real cell of the same
        // store: c0 stores hit banks 0..26, c1 27..31+0..21, c2 22..31+0..16)
        const int e = w.hl - 27;
        w.c0 = 91 + e;
        w.c1 = 86 + e;
        w.c2 = 81 + e;
        w.ucol = w.ur0 = w.ur1 = w.ur2 = w.ub0 = w.ub1 = w.ub2 = 27 + e;
    }
    // unit j's cell holding digit k+1 of G (see the header); spare lanes copy lane 0
    const int uj = w.act ? j : 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        int cell = 0;
        for (int q = 0; q < 9; ++q) {
            int r, c;
            if (uj < 9) { r = uj; c = q; }
            else if (uj < 18) { r = q; c = uj - 9; }
            else { r = ((uj - 18) / 3) * 3 + q / 3; c = ((uj - 18) % 3) * 3 + q % 3; }
            if ((3 * (r % 3) + 2 * (r / 3) + c) % 9 == k) cell = 9 * r + c;
        }
        w.ucell[k] = cell;
    }
    w.s_cell = s_cell_all + w.half * 96;
    w.s_unit = s_unit_all + w.half * 32;
}

// per-half vote: does any lane of MY half have `pred`?
__device__ __forceinline__ bool half_any(const Lane2& w, bool pred) {
    const unsigned long long b = __ballot(pred);
    const uint32_t lo = (uint32_t)b, hi = (uint32_t)(b >> 32);
    return (w.half ? hi : lo) != 0u;
}

// per-half vote on a lane mask, all scalar: a lane's result is whether any lane of
// its half has `pred` (inverse_ballot turns the uniform mask back into lane bools)
__device__ __forceinline__ bool half_any_s(bool pred) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(pred);
    const uint64_t lo = (__builtin_amdgcn_readfirstlane((int)m) != 0) ? 0x00000000FFFFFFFFull : 0ull;
    const uint64_t hi = (__builtin_amdgcn_readfirstlane((int)(m >> 32)) != 0) ? 0xFFFFFFFF00000000ull : 0ull;
    return __builtin_amdgcn_inverse_ballot_w64(lo | hi);
}

// min over the 32 lanes of each half (all lanes of the half must be active).
// ds_swizzle in bitmask mode (xor_mask << 10 | and_mask 0x1F) exchanges within 32
// lanes with no address register (a __shfl_xor's lane addresses are loop-invariant,
// so the compiler hoists and, under register pressure, spills them).
__device__ __forceinline__ uint32_t half_min(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (1 << 10) | 0x1F));
    v = min(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (2 << 10) | 0x1F));
    v = min(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (4 << 10) | 0x1F));
    v = min(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (8 << 10) | 0x1F));
    v = min(v, (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, (16 << 10) | 0x1F));
    return v;
}

// broadcast lane 0 of my half
__device__ __forceinline__ uint32_t half_first(const Lane2& w, uint32_t v) {
    return (uint32_t)__shfl((int)v, w.half * 32);
}

constexpr uint32_t kGiven2 = 0x3FE00u;      // [9..17] digit of a given
constexpr uint32_t kInert2 = 1u << 27;      // out-of-domain given
constexpr uint32_t kOpenLimit2 = 0x200u;    // states below this are non-given, unsolved (or empty)

// state of input byte v (0 = empty)
__device__ __forceinline__ uint32_t cell_init2(uint32_t v) {
    const uint32_t m = 1u << ((v - 1u) & 31u);
    return v == 0 ? kCands : (v <= 9 ? (m | (m << 9)) : kInert2);
}

// state of a non-given cell with candidates v: the solved field is set iff one is left
__device__ __forceinline__ uint32_t norm2(uint32_t v) {
    return v | (((v & (v - 1u)) == 0u) ? (v << 18) : 0u);
}

// 16-bit snapshot form (candidates | given << 9 | inert << 10) and back
__device__ __forceinline__ uint32_t pack2(uint32_t x) {
    return (x & kCands) | ((x & kGiven2) ? 0x200u : 0u) | ((x >> 27) << 10);
}
__device__ __forceinline__ uint32_t unpack2(uint32_t y) {
    const uint32_t v = y & kCands;
    return (y & 0x400u) ? kInert2 : ((y & 0x200u) ? (v | (v << 9)) : norm2(v));
}

// branchable cell: candidate count, else 0
__device__ __forceinline__ uint32_t open_count2(uint32_t x) {
    return x < kOpenLimit2 ? (uint32_t)__popc(x) : 0u;
}

// update_cell (solve_kernel.h) on the contribution-format state, as a branch-free
// value function: three guarded in-place updates of s0/s1/s2 get merged into one
// store through a phi of their addresses, which demotes the cells to scratch memory.
__device__ __forceinline__ uint32_t updated_cell(uint32_t x, uint32_t u, bool& bad, bool& chg) {
    // every state below 0x200 is an empty cell with >= 2 candidates, or 0
    const bool open = (x - 1u) < kOpenLimit2 - 1u;
    const uint32_t v1 = x & ~u;                 // (only meaningful when open: then x = candidates)
    const uint32_t h = v1 & (u >> 16);          // u >> 16 = hidden-single digits (9 bits)
    const uint32_t v2 = h ? h : v1;
    bad |= (open & (((h & (h - 1u)) != 0u) | (v2 == 0u))) | (x == 0u);
    const uint32_t n = open ? norm2(v2) : x;
    chg |= n != x;
    return n;
}

// One propagation round for both halves, branch-free (idle lanes work on spare
// slots).  Per lane: bad (contradiction in MY half), chg (a cell of MY half changed).
__device__ __forceinline__ void round2(const Lane2& w, uint32_t& s0, uint32_t& s1, uint32_t& s2, bool& bad,
                                       bool& chg) {
    w.s_cell[w.c0] = s0;
    w.s_cell[w.c1] = s1;
    w.s_cell[w.c2] = s2;
    __syncthreads();
    uint32_t ones = 0, twos = 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const uint32_t x = w.s_cell[w.ucell[k]];
        twos |= ones & x;
        ones |= x;
    }
    const uint32_t tc1 = (ones >> 9) & kCands, tc2 = (twos >> 9) & kCands;
    const uint32_t tn1 = (ones >> 18) & kCands, tn2 = (twos >> 18) & kCands;
    const bool exact = !(ones >> 27) && !tc2;    // exact unit: every digit exactly once
    const bool conflict = (tn2 | (tn1 & tc1)) != 0 || (exact && (ones & kCands) != kCands);
    const uint32_t once = exact ? (ones & ~twos & kCands) : 0u;
    const uint32_t summ = tc1 | tn1 | (once << 16);
    w.s_unit[w.hl] = summ;
    __syncthreads();
    bool b = w.act && conflict, c = false;
    const uint32_t uc = w.s_unit[w.ucol];
    s0 = updated_cell(s0, uc | w.s_unit[w.ur0] | w.s_unit[w.ub0], b, c);
    s1 = updated_cell(s1, uc | w.s_unit[w.ur1] | w.s_unit[w.ub1], b, c);
    s2 = updated_cell(s2, uc | w.s_unit[w.ur2] | w.s_unit[w.ub2], b, c);
    bad = half_any_s(b);
    chg = half_any_s(c);
}

// branch key of a cell: (candidates << 16 | cell << 9 | mask) for MRV, (cell << 9 | mask)
// for LEX; ~0 for cells that are not branchable
__device__ __forceinline__ uint32_t branch_key(uint32_t x, int cell, int order) {
    const uint32_t k = open_count2(x);
    if (k < 2) return ~0u;
    const uint32_t base = ((uint32_t)cell << 9) | (x & kCands);
    return order == ORDER_LEX ? base : (k << 16) | base;
}

__device__ __forceinline__ void set_cell2(const Lane2& w, uint32_t& s0, uint32_t& s1, uint32_t& s2, int cell,
                                          uint32_t d) {
    d |= d << 18;
    s0 = (w.act && cell == w.c0) ? d : s0;
    s1 = (w.act && cell == w.c1) ? d : s1;
    s2 = (w.act && cell == w.c2) ? d : s2;
}

__device__ __forceinline__ uint32_t out_byte(uint32_t in, uint32_t s, bool solved) {
    return (solved && in == 0) ? (uint32_t)__ffs(s & kCands) : in;
}

// per-half search state: uniform within the half (bidx .. rounds), per lane (in*, s*)
struct Board2 {
    uint32_t bidx, bend;          // current board, end of the dequeued chunk
    bool active;
    int depth, order;
    uint32_t count, lim;
    uint64_t nodes, rounds;
    uint32_t maxd;                // deepest DFS level reached (SDK_WORK_DEPTH)
    uint32_t in0, in1, in2;       // input bytes of the lane's cells
    uint32_t s0, s1, s2;          // cell states
};

// kernel arguments as plain values (a reference to the by-value kernel argument
// struct would put it in scratch memory)
struct Args2 {
    const uint8_t* in;
    uint64_t in_first, in_step;
    const uint16_t* mask;
    uint32_t* next;
    uint32_t chunk;
    uint64_t n;
    int order;
    uint8_t* out;
    int8_t* status;
    uint64_t* work;
    int work_rounds;
    uint64_t budget;
};

// (re)start the search of board b.bidx from its input (+ first-cell mask)
__device__ __forceinline__ void start_board(const Lane2& w, const Args2& a, Board2& b, bool reload) {
    if (reload) {
        const uint8_t* src = a.in + (a.in_first + (uint64_t)b.bidx * a.in_step) * 81;
        b.in0 = w.act ? (uint32_t)src[w.c0] : 0u;
        b.in1 = w.act ? (uint32_t)src[w.c1] : 0u;
        b.in2 = w.act ? (uint32_t)src[w.c2] : 0u;
    }
    b.s0 = w.act ? cell_init2(b.in0) : kInert2;
    b.s1 = w.act ? cell_init2(b.in1) : kInert2;
    b.s2 = w.act ? cell_init2(b.in2) : kInert2;
    if (a.mask) {
        // TASK `range` restricts the lowest-index empty input cell only (DHT_Node.py:474,522,531)
        const uint32_t fm = ((uint32_t)a.mask[b.bidx] >> 1) & kCands;
        uint32_t z = ~0u;
        if (w.act)
            z = b.in0 == 0 ? (uint32_t)w.c0 : (b.in1 == 0 ? (uint32_t)w.c1 : (b.in2 == 0 ? (uint32_t)w.c2 : ~0u));
        z = half_min(z);
        // branch-free: guarded stores to different cells would be merged into one
        // store through a phi of addresses, which demotes the cells to scratch
        // (that cell is empty: its state is kCands, restricted to norm2(fm))
        const uint32_t ms = norm2(fm);
        b.s0 = (w.act && z == (uint32_t)w.c0) ? ms : b.s0;
        b.s1 = (w.act && z == (uint32_t)w.c1) ? ms : b.s1;
        b.s2 = (w.act && z == (uint32_t)w.c2) ? ms : b.s2;
    }
    b.depth = 0;
    b.count = 0;
}

// next board for this half: within the chunk, else dequeue a new chunk
__device__ __forceinline__ void next_board(const Lane2& w, const Args2& a, Board2& b) {
    ++b.bidx;
    if (b.bidx >= b.bend) {
        uint32_t base = 0;
        if (w.hl == 0) base = atomicAdd(a.next, a.chunk);
        base = half_first(w, base);
        b.bidx = base;
        b.bend = (uint32_t)min((uint64_t)base + a.chunk, a.n);
    }
    b.active = (uint64_t)b.bidx < a.n;
    b.order = a.order == ORDER_LEX ? ORDER_LEX : ORDER_MRV;
    b.lim = b.order == ORDER_LEX ? 1u : 2u;
    b.nodes = b.rounds = 0;
    b.maxd = 0;
    if (b.active) start_board(w, a, b, true);
    else b.s0 = b.s1 = b.s2 = kInert2;
}

__device__ __forceinline__ void finish_board(const Lane2& w, const Args2& a, Board2& b, int st) {
    uint8_t* dst = a.out + (uint64_t)b.bidx * 81;
    if (st != 1 && w.act) {           // the reference restores the grid (DHT_Node.py:535)
        dst[w.c0] = (uint8_t)b.in0;
        dst[w.c1] = (uint8_t)b.in1;
        dst[w.c2] = (uint8_t)b.in2;
    }
    if (w.hl == 0) {
        a.status[b.bidx] = (int8_t)st;
        if (a.work) a.work[b.bidx] = a.work_rounds == 1 ? b.rounds : (a.work_rounds == 2 ? (uint64_t)b.maxd : b.nodes);
    }
    next_board(w, a, b);
}

#ifdef SDK_DEFINE_SOLVE2_KERNEL   // defined in solve2_launch.hip only
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(6))) void solve2_kernel(SolveArgs args) {
    __shared__ uint32_t s_cell[2 * 96];
    __shared__ uint32_t s_unit[2 * 32];
    __shared__ uint32_t s_br[2][kMaxDepth];
    __shared__ uint2 s_stk[kLdsLevels][64];
    Lane2 w;
    init_lane2(w, s_cell, s_unit);
    uint2* g_stk = reinterpret_cast<uint2*>(args.stack) + (size_t)blockIdx.x * (kMaxDepth * 64);
    Args2 a;
    a.in = args.in;
    a.in_first = args.in_first;
    a.in_step = args.in_step;
    a.mask = args.mask;
    a.next = args.next;
    a.chunk = args.chunk;
    a.n = args.n;
    a.order = args.order;
    a.out = args.out;
    a.status = args.status;
    a.work = args.work;
    a.work_rounds = args.work_rounds;
    a.budget = args.budget;

    Board2 b;
    b.bidx = 0xFFFFFFFFu;   // ++ -> 0 >= bend = 0: first dequeue
    b.bend = 0;
    b.in0 = b.in1 = b.in2 = 0;
    b.depth = 0;
    b.count = 0;
    next_board(w, a, b);

    for (;;) {
        if (!__any((int)b.active)) break;
        bool bad, chg;
        round2(w, b.s0, b.s1, b.s2, bad, chg);
        ++b.rounds;
        const bool ev = b.active && (bad || !chg);
        if (!__any((int)ev)) continue;
        if (!ev) continue;
        ++b.nodes;
        int r = bad ? P_CONTRA
                    : (half_any(w, open_count2(b.s0) >= 2 || open_count2(b.s1) >= 2 || open_count2(b.s2) >= 2) ? P_OPEN
                                                                                                          : P_SOLVED);
        if (a.budget && b.nodes > a.budget) {
            finish_board(w, a, b, -2);
            continue;
        }
        if (r == P_SOLVED) {
            ++b.count;
            if (b.count == 1 && w.act) {
                uint8_t* dst = a.out + (uint64_t)b.bidx * 81;
                dst[w.c0] = (uint8_t)out_byte(b.in0, b.s0, true);
                dst[w.c1] = (uint8_t)out_byte(b.in1, b.s1, true);
                dst[w.c2] = (uint8_t)out_byte(b.in2, b.s2, true);
            }
            if (b.count >= b.lim) {
                if (b.order == ORDER_MRV) {      // >= 2 completions: lex re-search
                    b.order = ORDER_LEX;
                    b.lim = 1;
                    start_board(w, a, b, false);
                } else {
                    finish_board(w, a, b, 1);
                }
                continue;
            }
            r = P_CONTRA;
        }
        if (r == P_OPEN) {
            uint32_t key = ~0u;
            if (w.act)
                key = min(branch_key(b.s0, w.c0, b.order), min(branch_key(b.s1, w.c1, b.order),
                                                               branch_key(b.s2, w.c2, b.order)));
            key = half_min(key);
            const int cell = (int)((key >> 9) & 0x7Fu);
            const uint32_t m = key & kCands;
            const uint32_t d = m & (0u - m);
            const uint2 snap = make_uint2(pack2(b.s0) | (pack2(b.s1) << 16), pack2(b.s2));
            if (b.depth < kLdsLevels) s_stk[b.depth][w.lane] = snap;
            else g_stk[b.depth * 64 + w.lane] = snap;
            if (w.hl == 0) s_br[w.half][b.depth] = (uint32_t)cell | ((m ^ d) << 16);
            ++b.depth;
            b.maxd = max(b.maxd, (uint32_t)b.depth);
            set_cell2(w, b.s0, b.s1, b.s2, cell, d);
            continue;
        }
        // contradiction: resume the deepest level with untried digits
        if (b.depth == 0) {
            finish_board(w, a, b, b.count > 0 ? 1 : 0);
            continue;
        }
        const uint32_t br = s_br[w.half][b.depth - 1];
        const int cell = (int)(br & 0xFFu);
        uint32_t rest = br >> 16;
        const uint32_t d = rest & (0u - rest);
        rest ^= d;
        const uint2 snap = b.depth - 1 < kLdsLevels ? s_stk[b.depth - 1][w.lane] : g_stk[(b.depth - 1) * 64 + w.lane];
        b.s0 = unpack2(snap.x & 0xFFFFu);
        b.s1 = unpack2(snap.x >> 16);
        b.s2 = unpack2(snap.y);
        if (rest == 0) --b.depth;
        else if (w.hl == 0) s_br[w.half][b.depth - 1] = (uint32_t)cell | (rest << 16);
        set_cell2(w, b.s0, b.s1, b.s2, cell, d);
    }
}
#endif  // SDK_DEFINE_SOLVE2_KERNEL

}  // namespace sdk
