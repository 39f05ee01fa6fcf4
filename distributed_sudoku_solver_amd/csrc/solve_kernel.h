// solve_kernel.h -- the solve path of DHTNode.solve_sudoku (DHT_Node.py:474-538) on gfx950.
//
// One board per wavefront (one 64-lane workgroup).  Lane l owns cell l (the "A"
// half of its state word) and, for l < 17, cell 64+l (the "B" half).  A cell
// state is 16 bits: bits 0..8 candidate digits 1..9, CLUE = given 1..9,
// INERT = given 10..255 (the reference compares cells with `== guess` only, so
// such a value never conflicts: utils.py:36,44,53).
//
// Constraint (exactly the naive DFS's): every pair of cells in a unit where at
// least one cell is NOT a given must differ.  Given-vs-given duplicates are
// ignored (the reference never validates clues).
//
// Propagation round (all in LDS, no atomics):
//   1. every lane writes a bit-sliced contribution word per cell to s_cell[81];
//   2. lanes 0..26 each summarise one unit (row/col/box) from its 9 words
//      (two ops per cell: twos |= ones & w; ones |= w):
//        T     = digits of single-candidate cells (givens and solved),
//        once  = digits with exactly one candidate cell (hidden singles) -- only
//                in "exact" units (no INERT cell, no duplicate given), where
//                every digit must occur exactly once in every completion,
//        conflict = two non-given singles share a digit, a non-given single
//                repeats a given, or an exact unit lost a digit entirely;
//   3. every lane ORs its three unit summaries and updates its cells:
//        cand &= ~T (naked-single elimination); cand & once -> hidden single.
//   Repeated to a fixpoint; wave votes (__any/__ballot) decide CONTRA / SOLVED / OPEN.
// Every step only removes digits that appear in no completion, so the set of
// completions below a node is unchanged by propagation.
//
// Search.  Branch cell chosen with __ballot + ctz:
//   ORDER_LEX: the lowest-index open cell, digits ascending.  All cells before
//     it are forced, so the first completion found is the lexicographically
//     first one = the reference's row-major ascending DFS result.
//   ORDER_MRV: fewest candidates (ties: lowest index).  Used to count up to 2
//     completions; a unique completion IS the lexicographically first one.  If
//     2 are found the board is re-searched with ORDER_LEX.
// The DFS stack (one 256-B snapshot of the wave's state words per level) lives
// in a per-workgroup HBM region (L2-resident in practice); branch records (cell,
// untried digits) live in LDS.
//
// Boards are handed out to persistent wavefronts `chunk` at a time by one atomic
// (one returning atomic on one word saturates near 88 dequeues/us on MI355X, so
// the host sizes the chunk to keep dequeues well below that).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Three-input OR and and-or in the kernels' inline asm.  v_or3_b32 and v_and_or_b32 (like every
// older 3-source VOP3 op) issue at most ~1 per SIMD quad-cycle whatever the operands; the same
// functions as v_bitop3_b32 truth tables (S0 | S1 | S2 = 0xFE, S0 & S1 | S2 = 0xEA) issue like
// 2-operand ops -- ~1.55 per quad-cycle, 1.6x -- unless all three sources sit in one VGPR bank
// (register index mod 4) (tools/bank_calib.hip, profiles/r06/bank_calib_r06x.txt).
#ifndef SDK_BITOP3_OR
#define SDK_BITOP3_OR 1
#endif
#if SDK_BITOP3_OR
#define SDK_OR3(d, a, b, c) "v_bitop3_b32 " d ", " a ", " b ", " c " bitop3:0xfe\n\t"
#define SDK_ANDOR(d, a, b, c) "v_bitop3_b32 " d ", " a ", " b ", " c " bitop3:0xea\n\t"
#else
#define SDK_OR3(d, a, b, c) "v_or3_b32 " d ", " a ", " b ", " c "\n\t"
#define SDK_ANDOR(d, a, b, c) "v_and_or_b32 " d ", " a ", " b ", " c "\n\t"
#endif
// a | b | c as one SDK_OR3 (written in C, a three-input OR becomes v_or3_b32)
__device__ __forceinline__ uint32_t sdk_or3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm(SDK_OR3("%0", "%1", "%2", "%3") : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

namespace sdk {

constexpr uint32_t kCands = 0x1FFu;
constexpr uint32_t kClue = 0x200u;
constexpr uint32_t kInert = 0x400u;
constexpr uint32_t kFixed = kClue | kInert;
constexpr int kMaxDepth = 81;
constexpr uint32_t kChunk = 4;        // expand_kernel chunk; solve_kernel takes SolveArgs::chunk
constexpr int kStackWordsPerBlock = kMaxDepth * 64;

enum { P_CONTRA = 0, P_SOLVED = 1, P_OPEN = 2 };
enum { ORDER_MRV = 0, ORDER_LEX = 1 };

struct SolveArgs {
    const uint8_t* in;
    const uint16_t* mask;      // nullable: first-cell digit mask, bit d = digit d
    uint8_t* out;
    int8_t* status;
    uint64_t* work;            // nullable
    uint64_t n;
    uint32_t* next;            // work counter (zeroed before launch)
    uint32_t* stack;           // gridDim.x * kStackWordsPerBlock words
    uint64_t budget;           // nodes per board, 0 = unlimited
    int order;                 // SDK_ORDER_*
    uint64_t limit;            // count mode: per-board completion limit (0 = none)
    unsigned long long* count; // count mode: running total over the batch (atomic)
    unsigned long long* counts;// count mode: per-board counts (nullable)
    int count_mode;
    uint32_t chunk;            // boards per dequeue (one atomic on `next` per chunk)
    int work_rounds;           // what work[] counts: 0 search nodes, 1 propagation rounds, 2 max DFS depth
    uint64_t in_first;         // board i of the launch reads in[(in_first + i*in_step)*81];
    uint64_t in_step;          // outputs stay dense (out[i*81], status[i]); 0/1 = contiguous
    int locked;                // QUAD solver: locked-candidates pass at fixpoints (SDK_OPT_LOCKED)
    uint32_t* heads;           // QUAD solver: kHeads dequeue heads, one per XCD segment (nullable)
    void* donate;              // QUAD solver, LEX solves: subtree-donation area (solve4_kernel.h, DnCtl first)
    const uint32_t* n_dev;     // donation kernel: board count read on the device (a phase's list
                               // length, written by an earlier launch); `n` is then its bound
    void* save = nullptr;      // QUAD split phase: stacks of boards that reach the split budget
                               // (solve4_kernel.h SplitSave; nullable)
    uint32_t* save_idx = nullptr;   // ... and each saved board's entry (by board index)
    uint64_t budget_big = 0;        // QUAD split phase of a device-counted batch (n_dev): the budget
                                    // when more than kBudgetBigBoards boards are searched (0 = budget)
    long long* found = nullptr;     // QUAD first-solution scan (sdk_frontier_first): the lowest board
                                    // index (in_first + i * in_step) with status 1 or -2 so far; boards
                                    // above it are cancelled (solve4_kernel.h, s_found4)
};
// the phased solve's default split budget doubles above this many searched boards (sudoku_hip.hip)
constexpr uint64_t kBudgetBigBoards = 1ull << 19;
// status of a board a first-solution scan stopped because it lies above a lower board's hit
constexpr int kStCancelled = -3;

// per-XCD dequeue: the first n - n/128 boards are cut into kHeads contiguous segments with a
// head each, workgroup g takes chunks of segment g % kHeads (the XCD the round-robin
// dispatch put it on) and, once that is drained, of the shared tail (one more head);
// heads kHeadStride words apart (own cache lines)
#ifndef SDK_HEADS
#define SDK_HEADS 8
#endif
constexpr int kHeads = SDK_HEADS;   // a multiple of 8: segment g % kHeads stays on one XCD
constexpr int kHeadStride = 64;
// the heads buffer: kHeads segment heads, the shared tail, then the launch's dequeue counter, so
// one memset clears a QUAD launch's dequeue state
constexpr int kHeadNext = (kHeads + 1) * kHeadStride;
constexpr int kHeadWords = (kHeads + 2) * kHeadStride;

__device__ __forceinline__ uint32_t cell_init(uint32_t v) {
    return v == 0 ? kCands : (v <= 9 ? ((1u << (v - 1)) | kClue) : kInert);
}

__device__ __forceinline__ bool is_single(uint32_t v) { return v != 0 && (v & (v - 1)) == 0; }

// candidates count of a branchable cell, else 0
__device__ __forceinline__ uint32_t open_count(uint32_t x) {
    return (x & kFixed) ? 0u : (uint32_t)__popc(x & kCands);
}

struct Wave {
    uint32_t* s_cell;   // [96]
    uint32_t* s_unit;   // [32]
    uint32_t* s_br;     // [kMaxDepth]
    uint32_t* stk;      // this workgroup's HBM stack
    int lane;
    bool hasB;
    int uA0, uA1, uA2, uB0, uB1, uB2;
    int ucell[9];
};

__device__ __forceinline__ void update_cell(uint32_t& x, uint32_t u, bool& bad, bool& chg) {
    if (x & kFixed) return;
    const uint32_t v = x & kCands;
    if (v & (v - 1)) {
        uint32_t v1 = v & ~u;
        const uint32_t h = v1 & (u >> 16) & kCands;
        if (h) {
            if (h & (h - 1)) bad = true;
            v1 = h;
        }
        if (v1 == 0) bad = true;
        if (v1 != v) { chg = true; x = v1; }
    } else if (v == 0) {
        bad = true;
    }
}

// A cell's contribution to its units, as bit-sliced fields so that a unit is
// summarised with two ops per cell (twos |= ones & w; ones |= w):
//   [0..8]   candidates                 -> hidden singles / lost digits
//   [9..17]  digit of a given           -> duplicate givens make a unit non-exact
//   [18..26] digit of a solved non-given -> duplicates are a conflict
//   [27]     out-of-domain given        -> unit non-exact
// (arithmetic only: early returns or ternaries over shifted values compile to
// nested exec-mask blocks)
__device__ __forceinline__ uint32_t contrib(uint32_t x) {
    const uint32_t v = x & kCands;
    const uint32_t clue = (x >> 9) & 1u, inert = (x >> 10) & 1u;
    const uint32_t single = (uint32_t)((v & (v - 1)) == 0);   // v == 0 contributes nothing either way
    const uint32_t shift = 18u - 9u * clue;
    const uint32_t r = v | ((v << shift) & (0u - (clue | single)));
    return (r & (inert - 1u)) | (inert << 27);
}

__device__ __forceinline__ int propagate(const Wave& w, uint32_t& sa, uint32_t& sb, uint64_t& rounds) {
    for (;;) {
        ++rounds;
        w.s_cell[w.lane] = contrib(sa);
        if (w.hasB) w.s_cell[64 + w.lane] = contrib(sb);
        __syncthreads();
        uint32_t summ = 0;
        if (w.lane < 27) {
            uint32_t ones = 0, twos = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const uint32_t x = w.s_cell[w.ucell[k]];
                twos |= ones & x;
                ones |= x;
            }
            const uint32_t tc1 = (ones >> 9) & kCands, tc2 = (twos >> 9) & kCands;
            const uint32_t tn1 = (ones >> 18) & kCands, tn2 = (twos >> 18) & kCands;
            bool conflict = (tn2 | (tn1 & tc1)) != 0;
            uint32_t once = 0;
            if (!(ones >> 27) && !tc2) {           // exact unit: every digit exactly once
                if ((ones & kCands) != kCands) conflict = true;
                once = ones & ~twos & kCands;
            }
            summ = tc1 | tn1 | (once << 16) | (conflict ? 0x80000000u : 0u);
            w.s_unit[w.lane] = summ;
        }
        if (__any((int)(summ >> 31))) return P_CONTRA;
        __syncthreads();
        const uint32_t ua = w.s_unit[w.uA0] | w.s_unit[w.uA1] | w.s_unit[w.uA2];
        const uint32_t ub = w.hasB ? (w.s_unit[w.uB0] | w.s_unit[w.uB1] | w.s_unit[w.uB2]) : 0u;
        bool bad = false, chg = false;
        update_cell(sa, ua, bad, chg);
        if (w.hasB) update_cell(sb, ub, bad, chg);
        if (__any((int)bad)) return P_CONTRA;
        if (!__any((int)chg)) {
            const bool open = open_count(sa) >= 2 || (w.hasB && open_count(sb) >= 2);
            return __any((int)open) ? P_OPEN : P_SOLVED;
        }
    }
}

__device__ __forceinline__ void write_board(const Wave& w, uint8_t* dst, uint32_t inA, uint32_t inB,
                                            uint32_t sa, uint32_t sb, bool solved) {
    uint32_t a = inA, b = inB;
    if (solved) {
        if (a == 0) a = (uint32_t)__ffs(sa & kCands);
        if (b == 0) b = (uint32_t)__ffs(sb & kCands);
    }
    dst[w.lane] = (uint8_t)a;
    if (w.hasB) dst[64 + w.lane] = (uint8_t)b;
}

// Branch-free on purpose: two guarded stores to sa / sb get merged by the
// compiler into one store through a phi of their addresses, which demotes both
// to scratch memory.
__device__ __forceinline__ void set_cell(const Wave& w, uint32_t& sa, uint32_t& sb, int cell, uint32_t d) {
    const bool mine = w.lane == (cell & 63);
    sa = (mine && cell < 64) ? d : sa;
    sb = (mine && cell >= 64) ? d : sb;
}

// Returns the number of completions found (stopping at `limit`, 0 = no limit),
// or -1 when the node budget ran out.  The first completion is written to
// `sol` when non-null.
__device__ __forceinline__ int64_t search(const Wave& w, int order, uint32_t sa0, uint32_t sb0, uint64_t limit,
                          uint64_t budget, uint64_t& nodes, uint64_t& rounds, uint64_t& maxd, uint8_t* sol,
                          uint32_t inA, uint32_t inB) {
    uint32_t sa = sa0, sb = sb0;
    int depth = 0;
    int64_t count = 0;
    for (;;) {
        int r = propagate(w, sa, sb, rounds);
        ++nodes;
        if (budget && nodes > budget) return -1;
        if (r == P_SOLVED) {
            ++count;
            if (count == 1 && sol) write_board(w, sol, inA, inB, sa, sb, true);
            if (limit && (uint64_t)count >= limit) return count;
            r = P_CONTRA;
        }
        if (r == P_OPEN) {
            const uint32_t pa = open_count(sa);
            const uint32_t pb = w.hasB ? open_count(sb) : 0u;
            unsigned long long ma, mb;
            if (order == ORDER_LEX) {
                ma = __ballot(pa >= 2);
                mb = __ballot(pb >= 2);
            } else {
                ma = mb = 0;
                for (uint32_t k = 2; k <= 9; ++k) {
                    ma = __ballot(pa == k);
                    mb = __ballot(pb == k);
                    if (ma | mb) break;
                }
            }
            const int cell = ma ? (int)__builtin_ctzll(ma) : 64 + (int)__builtin_ctzll(mb);
            // read both halves (a select of the two values would make the compiler take
            // their addresses and demote sa/sb to scratch)
            const uint32_t mA = (uint32_t)__builtin_amdgcn_readlane((int)sa, cell & 63);
            const uint32_t mB = (uint32_t)__builtin_amdgcn_readlane((int)sb, cell & 63);
            const uint32_t m = (cell < 64 ? mA : mB) & kCands;
            const uint32_t d = m & (0u - m);
            w.stk[depth * 64 + w.lane] = sa | (sb << 16);
            if (w.lane == 0) w.s_br[depth] = (uint32_t)cell | ((m ^ d) << 16);
            ++depth;
            maxd = max(maxd, (uint64_t)depth);
            set_cell(w, sa, sb, cell, d);
            continue;
        }
        // contradiction: resume the deepest level that still has untried digits
        if (depth == 0) return count;
        const uint32_t br = w.s_br[depth - 1];
        const int cell = (int)(br & 0xFFu);
        uint32_t rest = br >> 16;
        const uint32_t d = rest & (0u - rest);
        rest ^= d;
        const uint32_t snap = w.stk[(depth - 1) * 64 + w.lane];
        sa = snap & 0xFFFFu;
        sb = snap >> 16;
        if (rest == 0) {
            --depth;
        } else if (w.lane == 0) {
            w.s_br[depth - 1] = (uint32_t)cell | (rest << 16);
        }
        set_cell(w, sa, sb, cell, d);
    }
}

__device__ __forceinline__ void init_wave(Wave& w, uint32_t* s_cell, uint32_t* s_unit, uint32_t* s_br) {
    w.s_cell = s_cell;
    w.s_unit = s_unit;
    w.s_br = s_br;
    w.stk = nullptr;
    const int lane = threadIdx.x;
    w.lane = lane;
    w.hasB = lane < 17;
    const int c = lane;
    w.uA0 = c / 9;
    w.uA1 = 9 + c % 9;
    w.uA2 = 18 + (c / 27) * 3 + (c % 9) / 3;
    const int cb = w.hasB ? 64 + lane : 0;
    w.uB0 = cb / 9;
    w.uB1 = 9 + cb % 9;
    w.uB2 = 18 + (cb / 27) * 3 + (cb % 9) / 3;
    const int u = lane < 27 ? lane : 0;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        int cell;
        if (u < 9) cell = 9 * u + k;
        else if (u < 18) cell = 9 * k + (u - 9);
        else {
            const int b = u - 18;
            cell = ((b / 3) * 3 + k / 3) * 9 + (b % 3) * 3 + k % 3;
        }
        w.ucell[k] = cell;
    }
}

#ifndef SDK_NO_SOLVE_KERNEL   // solve2_launch.hip takes the helpers only
__global__ __launch_bounds__(64, 8) void solve_kernel(SolveArgs a) {
    __shared__ uint32_t s_cell[96];
    __shared__ uint32_t s_unit[32];
    __shared__ uint32_t s_br[kMaxDepth];
    Wave w;
    init_wave(w, s_cell, s_unit, s_br);
    w.stk = a.stack + (size_t)blockIdx.x * kStackWordsPerBlock;
    const int lane = w.lane;
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(a.next, a.chunk);
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
        if ((uint64_t)base >= a.n) break;
        const uint64_t end = min((uint64_t)base + a.chunk, a.n);
        for (uint64_t i = base; i < end; ++i) {
            const uint8_t* src = a.in + (a.in_first + i * a.in_step) * 81;
            const uint32_t inA = src[lane];
            const uint32_t inB = w.hasB ? (uint32_t)src[64 + lane] : 0u;
            uint32_t sa = cell_init(inA);
            uint32_t sb = w.hasB ? cell_init(inB) : kInert;
            // TASK `range` restricts the lowest-index empty input cell only (DHT_Node.py:474,522,531)
            const uint32_t fm = a.mask ? (((uint32_t)a.mask[i] >> 1) & kCands) : kCands;
            const unsigned long long za = __ballot(inA == 0);
            const unsigned long long zb = __ballot(w.hasB && inB == 0);
            if (za) {
                if (lane == (int)__builtin_ctzll(za)) sa &= fm | ~kCands;
            } else if (zb) {
                if (lane == (int)__builtin_ctzll(zb)) sb &= fm | ~kCands;
            }
            uint8_t* dst = a.out ? a.out + i * 81 : nullptr;
            uint64_t nodes = 0, rounds = 0, maxd = 0;
            int8_t st;
            // count mode: whole-subtree count (order-independent, so MRV); the
            // batch stops early once the running total reaches the limit.
            // solve mode: MRV search for <= 2 completions, or LEX for the first.
            bool skip = false;
            if (a.count_mode && a.limit) {
                unsigned long long tot = 0;
                if (lane == 0) tot = __hip_atomic_load(a.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                tot = __shfl(tot, 0);
                skip = tot >= a.limit;
            }
            const int order0 = (a.count_mode || a.order != ORDER_LEX) ? ORDER_MRV : ORDER_LEX;
            const uint64_t lim0 = a.count_mode ? a.limit : (order0 == ORDER_LEX ? 1u : 2u);
            int64_t c = 0;
            if (!skip) c = search(w, order0, sa, sb, lim0, a.budget, nodes, rounds, maxd, dst, inA, inB);
            if (!a.count_mode && order0 == ORDER_MRV && c >= 2)
                c = search(w, ORDER_LEX, sa, sb, 1, a.budget, nodes, rounds, maxd, dst, inA, inB);
            if (a.count_mode && lane == 0) {
                if (c > 0) atomicAdd(a.count, (unsigned long long)c);
                if (a.counts) a.counts[i] = (unsigned long long)(c < 0 ? 0 : c);
            }
            st = c < 0 ? (int8_t)-2 : (c > 0 ? (int8_t)1 : (int8_t)0);
            if (dst && c <= 0) write_board(w, dst, inA, inB, sa, sb, false);
            if (lane == 0) {
                if (a.status) a.status[i] = st;
                if (a.work) a.work[i] = a.work_rounds == 1 ? rounds : (a.work_rounds == 2 ? maxd : nodes);
            }
        }
    }
}
#endif  // SDK_NO_SOLVE_KERNEL

}  // namespace sdk
