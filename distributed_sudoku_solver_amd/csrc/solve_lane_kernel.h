// solve_lane_kernel.h -- DHTNode.solve_sudoku (DHT_Node.py:474-538) as the reference
// runs it, ONE BOARD PER LANE: the bounded per-lane DFS with an LDS-resident stack.
//
// Each lane runs the reference's naive DFS on its own board, step by step:
// the lowest empty cell (find_next_empty, utils.py:14-25), digits ascending, a
// guess accepted when it is in none of the cell's row, column and box
// (is_valid, utils.py:27-56, restated as per-unit digit masks), restore on
// failure (DHT_Node.py:535).  Because the DFS only ever fills the next empty
// cell of the input, its whole stack is the digit placed in each empty cell:
// that array (a nibble per cell) and the 27 unit masks live in LDS, lane-
// interleaved ([entry][lane]), 6 KB per wave; registers hold the current cell,
// the input's empty-cell bitmap and the counters.  One step = one level of the
// reference's recursion: take back this level's digit if any, place the next
// allowed digit and move to the next empty cell, or move back to the previous one.
//
// `work` counts exactly the reference's `validations` (+1 for the top-level
// call, +2 per placement: DHT_Node.py:513,527-531 -- the oracle's orc_naive_solve
// and the golden fixtures' counts), and the node budget is a budget of
// validations, checked where the oracle checks it, so statuses agree exactly.
//
// Lanes that finish (solved, exhausted, budget) write their board and are refilled
// together: one atomic per wave takes as many new boards as lanes are free.
//
// This is the design the north star's part (3) names; DESIGN.md compares it with
// the propagating solvers (it executes the reference's search, millions of
// validations per 17-clue board, where solve4 needs ~25 propagation rounds).
#pragma once
#include "solve_kernel.h"

namespace sdk {

constexpr int kLaneThreads = 256;          // 4 independent waves per workgroup
constexpr int kLaneSteps = 32;             // DFS steps between refills
constexpr uint32_t kLaneAll = 0x3FEu;      // digits 1..9 as bits 1..9 (the oracle's layout)

struct LaneLds {
    uint16_t mask[27][64];                 // units: rows 0..8, columns 9..17, boxes 18..26
    uint8_t dig[41][64];                   // digit placed in cell c: nibble c & 1 of byte c >> 1
};

__device__ __forceinline__ uint32_t lane_row(uint32_t p) { return (p * 57u) >> 9; }   // p / 9 for p < 81
__device__ __forceinline__ uint32_t lane_div3(uint32_t x) { return (x * 11u) >> 5; }  // x / 3 for x < 9

#ifdef SDK_DEFINE_LANE_KERNEL
__global__ __launch_bounds__(kLaneThreads) void solve_lane_kernel(SolveArgs a) {
    __shared__ LaneLds s_lane[kLaneThreads / 64];
    const int lane = threadIdx.x & 63;
    LaneLds& L = s_lane[threadIdx.x >> 6];

    uint64_t bidx = 0, val = 0;
    uint64_t elo = 0, ehi = 0;             // empty cells of the input: 0..63, 64..80
    uint32_t p = 0, first = 0, fm = kLaneAll;
    bool live = false;                     // a board is being searched
    bool fin = false;                      // finished, results not yet written
    int st = 0;
    bool more = true;                      // the queue may still hold boards (wave-uniform)

    for (;;) {
        // ---- write finished boards, take new ones (all lanes that are free) ----
        if (fin) {
            const uint8_t* src = a.in + (a.in_first + bidx * a.in_step) * 81;
            uint8_t* dst = a.out + bidx * 81;
            for (int i = 0; i < 81; ++i) {
                uint32_t v = src[i];
                if (st == 1 && v == 0) {
                    const uint32_t byte = L.dig[i >> 1][lane];
                    v = (i & 1) ? (byte >> 4) : (byte & 15u);
                }
                dst[i] = (uint8_t)v;       // status 1: the completion; else the input (restored)
            }
            a.status[bidx] = (int8_t)st;
            if (a.work) a.work[bidx] = val;
            fin = false;
        }
        if (more) {
            const uint64_t freem = __builtin_amdgcn_ballot_w64(!live);
            if (freem) {
                uint32_t base = 0;
                const int leader = __builtin_ctzll(freem);
                if (lane == leader) base = atomicAdd(a.next, (uint32_t)__popcll(freem));
                base = __builtin_amdgcn_readlane(base, leader);
                if ((uint64_t)base + __popcll(freem) >= a.n) more = false;
                if (!live) {
                    const uint64_t idx = (uint64_t)base + __popcll(freem & ((1ull << lane) - 1));
                    if (idx < a.n) {
                        // start: masks and empties from the input givens (10..255 are inert:
                        // never equal to a guess, as in the reference's equality test)
                        bidx = idx;
                        const uint8_t* src = a.in + (a.in_first + bidx * a.in_step) * 81;
                        uint32_t m[27];
#pragma unroll
                        for (int u = 0; u < 27; ++u) m[u] = 0;
                        elo = ehi = 0;
#pragma unroll
                        for (int i = 0; i < 81; ++i) {
                            const uint32_t v = src[i];
                            const uint32_t bit = (v >= 1 && v <= 9) ? (1u << v) : 0u;
                            m[i / 9] |= bit;
                            m[9 + i % 9] |= bit;
                            m[18 + (i / 27) * 3 + (i % 9) / 3] |= bit;
                            if (v == 0) {
                                if (i < 64) elo |= 1ull << i;
                                else ehi |= 1ull << (i - 64);
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 27; ++u) L.mask[u][lane] = (uint16_t)m[u];
#pragma unroll
                        for (int k = 0; k < 41; ++k) L.dig[k][lane] = 0;
                        val = 1;                   // the top-level call (DHT_Node.py:513)
                        fm = a.mask ? ((uint32_t)a.mask[bidx] & kLaneAll) : kLaneAll;
                        if (elo | ehi) {
                            first = elo ? (uint32_t)__builtin_ctzll(elo) : 64u + (uint32_t)__builtin_ctzll(ehi);
                            p = first;
                            live = true;
                        } else {                   // no empty cell: solved as given
                            st = 1;
                            fin = true;
                        }
                    }
                }
            }
        }
        if (__builtin_amdgcn_ballot_w64(live || fin) == 0 && !more) break;
        // ---- DFS steps ----
#pragma nounroll
        for (int k = 0; k < kLaneSteps; ++k) {
            if (live) {
                if (a.budget && val > a.budget) {
                    st = -2;
                    live = false;
                    fin = true;
                } else {
                    const uint32_t r = lane_row(p), c = p - 9u * r, b = lane_div3(r) * 3u + lane_div3(c);
                    uint8_t& db = L.dig[p >> 1][lane];
                    const uint32_t byte = db, sh = (p & 1u) * 4u;
                    const uint32_t d = (byte >> sh) & 15u;
                    const uint32_t dbit = d ? (1u << d) : 0u;
                    uint32_t mr = L.mask[r][lane] & ~dbit, mc = L.mask[9 + c][lane] & ~dbit,
                             mb = L.mask[18 + b][lane] & ~dbit;
                    const uint32_t allowed = p == first ? fm : kLaneAll;
                    const uint32_t cand = allowed & ~(mr | mc | mb) & ~((2u << d) - 1u);   // digits above d
                    uint32_t g = 0;
                    if (cand) {                    // place the next digit (DHT_Node.py:527-531)
                        g = (uint32_t)__builtin_ctz(cand);
                        const uint32_t gb = 1u << g;
                        mr |= gb;
                        mc |= gb;
                        mb |= gb;
                        val += 2;                  // +1 placement, +1 for the callee's entry
                    }
                    L.mask[r][lane] = (uint16_t)mr;
                    L.mask[9 + c][lane] = (uint16_t)mc;
                    L.mask[18 + b][lane] = (uint16_t)mb;
                    db = (uint8_t)((byte & ~(15u << sh)) | (g << sh));
                    if (cand) {                    // the next empty cell, or solved
                        const uint32_t q = p + 1;
                        const uint64_t lo = q < 64 ? (elo & (~0ull << q)) : 0ull;
                        const uint64_t hi = q < 64 ? ehi : (q < 81 ? (ehi & (~0ull << (q - 64))) : 0ull);
                        if (lo) p = (uint32_t)__builtin_ctzll(lo);
                        else if (hi) p = 64u + (uint32_t)__builtin_ctzll(hi);
                        else {
                            st = 1;
                            live = false;
                            fin = true;
                        }
                    } else {                       // exhausted: back to the previous empty cell
                        const uint64_t lo = p < 64 ? (elo & ((1ull << p) - 1ull)) : elo;
                        const uint64_t hi = p < 64 ? 0ull : (ehi & ((1ull << (p - 64)) - 1ull));
                        if (hi) p = 64u + 63u - (uint32_t)__builtin_clzll(hi);
                        else if (lo) p = 63u - (uint32_t)__builtin_clzll(lo);
                        else {
                            st = 0;
                            live = false;
                            fin = true;
                        }
                    }
                }
            }
            if (__builtin_amdgcn_ballot_w64(live) == 0) break;
        }
    }
}
#endif  // SDK_DEFINE_LANE_KERNEL

}  // namespace sdk
