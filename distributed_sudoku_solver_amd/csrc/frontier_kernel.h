// frontier_kernel.h -- breadth-first frontier expansion for whole-tree searches
// (solution counting).
//
// One expansion level turns a frontier of boards into the boards of their
// children, deterministically (same order on every GPU, so a replicated
// frontier can be sliced across GPUs without an exchange):
//   expand_kernel  one wave per board: propagate (solve_kernel.h), then
//                  CONTRA -> 0 children; SOLVED -> 0 children and one leaf;
//                  OPEN -> branch on the MRV cell, nchild = #candidates.  The
//                  propagated board is written back with every single-valued
//                  cell as a given (a fixpoint has no conflict among them, so
//                  treating them as givens changes no completion).
//   scan_tiles_kernel + scan_top_kernel   exclusive prefix sum of nchild over
//                  the whole chip: every workgroup scans 4096-entry tiles
//                  (wave __shfl_up scans + LDS for the wave totals) and writes
//                  the tile total; one workgroup then scans the tile totals.
//   emit_kernel    one wave per parent writes its children contiguously at
//                  offset[parent] + tile offset, digits ascending: children of
//                  one parent and parents in order -> a coalesced, ordered HBM array.
// The level loop runs on the device: every kernel reads the frontier size and a
// stop flag from FrontierCtl (frontier_begin/end_kernel update them), so the host
// enqueues levels without waiting and reads the control block every few levels.
//   first_hit_kernel  after a batched solve of frontier boards [lo, hi): the
//                  lowest index whose status is not "no solution" (nor "cancelled": above a
//                  lower hit, kStCancelled) and its board.
//
// First-solution mode (keep_leaves): a board that propagates to SOLVED stays in
// the frontier as its own single child instead of being counted, and the branch
// cell is the lowest-index open cell (ORDER_LEX) with children in ascending digit
// order.  Every cell before the branch cell is forced, so the frontier in index
// order is sorted by the completions below each board: the reference's lex-first
// solution (DHT_Node.py:474-538) is the lex-first completion of the lowest-index
// frontier board that has one.
#pragma once
#include "solve_kernel.h"
#include "frontier_args.h"

namespace sdk {

__device__ __forceinline__ uint32_t board_byte(uint32_t in, uint32_t s) {
    // givens keep their byte; single-valued cells become givens; open cells stay 0
    if (in) return in;
    const uint32_t v = s & kCands;
    return is_single(v) ? (uint32_t)__ffs(v) : 0u;
}

// level start: stop when the frontier is empty or reached `target` (level 0 with a
// first-cell mask always runs: the mask lives only in that level's expansion)
__global__ void frontier_begin_kernel(FrontierCtl* ctl, uint64_t target, int force) {
    if (ctl->done) return;
    if (ctl->m == 0 || (ctl->m >= target && !force) || ctl->level >= 81) {
        ctl->done = 1;
        return;
    }
    ctl->next = 0;
    ctl->open = 0;
    ctl->lvl_leaves = 0;
}

// level end: the children become the frontier; first-solution mode stops when nothing
// branched (the next level would equal this one)
__global__ void frontier_end_kernel(FrontierCtl* ctl, int first) {
    if (ctl->done) return;   // also a level that scan_top_kernel rejected: its leaves are dropped, its
                             // parents (which contain them) stay the frontier
    ctl->m = ctl->total;
    ctl->leaves += ctl->lvl_leaves;
    ctl->level += 1;
    if (ctl->total == 0 || (first && ctl->open == 0)) ctl->done = 1;
}

__global__ __launch_bounds__(64) void expand_kernel(ExpandArgs a) {
    __shared__ uint32_t s_cell[96];
    __shared__ uint32_t s_unit[32];
    __shared__ uint32_t s_br[4];
    if (a.ctl->done) return;
    const uint64_t m_lvl = a.ctl->m;
    Wave w;
    init_wave(w, s_cell, s_unit, s_br);
    const int lane = w.lane;
    // the level's leaves and branching boards, counted per wave and added once at the end
    // (one same-address atomic per board serialized at ~10 ns)
    unsigned long long nleaves = 0, nopen = 0;
    for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&a.ctl->next, kChunk);
        base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
        if ((uint64_t)base >= m_lvl) break;
        const uint64_t end = min((uint64_t)base + kChunk, m_lvl);
        for (uint64_t i = base; i < end; ++i) {
            const uint8_t* src = a.in + i * 81;
            const uint32_t inA = src[lane];
            const uint32_t inB = w.hasB ? (uint32_t)src[64 + lane] : 0u;
            uint32_t sa = cell_init(inA);
            uint32_t sb = w.hasB ? cell_init(inB) : kInert;
            if (a.mask) {
                // TASK `range` on the lowest-index empty input cell (DHT_Node.py:474,522,531)
                const uint32_t fm = ((uint32_t)a.mask[i] >> 1) & kCands;
                const unsigned long long za = __ballot(inA == 0);
                const unsigned long long zb = __ballot(w.hasB && inB == 0);
                if (za) {
                    if (lane == (int)__builtin_ctzll(za)) sa &= fm | ~kCands;
                } else if (zb) {
                    if (lane == (int)__builtin_ctzll(zb)) sb &= fm | ~kCands;
                }
            }
            uint64_t rounds = 0;
            const int r = propagate(w, sa, sb, rounds);
            uint32_t nch = 0, cell = 0, m = 0;
            if (r == P_SOLVED) {
                if (a.keep_leaves) {
                    nch = 1;
                    m = kKeepBoard;
                    uint8_t* dst = a.prop + i * 81;
                    dst[lane] = (uint8_t)board_byte(inA, sa);
                    if (w.hasB) dst[64 + lane] = (uint8_t)board_byte(inB, sb);
                } else {
                    ++nleaves;
                }
            } else if (r == P_OPEN) {
                ++nopen;
                const uint32_t pa = open_count(sa);
                const uint32_t pb = w.hasB ? open_count(sb) : 0u;
                unsigned long long ma, mb;
                if (a.order == ORDER_LEX) {
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
                cell = ma ? (uint32_t)__builtin_ctzll(ma) : 64u + (uint32_t)__builtin_ctzll(mb);
                const uint32_t mA = (uint32_t)__builtin_amdgcn_readlane((int)sa, (int)(cell & 63));
                const uint32_t mB = (uint32_t)__builtin_amdgcn_readlane((int)sb, (int)(cell & 63));
                m = (cell < 64 ? mA : mB) & kCands;
                nch = (uint32_t)__popc(m);
                uint8_t* dst = a.prop + i * 81;
                dst[lane] = (uint8_t)board_byte(inA, sa);
                if (w.hasB) dst[64 + lane] = (uint8_t)board_byte(inB, sb);
            }
            if (lane == 0) {
                a.nchild[i] = nch;
                a.bcell[i] = (uint8_t)cell;
                a.bmask[i] = (uint16_t)m;
            }
        }
    }
    if (lane == 0 && nleaves) atomicAdd(&a.ctl->lvl_leaves, nleaves);
    if (lane == 0 && nopen) atomicAdd(&a.ctl->open, nopen);
}

// Tile-local exclusive scan: tile t = entries [t*4096, (t+1)*4096) of nchild[0..m);
// off[i] = prefix within the tile, tsum[t] = tile total.  Grid-stride over tiles.
__global__ __launch_bounds__(1024) void scan_tiles_kernel(const uint32_t* __restrict__ cnt, uint64_t* __restrict__ off,
                                                          const FrontierCtl* ctl, uint64_t* __restrict__ tsum) {
    __shared__ uint32_t s_wave[16];
    if (ctl->done) return;
    const uint64_t n = ctl->m;
    const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const uint64_t i0 = tile * kScanTile + 4u * (uint64_t)t;
        uint32_t x[4], own = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            x[k] = i0 + k < n ? cnt[i0 + k] : 0u;
            own += x[k];
        }
        uint32_t inc = own;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)inc, d);
            if (lane >= d) inc += y;
        }
        if (lane == 63) s_wave[wv] = inc;
        __syncthreads();
        uint32_t wbase = 0, all = 0;
        for (int k = 0; k < 16; ++k) {
            wbase += k < wv ? s_wave[k] : 0u;
            all += s_wave[k];
        }
        uint32_t run = wbase + inc - own;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (i0 + k < n) off[i0 + k] = run;
            run += x[k];
        }
        if (t == 0) tsum[tile] = all;
        __syncthreads();
    }
}

// Exclusive scan of the tile totals in place (one workgroup); the level's child count
// goes to ctl->total, and a level whose children exceed `cap` boards stops the build
// (the frontier stays the current one).
__global__ __launch_bounds__(1024) void scan_top_kernel(uint64_t* __restrict__ tsum, FrontierCtl* ctl, uint64_t cap) {
    __shared__ uint64_t s_wave[16];
    __shared__ uint64_t s_carry;
    if (ctl->done) return;
    const uint64_t n = (ctl->m + kScanTile - 1) / kScanTile;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) s_carry = 0;
    __syncthreads();
    for (uint64_t base = 0; base < n; base += 1024) {
        const uint64_t i = base + t;
        const uint64_t x = i < n ? tsum[i] : 0;
        uint64_t inc = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(inc, d);
            if (lane >= d) inc += y;
        }
        if (lane == 63) s_wave[wv] = inc;
        __syncthreads();
        uint64_t wbase = 0;
        for (int k = 0; k < wv; ++k) wbase += s_wave[k];
        const uint64_t carry = s_carry;
        if (i < n) tsum[i] = carry + wbase + inc - x;
        __syncthreads();
        if (t == 1023) s_carry = carry + wbase + inc;
        __syncthreads();
    }
    if (t == 0) {
        ctl->total = s_carry;
        if (s_carry > cap) ctl->done = 1;
    }
}

__global__ __launch_bounds__(64) void emit_kernel(const uint8_t* __restrict__ prop, const uint8_t* __restrict__ bcell,
                                                  const uint16_t* __restrict__ bmask, const uint64_t* __restrict__ off,
                                                  const uint64_t* __restrict__ tsum, const FrontierCtl* ctl,
                                                  uint8_t* __restrict__ out) {
    if (ctl->done) return;
    const uint64_t m = ctl->m;
    const int lane = threadIdx.x;
    const bool hasB = lane < 17;
    for (uint64_t i = blockIdx.x; i < m; i += gridDim.x) {
        uint32_t mask = bmask[i];
        if (!mask) continue;
        const uint32_t a = prop[i * 81 + lane];
        const uint32_t b = hasB ? prop[i * 81 + 64 + lane] : 0u;
        uint64_t j = off[i] + tsum[i / kScanTile];
        if (mask & kKeepBoard) {   // solved leaf kept in place (first-solution mode)
            uint8_t* dst = out + j * 81;
            dst[lane] = (uint8_t)a;
            if (hasB) dst[64 + lane] = (uint8_t)b;
            continue;
        }
        const uint32_t cell = bcell[i];
        while (mask) {
            const uint32_t d = (uint32_t)__ffs(mask);  // digit
            mask &= mask - 1;
            uint8_t* dst = out + j * 81;
            dst[lane] = (uint8_t)((uint32_t)lane == cell ? d : a);
            if (hasB) dst[64 + lane] = (uint8_t)((uint32_t)(64 + lane) == cell ? d : b);
            ++j;
        }
    }
}

// status[0..n) of frontier boards lo .. lo+n-1 (dense).  found <- lo + the first i
// whose status is not 0 (solved, or budget hit: either ends a lex-ordered scan),
// INT64_MAX if none; best[0..80] <- that board's output, best[81] <- its status.
// out[k] = in[first + k * step] (81-byte boards), k < n: a rank's share of a frontier
__global__ __launch_bounds__(256) void gather_boards_kernel(const uint8_t* __restrict__ in, uint64_t first,
                                                            uint64_t step, uint64_t n, uint8_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n * 81; i += (uint64_t)gridDim.x * 256) {
        const uint64_t b = i / 81, k = i - b * 81;
        out[i] = in[(first + b * step) * 81 + k];
    }
}

// the found word of a first-solution scan before its solve launch (no hit yet)
__global__ void first_init_kernel(long long* found) { *found = 0x7FFFFFFFFFFFFFFFll; }

__global__ __launch_bounds__(256) void first_hit_kernel(const int8_t* __restrict__ status,
                                                        const uint8_t* __restrict__ out, uint64_t n, uint64_t lo,
                                                        long long* found, uint8_t* best) {
    __shared__ unsigned long long s_min[4];
    const int t = threadIdx.x;
    unsigned long long mine = ~0ull;
    for (uint64_t i = t; i < n; i += 256)
        if (status[i] != 0 && status[i] != kStCancelled) { mine = i; break; }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mine = min(mine, (unsigned long long)__shfl_xor(mine, d));
    if ((t & 63) == 0) s_min[t >> 6] = mine;
    __syncthreads();
    const unsigned long long first = min(min(s_min[0], s_min[1]), min(s_min[2], s_min[3]));
    if (first == ~0ull) {
        if (t == 0) *found = 0x7FFFFFFFFFFFFFFFll;
        return;
    }
    if (t < 81) best[t] = out[first * 81 + t];
    if (t == 81) best[81] = (uint8_t)status[first];
    if (t == 0) *found = (long long)(lo + first);
}

// d_result <- {*count, number of status == -2 (node budget hit)} for n count-mode boards.
__global__ __launch_bounds__(256) void count_result_kernel(const int8_t* __restrict__ status, uint64_t n,
                                                           const unsigned long long* count,
                                                           unsigned long long* result) {
    __shared__ unsigned long long s_hits[4];
    const int t = threadIdx.x;
    unsigned long long hits = 0;
    for (uint64_t i = t; i < n; i += 256) hits += status[i] == -2;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) hits += __shfl_xor(hits, d);
    if ((t & 63) == 0) s_hits[t >> 6] = hits;
    __syncthreads();
    if (t == 0) {
        result[0] = *count;
        result[1] = s_hits[0] + s_hits[1] + s_hits[2] + s_hits[3];
    }
}

}  // namespace sdk
