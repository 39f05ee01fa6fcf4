// expand4_kernel.h -- one frontier expansion level (frontier_kernel.h) on solve4's layout:
// four boards per wavefront, two per 32-lane half in the 16-bit halves of every word.
//
// expand_kernel (frontier_kernel.h) propagates one board per wave with the round-1 solver's
// propagation; this kernel runs solve4's round (round4: the same naked / hidden single rules,
// so the same fixpoint of every board) on four boards at once, then classifies each board and
// picks its branch exactly as expand_kernel does -- contradiction: no child; solved: a leaf
// (count mode) or itself as its only child (first-solution mode); open: the MRV cell (count
// mode) or the lowest open cell (first-solution mode), children in ascending digit order.
// The frontier it builds is therefore the same array, byte for byte (GPU test).  Boards are
// assigned grid-stride, four per wave, with no dequeue atomics.
#pragma once
#include "frontier_args.h"
#include "solve4_kernel.h"

namespace sdk {

// the board of frontier index i into slot HI of this half (inert when !valid)
template <int HI>
__device__ __forceinline__ void expand4_load(const Lane4& w, const ExpandArgs& a, uint64_t i, bool valid, Cells4& c) {
    uint8_t* sin = w.s_in + HI * 81;
    uint32_t i0 = 0u, i1 = 0u, i2 = 0u;
    const bool on = valid && w.act;
    if (on) {
        const uint8_t* src = a.in + i * 81;
        i0 = src[w.c0];
        i1 = src[w.c0 + 27];
        i2 = src[w.c0 + 54];
        sin[w.c0] = (uint8_t)i0;
        sin[w.c0 + 27] = (uint8_t)i1;
        sin[w.c0 + 54] = (uint8_t)i2;
    }
    uint32_t x0 = on ? cell_x4(i0) : 0u, x1 = on ? cell_x4(i1) : 0u, x2 = on ? cell_x4(i2) : 0u;
    const uint32_t s0 = on ? cell_s4(i0) : kInert4, s1 = on ? cell_s4(i1) : kInert4, s2 = on ? cell_s4(i2) : kInert4;
    if (valid && a.mask) {
        // level 0: each board's TASK `range` on its lowest-index empty input cell
        // (DHT_Node.py:474,522,531)
        const uint32_t fm = ((uint32_t)a.mask[i] >> 1) & kCands;
        uint32_t z = ~0u;
        if (w.act) z = i0 == 0 ? (uint32_t)w.c0 : (i1 == 0 ? (uint32_t)w.c0 + 27 : (i2 == 0 ? (uint32_t)w.c0 + 54 : ~0u));
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
}

// classification, branch and propagated board of slot HI (its round ended in an event)
template <int HI>
__device__ __forceinline__ void expand4_out(const Lane4& w, const ExpandArgs& a, uint64_t i, bool contra,
                                            const Cells4& c, uint32_t& nleaves, uint32_t& nopen) {
    const uint32_t x0 = fld<HI>(c.x0), x1 = fld<HI>(c.x1), x2 = fld<HI>(c.x2);
    const uint32_t s0 = fld<HI>(c.s0), s1 = fld<HI>(c.s1), s2 = fld<HI>(c.s2);
    uint32_t nch = 0u, cell = 0u, m = 0u;
    bool write = false;
    if (!contra) {
        const bool open = half_any4(w, w.act && (x0 | x1 | x2) != 0u);
        if (!open) {
            if (a.keep_leaves) {
                nch = 1u;
                m = kKeepBoard;
                write = true;
            } else {
                ++nleaves;
            }
        } else {
            ++nopen;
            if (a.order == ORDER_LEX) {
                int cl;
                uint32_t mm;
                lex_pick4(w, x0, x1, x2, cl, mm);
                cell = (uint32_t)cl;
                m = mm & kCands;
            } else {
                uint32_t key = ~0u;
                if (w.act)
                    key = min(branch_key4(x0, s0, w.c0, ORDER_MRV),
                              min(branch_key4(x1, s1, w.c0 + 27, ORDER_MRV), branch_key4(x2, s2, w.c0 + 54, ORDER_MRV)));
                key = half_min(key);
                cell = (key >> 9) & 0x7Fu;
                m = key & kCands;
            }
            nch = (uint32_t)__popc(m);
            write = true;
        }
    }
    if (write && w.act) {
        // givens keep their byte, closed cells become givens, open cells stay 0 (board_byte)
        const uint8_t* sin = w.s_in + HI * 81;
        uint8_t* dst = a.prop + i * 81;
        const uint32_t i0 = sin[w.c0], i1 = sin[w.c0 + 27], i2 = sin[w.c0 + 54];
        dst[w.c0] = (uint8_t)(i0 ? i0 : (x0 ? 0u : (uint32_t)__ffs(s0)));
        dst[w.c0 + 27] = (uint8_t)(i1 ? i1 : (x1 ? 0u : (uint32_t)__ffs(s1)));
        dst[w.c0 + 54] = (uint8_t)(i2 ? i2 : (x2 ? 0u : (uint32_t)__ffs(s2)));
    }
    if (w.hl == 0) {
        a.nchild[i] = nch;
        a.bcell[i] = (uint8_t)cell;
        a.bmask[i] = (uint16_t)m;
    }
}

#ifdef SDK_DEFINE_SOLVE4_KERNEL
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SDK_SOLVE4_WAVES_PER_EU))) void expand4_kernel(ExpandArgs a) {
    __shared__ uint2 s_region[2 * kRegion4];
    __shared__ uint8_t s_in[2 * 2 * 81];
    if (a.ctl->done) return;
    const uint64_t m = a.ctl->m;
    Lane4 w;
    init_lane4(w, s_region, s_in);
    // the level's leaves and branching boards, counted per half and added once per wave at the
    // end: one same-address atomic per board serialized (~10 ns each) and bound the level
    uint32_t nleaves = 0u, nopen = 0u;
    for (uint64_t base = (uint64_t)blockIdx.x * 4u; base < m; base += (uint64_t)gridDim.x * 4u) {
        const uint64_t i0 = base + 2u * (uint64_t)w.half, i1 = i0 + 1u;   // this half's slots 0 and 1
        const bool v0 = i0 < m, v1 = i1 < m;
        Cells4 c;
        c.x0 = c.x1 = c.x2 = 0u;
        c.s0 = c.s1 = c.s2 = kInert4x2;
        c.D = kC2;
        c.E = 0u;
        expand4_load<0>(w, a, i0, v0, c);
        expand4_load<1>(w, a, i1, v1, c);
        statics4<0>(w, c);
        statics4<1>(w, c);
        // rounds until every slot's board met its event (contradiction, or a round that changed
        // nothing: a fixpoint stays one); contradictions are latched at their first round
        uint64_t act0 = spread_halves(__builtin_amdgcn_ballot_w64(v0)), act1 = spread_halves(__builtin_amdgcn_ballot_w64(v1));
        uint64_t con0 = 0, con1 = 0;
        while ((act0 | act1) != 0) {
            uint32_t badw, chg;
            round4<false>(w, c, badw, chg);
            const uint64_t B0 = spread_halves(__builtin_amdgcn_ballot_w64((badw & 0xFFFFu) != 0u));
            const uint64_t B1 = spread_halves(__builtin_amdgcn_ballot_w64(badw > 0xFFFFu));
            const uint64_t C0 = spread_halves(__builtin_amdgcn_ballot_w64((chg & 0xFFFFu) != 0u));
            const uint64_t C1 = spread_halves(__builtin_amdgcn_ballot_w64(chg > 0xFFFFu));
            const uint64_t E0 = act0 & (B0 | ~C0), E1 = act1 & (B1 | ~C1);
            con0 |= E0 & B0;
            con1 |= E1 & B1;
            act0 &= ~E0;
            act1 &= ~E1;
        }
        if (v0) expand4_out<0>(w, a, i0, __builtin_amdgcn_inverse_ballot_w64(con0), c, nleaves, nopen);
        if (v1) expand4_out<1>(w, a, i1, __builtin_amdgcn_inverse_ballot_w64(con1), c, nleaves, nopen);
    }
    const uint32_t tl = __builtin_amdgcn_readlane(nleaves, 0) + __builtin_amdgcn_readlane(nleaves, 32);
    const uint32_t to = __builtin_amdgcn_readlane(nopen, 0) + __builtin_amdgcn_readlane(nopen, 32);
    if (threadIdx.x == 0 && tl) atomicAdd(&a.ctl->lvl_leaves, (unsigned long long)tl);
    if (threadIdx.x == 0 && to) atomicAdd(&a.ctl->open, (unsigned long long)to);
}
#endif

}  // namespace sdk
