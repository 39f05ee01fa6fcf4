// sudoku_hip.hip -- libsudoku_hip.so: C-ABI (include/sudoku_hip.h) over the gfx950 kernels.
//
// Host side is deliberately thin: a context = (device, stream, grow-only device
// workspaces, HIP event pairs for kernel timing, options) behind a mutex.  No
// CPU compute path exists: every board is checked / solved by a HIP kernel.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/sudoku_hip.h"
#include "check_kernel.h"
#include "solve_kernel.h"
#include "frontier_kernel.h"
#include "solve2_kernel.h"   // constants only: the kernel lives in solve2_launch.hip
#include "solve4_kernel.h"   // constants only: the kernel lives in solve4_launch.hip
#include "prop32_kernel.h"   // constants only: the kernel lives in prop32_launch.hip
#define SDK_DEFINE_LANE_KERNEL
#include "solve_lane_kernel.h"

namespace sdk {
hipError_t launch_solve2(const SolveArgs& a, unsigned grid, hipStream_t stream);
hipError_t launch_solve4(const SolveArgs& a, unsigned grid, hipStream_t stream);
int solve4_dn_blocks_per_cu();   // resident workgroups per CU of solve4_kernel<true>
hipError_t launch_prop32(const Prop32Args& a, unsigned grid, hipStream_t stream, uint64_t* stamps);
hipError_t launch_p32_scatter(const uint32_t* list, const uint8_t* sub_out, const int8_t* sub_st, const uint8_t* in,
                              uint8_t* out, int8_t* status, unsigned grid, hipStream_t stream);
hipError_t launch_expand4(const ExpandArgs& a, unsigned grid, hipStream_t stream);   // expand4_kernel.h
}

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIPCALL(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? SDK_ENOMEM : SDK_EHIP, "%s: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                    \
    } while (0)

constexpr size_t kMaxTimedLaunches = 1u << 16;

// A device allocation owned by its holder: freed when the holder goes (sdk_destroy deletes the
// context after selecting its device), so no buffer added to sdk_ctx can leak.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) {
        o.p = nullptr;
        o.bytes = 0;
    }
    DevBuf& operator=(DevBuf&& o) noexcept {      // (std::swap of two buffers moves through this)
        if (this != &o) {
            if (p) (void)hipFree(p);
            p = o.p;
            bytes = o.bytes;
            o.p = nullptr;
            o.bytes = 0;
        }
        return *this;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(bytes, o.bytes);
    }
};

// A host-pointer call that staged through the pinned area: an error return may leave copies
// from / into it queued, so drain the stream first -- the next call's memcpy into the area (or a
// grow that frees it) cannot race them.  Disarmed once the call has synchronized.
struct DrainOnError {
    hipStream_t s;
    bool armed;
    ~DrainOnError() {
        if (armed) (void)hipStreamSynchronize(s);
    }
};

}  // namespace

namespace sdk {
// two-phase solve (launch_solve): list the split phase's budget hits, gather them into a
// dense batch, scatter their answers back
// A list is a length word and the board indices after it; its length is read on the device
// (the phases are enqueued without the host).  Collecting a board also copies it (and its
// first-cell mask) to the list's position in the next phase's dense input: the boards
// listed are a launch's tail, a few per thousand, so one thread per board does.  n_dev
// (nullable) bounds n by an earlier list.
// Resuming (`save` non-null, the split phase's list): a board whose stack the split phase left
// (SplitSave, validated by its header) goes to the seed list instead -- (board, save entry)
// pairs after a length word, with the words the records and items it needs reserved in the
// donation area's DnSeed -- and dn_seed_kernel lists it after the restarted ones; `rcount`
// counts the restarted boards alone (the donation launch's dequeue).
struct DnResume {
    const SplitSave* save;
    const uint32_t* save_idx;
    DnCtl* ctl;
    uint32_t* seeds;          // [0] seeded boards, [1] restarted boards, then (board, entry) pairs
};
__global__ void dn_collect_kernel(const int8_t* status, uint64_t n, const uint32_t* n_dev, int8_t code,
                                  uint32_t* list, uint32_t* total, const uint8_t* in, const uint16_t* mask,
                                  uint64_t in_first, uint64_t in_step, uint8_t* out, uint16_t* out_mask, DnResume rs) {
    if (n_dev) n = min<uint64_t>(n, *n_dev);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (status[i] == code) {
            if (rs.save) {
                const uint32_t e = rs.save_idx[i];
                if (e < min(rs.save->count, kSaveCap) && rs.save->hdr[e].x == (uint32_t)i) {
                    // items: the deepest level's current digit and every level's untried ones
                    const uint32_t depth = rs.save->hdr[e].y;
                    uint32_t items = 1;
                    for (uint32_t l = 0; l < depth; ++l) items += (uint32_t)__popc(rs.save->lv[e][l][0].y >> 23);
                    // reserve a board slot, then the items by compare-and-swap: a reservation is
                    // committed only when it fits, and a board whose items do not fit gives its
                    // slot back -- one deep stack does not use up the room of later small ones
                    // (two unconditional adds consumed both on a failed reservation)
                    bool fits = false;
                    if (atomicAdd(&rs.ctl->seed.res_boards, 1u) < kSeedBoards) {
                        uint32_t cur = __hip_atomic_load(&rs.ctl->seed.res_items, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                        while (cur + items <= kSeedItems) {
                            const uint32_t prev = atomicCAS(&rs.ctl->seed.res_items, cur, cur + items);
                            if (prev == cur) {
                                fits = true;
                                break;
                            }
                            cur = prev;
                        }
                    }
                    if (!fits) atomicSub(&rs.ctl->seed.res_boards, 1u);
                    if (fits) {
                        const uint32_t s = atomicAdd(rs.seeds, 1u);
                        rs.seeds[2 + 2 * s] = (uint32_t)i;
                        rs.seeds[3 + 2 * s] = e;
                        continue;
                    }
                }
                atomicAdd(rs.seeds + 1, 1u);
            }
            const uint32_t k = atomicAdd(list, 1u);
            list[1 + k] = (uint32_t)i;
            atomicAdd(total, 1u);
            const uint8_t* src = in + (in_first + i * in_step) * 81;
            uint8_t* dst = out + (uint64_t)k * 81;
            for (int j = 0; j < 81; ++j) dst[j] = src[j];
            if (mask) out_mask[k] = mask[i];
        }
}
// A phased solve's control words, zeroed in one launch before its first phase: the split
// phase's dequeue counter and heads, the statistics, both donation launches' control blocks
// (their epochs set) and list lengths.
struct DnPrep {
    uint32_t* counter;
    uint32_t* heads;
    uint32_t heads_words;
    uint32_t* stat;
    uint32_t* ctl[2];
    uint32_t epoch[2];
    uint32_t fault;      // DnCtl.fault (SDK_OPT_DN_FAULT, test only)
    uint32_t helpers;    // DnCtl.helpers (SDK_OPT_DONATE_HELPERS)
    uint32_t* list[2];
    uint32_t* seeds;     // the seed list's two length words (nullable)
    uint32_t* save;      // SplitSave::count (nullable)
};
__global__ void dn_prep_kernel(DnPrep p) {
    const uint32_t t = threadIdx.x;
    if (t == 0) {
        p.counter[0] = 0;
        p.list[0][0] = 0;
        p.list[1][0] = 0;
        if (p.seeds) p.seeds[0] = p.seeds[1] = 0;
        if (p.save) p.save[0] = 0;
    }
    if (p.stat && t < 2) p.stat[t] = 0;
    if (p.heads)
        for (uint32_t i = t; i < p.heads_words; i += blockDim.x) p.heads[i] = 0;
    // every word but the sticky error word (the host reads and clears it after the solve)
    constexpr uint32_t kEpoch = offsetof(DnCtl, epoch) / 4, kErr = offsetof(DnCtl, err) / 4,
                       kFault = offsetof(DnCtl, fault) / 4, kHelpers = offsetof(DnCtl, helpers) / 4;
    for (int k = 0; k < 2; ++k)
        for (uint32_t i = t; i < sizeof(DnCtl) / 4; i += blockDim.x)
            if (i != kErr)
                p.ctl[k][i] = i == kEpoch ? p.epoch[k] : (i == kFault ? p.fault : (i == kHelpers ? p.helpers : 0u));
}
// The resumed boards (dn_collect_kernel's seed list), one workgroup of 64 each: listed after the
// restarted boards (input and mask copied to the dense batch like theirs), a board record with
// one open part per item, and the items -- each level's snapshot with its branch cell set to
// one open digit (the deepest level: also the digit it was searching) -- appended to the
// seed queue, shallowest level first (the largest subtrees start first).
__global__ void dn_seed_kernel(const uint32_t* seeds, const SplitSave* save, uint32_t* list, uint32_t* total,
                               const uint8_t* in, const uint16_t* mask, uint64_t in_first, uint64_t in_step,
                               uint8_t* out, uint16_t* out_mask, DnCtl* ctl) {
    __shared__ uint32_t sh[4];
    const uint32_t t = threadIdx.x;
    DnRec* recs = reinterpret_cast<DnRec*>(reinterpret_cast<char*>(ctl) + kDnRecOffset);
    DnItem* items = reinterpret_cast<DnItem*>(reinterpret_cast<char*>(ctl) + kDnItemOffset);
    uint32_t* seedq = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(ctl) + kDnSeedQOffset);
    const uint32_t ns = min(seeds[0], kSeedBoards);
    for (uint32_t s = blockIdx.x; s < ns; s += gridDim.x) {
        const uint32_t i = seeds[2 + 2 * s], e = seeds[3 + 2 * s];
        const uint32_t depth = save->hdr[e].y;
        uint32_t nit = 1;
        for (uint32_t l = 0; l < depth; ++l) nit += (uint32_t)__popc(save->lv[e][l][0].y >> 23);
        if (t == 0) {
            sh[0] = atomicAdd(list, 1u);
            sh[1] = atomicAdd(&ctl->nrec, 1u);
            sh[2] = atomicAdd(&ctl->item_alloc, nit);
            sh[3] = atomicAdd(&ctl->seed.total, nit);
            atomicAdd(total, 1u);
        }
        __syncthreads();
        const uint32_t k = sh[0], r = sh[1], i0 = sh[2], q0 = sh[3];
        if (t == 0) list[1 + k] = i;
        const uint8_t* src = in + (in_first + (uint64_t)i * in_step) * 81;
        for (uint32_t j = t; j < 81; j += blockDim.x) out[(uint64_t)k * 81 + j] = src[j];
        if (t == 0 && mask) out_mask[k] = mask[i];
        DnRec* R = recs + r;
        if (t == 0) {
            R->board = k;
            R->open = nit;
            R->nhit = R->flags = R->maxd = R->lock = R->version = R->have = 0;
            R->work = 0;
            R->total = 0;
            R->first = kDnNone;
        }
        if (t < (uint32_t)kDnList) R->hit[t] = kDnNone;
        // lane t < 27 of the half owns cells t, t + 27, t + 54: one snapshot word each
        uint32_t q = 0;
        for (uint32_t l = 0; l < depth; ++l) {
            const uint2 hw = save->lv[e][l][0];
            const uint32_t rec = hw.y >> 16, cell = rec & 0x7Fu;
            uint32_t digits = rec >> 7;
            if (l + 1 == depth) {
                // the digit being searched: the highest one taken (digits go in ascending order)
                const uint2 cw = save->lv[e][l][cell % 27];
                const uint32_t third = cell / 27;
                const uint32_t xc = (third == 0 ? cw.x : (third == 1 ? cw.x >> 16 : cw.y)) & 0x1FFu;
                const uint32_t taken = xc & ~digits;
                if (taken) digits |= 1u << (31 - __clz(taken));
            }
            const uint2 v = t < 27 ? save->lv[e][l][t] : make_uint2(0, 0);
            const uint32_t y0 = v.x & 0xFFFFu, y1 = v.x >> 16, y2 = v.y & 0xFFFFu;
            const bool k0 = cell == t, k1 = cell == t + 27, k2 = cell == t + 54;
            for (uint32_t g = digits; g; g &= g - 1u, ++q) {
                const uint32_t dv = (g & (0u - g)) | 0x400u;
                DnItem* it = items + i0 + q;
                if (t < 27) it->w[t] = make_uint2((k0 ? dv : y0) | ((k1 ? dv : y1) << 16), k2 ? dv : y2);
                if (t == 0) {
                    it->board = k;
                    it->rec = r;
                    it->plen = cell + 1u;
                    seedq[q0 + q] = i0 + q;
                }
            }
        }
        if (t == 0) {
            if (q != nit) atomicOr(&ctl->err, kDnErrSeed);   // the reservation and the items disagree
            atomicAdd(&ctl->seed.boards, 1u);
        }
        __syncthreads();
    }
}
__global__ void dn_scatter_kernel(const uint32_t* list, const uint8_t* sub_out, const int8_t* sub_st,
                                  const uint64_t* sub_work, bool depth, uint8_t* out, int8_t* status, uint64_t* work) {
    const uint32_t m = list[0];
    const uint32_t* hits = list + 1;
    for (uint32_t i = blockIdx.x; i < m; i += gridDim.x) {
        const uint64_t j = hits[i];
        if (threadIdx.x < 81) out[j * 81 + threadIdx.x] = sub_out[(uint64_t)i * 81 + threadIdx.x];
        if (threadIdx.x == 0) {
            status[j] = sub_st[i];
            if (work && sub_work) work[j] = depth ? max(work[j], sub_work[i]) : work[j] + sub_work[i];
        }
    }
}
}  // namespace sdk

// Pinned host staging of the host-pointer calls (sdk_solve_batch_ex, sdk_expand_boards): the
// caller's arrays are copied into it on the CPU and moved by true asynchronous DMA.  HIP's own path
// for pageable memory took 12-25 ms per call now and then for a 1.3 MB transfer whose kernel ran
// 0.2 ms (profiles/r05/slice_probe_timing_r05c.log: a node's search slices), all of it CPU time in
// the calling thread.  Grown as needed up to kStageMax; larger calls keep the pageable path.
struct HostBuf {
    void* p = nullptr;
    size_t bytes = 0;
};
constexpr size_t kStageMax = size_t(256) << 20;
constexpr size_t kStageInit = size_t(8) << 20;   // allocated with the context: pinning costs ~ms
                                                 // (the first slice of a node paid 34 ms growing it)

struct sdk_ctx {
    int device = 0;
    int cus = 256;
    hipStream_t stream = nullptr;
    std::mutex mu;
    HostBuf stage;                 // pinned staging (see HostBuf)
    // options
    int order = SDK_ORDER_LEX;     // lex-first DFS: no uniqueness proof needed (faster than MRV_UNIQUE, r02)
    uint64_t budget = 0;
    int waves_per_cu = 32;
    int check_blocks_per_cu = 3;
    int check_variant = SDK_CHECK_REG1;
    int solve_chunk = 0;          // boards per dequeue, 0 = automatic
    int work_rounds = 0;
    int solver = SDK_SOLVER_QUAD;
    int locked = 1;                // QUAD: locked candidates at fixpoints (fewer search nodes, same answers)
    int waves_per_cu2 = 28;       // solve2/solve4 grid per CU = solve4's resident waves (7 per SIMD; a larger
                                  // grid only adds waves that start once the queue is drained: 1 % slower, r02)
    // workspaces
    DevBuf stack, counter, heads, in, mask, out, status, work, verdict;
    uint32_t heads_round = 0;      // launches since the heads pool was cleared (kHeadRounds regions)
    int xcd_heads = 1;             // QUAD: per-XCD dequeue heads (SDK_OPT_XCD_HEADS)
    int donate = 1;                // QUAD, LEX solves: subtree donation (SDK_OPT_DONATE)
    DevBuf dn;                     // two donation areas (solve4_kernel.h: DnCtl, records, items,
                                   // mailboxes), one per donation phase of a phased solve
    void* dn_area = nullptr;       // the area of the donation launch being enqueued
    DevBuf dn_in, dn_mask, dn_out, dn_st, dn_work, dn_list;        // the phased solve's tail boards
    DevBuf dn3_in, dn3_mask, dn3_out, dn3_st, dn3_work, dn3_list;   // ... and its LEX re-solves
    DevBuf dn_stat;                // [0] boards the last phased solve passed to the donation
                                   // kernel, [1] of those, boards re-solved in LEX order
    bool dn_ran = false;           // the last solve was phased (dn_stat and `delivered` are its)
    bool timer_hold = false;       // a phased solve is being timed as one span
    bool dn_err_check = false;     // a phased solve ran since its control blocks' error words were read
    int dn_fault = 0;              // SDK_OPT_DN_FAULT (test only)
    int dn_helpers = 2;            // SDK_OPT_DONATE_HELPERS: donation-launch waves per listed board (+ 64)
    int dn_resume = 1;             // SDK_OPT_DONATE_RESUME: split boards resume from their saved stacks
    bool dn_resume_now = false;    // ... in the phased solve being enqueued (launch_solve)
    DevBuf dn_save, dn_save_idx, dn_seeds;   // sdk::SplitSave, its entry per board, the seed list
    int dn_exhaustive = 1;         // phase 2 in MRV count-to-2 order (SDK_OPT_DONATE_MODE)
    int64_t dn_max = 1 << 19;      // largest batch solved in phases (SDK_OPT_DONATE_MAX, 0 = any)
    uint32_t dn_epoch = 0;         // launches that used it (mailbox / registration entries carry it)
    int dn_blocks_per_cu = 0;      // resident solve4_kernel<true> workgroups per CU (queried once)
    uint64_t split_big = 0;        // the phased solve being enqueued: its split budget above
                                   // sdk::kBudgetBigBoards searched boards (device-counted batches)
    int prop32 = 1;                // QUAD: bit-sliced root propagation first (SDK_OPT_PROP32)
    int prop32_lc = 5 | (3 << 8);  // ... a locked-candidates pass every this many steps (low byte),
                                   //     the first after step (value >> 8), 0 = the period: after
                                   //     steps 3, 8, 13, ... (prop32 "schedule")
    int64_t prop32_min = 4096;     // ... for batches of at least this many boards
    int prop32_handover = 1;       // ... undecided boards searched from their propagated grids
    int prop32_tail_live = 0;      // ... a group's last (at most this many) live boards handed over
    int prop32_tail_step = 24;     //     from this step on (SDK_OPT_PROP32_TAIL = live | step << 8)
    bool prop32_ran = false;       // the last solve ran it (p32_list[0] = its undecided boards)
    DevBuf p32_ctl, p32_list, p32_in, p32_out, p32_st;
    int clock_probe = 0;           // sdk_debug_clock_arm: prop32 passes run the stamped twin
    DevBuf p32_stamps;             // ... its stamps, 4 words per workgroup of the last such pass
    uint32_t p32_stamp_wgs = 0;
    DevBuf fr_a, fr_b, prop, bcell, bmask, nchild, offs, fr_status, fr_mask, tsum, fr_ctl;
    DevBuf fr_tail;                // refine_head: the boards kept after the refined ones
    // the device-resident frontier of the last sdk_frontier_build (in fr_a)
    uint64_t fr_size = 0;
    uint64_t fr_leaves = 0;
    uint32_t fr_levels = 0;
    bool fr_valid = false;
    int fr_mode = SDK_FRONTIER_COUNT;   // kept by refinements and loaded records
    long long* first_found = nullptr;   // set by frontier_first for its solve launch (SolveArgs::found)
    // RCCL communicator (sdk_comm_init), one rank per context
    ncclComm_t comm = nullptr;
    int comm_rank = 0;
    int comm_world = 1;
    // timing
    bool timing = false;          // SDK_OPT_TIMING
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    size_t events_used = 0;
};

namespace {

constexpr uint64_t kDnSplitDefault = 128;   // SDK_OPT_DONATE = 1: split budget (search nodes) of the plain phase
                                            // (256 to round 3; profiles/r03/sweep_split_r03.log)
constexpr uint32_t kHeadRounds = 64;        // dequeue-head regions per clear (launch_solve_once)

// a pinned staging area of at least `bytes` (nullptr: too large, use the pageable path)
void* stage_host(HostBuf& b, size_t bytes) {
    if (bytes > kStageMax) return nullptr;
    if (b.bytes >= bytes) return b.p;
    if (b.p) (void)hipHostFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    // doubling growth: a node's slices grow their batches a little at a time
    const size_t want = std::min(kStageMax, std::max(bytes, std::max(b.bytes * 2, kStageInit)));
    if (hipHostMalloc(&b.p, want, hipHostMallocDefault) != hipSuccess) {
        b.p = nullptr;
        return nullptr;
    }
    b.bytes = want;
    return b.p;
}

int ensure(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes) return SDK_OK;
    if (b.p) HIPCALL(hipFree(b.p));
    b.p = nullptr;
    b.bytes = 0;
    size_t want = std::max(bytes, (size_t)256);
    HIPCALL(hipMalloc(&b.p, want));
    b.bytes = want;
    return SDK_OK;
}

// Kernel timing is opt-in (SDK_OPT_TIMING): with it off no event is created or
// recorded, so a long-running node or drop-in solver holds no per-launch state.
int timer_begin(sdk_ctx* c, hipEvent_t* stop_out) {
    *stop_out = nullptr;
    if (!c->timing || c->timer_hold) return SDK_OK;
    if (c->events_used >= kMaxTimedLaunches) return fail(SDK_EINVAL, "%zu timed launches since sdk_timer_reset", kMaxTimedLaunches);
    if (c->events_used == c->events.size()) {
        hipEvent_t a, b;
        HIPCALL(hipEventCreate(&a));
        HIPCALL(hipEventCreate(&b));
        c->events.emplace_back(a, b);
    }
    auto& pr = c->events[c->events_used++];
    HIPCALL(hipEventRecord(pr.first, c->stream));
    *stop_out = pr.second;
    return SDK_OK;
}

int timer_end(sdk_ctx* c, hipEvent_t stop) {
    if (stop) HIPCALL(hipEventRecord(stop, c->stream));
    return SDK_OK;
}

int launch_check(sdk_ctx* c, const uint8_t* d_in, uint8_t* d_out, size_t n) {
    if (n == 0) return SDK_OK;
    if (reinterpret_cast<uintptr_t>(d_in) & 15) return fail(SDK_EINVAL, "device boards must be 16-byte aligned");
    const uint64_t tiles = (n + sdk::kCheckThreads - 1) / sdk::kCheckThreads;
    const unsigned grid = (unsigned)std::min<uint64_t>(tiles, (uint64_t)c->cus * c->check_blocks_per_cu);
    hipEvent_t stop;
    int rc = timer_begin(c, &stop);
    if (rc) return rc;
    int variant = c->check_variant;
    if (variant == SDK_CHECK_REG2 && tiles < 2ull * grid) variant = SDK_CHECK_REG1;   // rr2 needs a full tile per slot
    switch (variant) {
        case SDK_CHECK_REG2: sdk::check_kernel_rr2<<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n); break;
        case SDK_CHECK_GLDS2: sdk::check_kernel_glds<2><<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n); break;
        case SDK_CHECK_GLDS3: sdk::check_kernel_glds<3><<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n); break;
        case SDK_CHECK_GLDS4: sdk::check_kernel_glds<4><<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n); break;
        case SDK_CHECK_WAVE1: sdk::check_kernel_wave<1><<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n); break;
        case SDK_CHECK_WAVE2: sdk::check_kernel_wave<2><<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n); break;
        default: sdk::check_kernel<<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n); break;
    }
    HIPCALL(hipGetLastError());
    if ((rc = timer_end(c, stop))) return rc;
    return SDK_OK;
}


// dn_phase (QUAD, LEX solves with SDK_OPT_DONATE): 0 plain launch; 1 the split phase (plain
// kernel, split budget); 2 the donation kernel solve4_kernel<true> on the full resident grid,
// donation area c->dn_area (see launch_solve).  The phases' control words are zeroed by
// launch_solve's prep launch.
int launch_solve_once(sdk_ctx* c, const uint8_t* d_in, const uint16_t* d_mask, uint8_t* d_out, int8_t* d_status,
                      uint64_t* d_work, size_t n, int count_mode, uint64_t limit, unsigned long long* d_count,
                      unsigned long long* d_counts, uint64_t in_first, uint64_t in_step, int order, int64_t budget,
                      int dn_phase, const uint32_t* n_dev = nullptr) {
    // budget: node budget per board for this launch (-1 = the context's SDK_OPT_NODE_BUDGET)
    const uint64_t node_budget = budget >= 0 ? (uint64_t)budget : c->budget;
    if (n == 0) return SDK_OK;
    if (n > 0x7FFFFFFFull) return fail(SDK_EINVAL, "at most 2^31-1 boards per call");
    if (c->solver == SDK_SOLVER_LANE && !count_mode) {
        // one board per lane: the reference's own DFS (solve_lane_kernel.h); `work` =
        // the reference's validations, the budget counts validations
        if (!d_out || !d_status) return fail(SDK_EINVAL, "solve needs out and status buffers");
        if (order == SDK_ORDER_MRV_UNIQUE || (order < 0 && c->order == SDK_ORDER_MRV_UNIQUE))
            return fail(SDK_EINVAL, "the LANE solver runs the reference's order only (SDK_ORDER_LEX)");
        int rc = ensure(c->counter, 256);
        if (rc) return rc;
        HIPCALL(hipMemsetAsync(c->counter.p, 0, 8, c->stream));
        sdk::SolveArgs a{};
        a.in = d_in;
        a.mask = d_mask;
        a.out = d_out;
        a.status = d_status;
        a.work = d_work;
        a.n = n;
        a.next = static_cast<uint32_t*>(c->counter.p);
        a.budget = node_budget;
        a.in_first = in_first;
        a.in_step = in_step;
        const uint64_t blocks = (n + sdk::kLaneThreads - 1) / sdk::kLaneThreads;
        const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)c->cus * 6));
        hipEvent_t stop;
        rc = timer_begin(c, &stop);
        if (rc) return rc;
        sdk::solve_lane_kernel<<<grid, sdk::kLaneThreads, 0, c->stream>>>(a);
        HIPCALL(hipGetLastError());
        return timer_end(c, stop);
    }
    // two (solve2_kernel) or four (solve4_kernel) boards per wave for solves; count mode stays
    // one board per wave
    // count mode: QUAD counts four boards per wave (solve4's count mode) unless per-board counts
    // are asked for; the other solvers count with the one-board-per-wave kernel
    const int per_wave = count_mode ? ((c->solver == SDK_SOLVER_QUAD && !d_counts) ? 4 : 1)
                                    : (c->solver == SDK_SOLVER_QUAD ? 4 : (c->solver == SDK_SOLVER_HALFWAVE ? 2 : 1));
    const bool two = per_wave == 2, four = per_wave == 4;
    if ((two || four) && !d_status) return fail(SDK_EINVAL, "solve needs a status buffer");
    if ((two || four) && !count_mode && !d_out) return fail(SDK_EINVAL, "solve needs an out buffer");
    const uint64_t slots = (uint64_t)c->cus * (per_wave > 1 ? c->waves_per_cu2 : c->waves_per_cu) * per_wave;
    // 16 boards per dequeue (fewer when a slot would get < 2 dequeues); 8 for the QUAD solver,
    // whose dequeues go to per-XCD heads with one stage per wave and dealt first chunks: there
    // 8 is the fastest at every C4 shard size and on 30-clue boards (round 3,
    // profiles/r03/sweep_chunk_r03.log: 1.25M 17-clue 1.489 vs 1.557 ms at 16, 10M 10.01 vs
    // 10.05, 30-clue 1M 0.648 vs 0.676).  Count mode uses single boards (subtrees differ by
    // orders of magnitude).
    // Round 4, QUAD by batch size (profiles/r04/ab_chunk_by_size_r04u.log, M 17-clue puzzles/s at
    // chunk 4 / 6 / 8): 1.25M boards 882 / 867 / 862, 2.5M 939 / 958 / 924, 5M 992 / 1000 / 994, 10M
    // 1026 / 1036 / 1036 -- below 64 boards per slot the launch drain (the last chunks) outweighs
    // the extra dequeues, so 4; else 6
    const uint64_t quad_chunk = n < slots * 64 ? 4 : 6;
    const uint32_t chunk = count_mode ? 1u
        : c->solve_chunk ? (uint32_t)c->solve_chunk
        : (uint32_t)std::min<uint64_t>(per_wave == 4 ? quad_chunk : 16, std::max<uint64_t>(1, n / (slots * 2)));
    const uint64_t want = (n + chunk - 1) / chunk;
    const unsigned grid = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>((want + per_wave - 1) / per_wave, slots / per_wave));
    const size_t stack_words = four ? sdk::kStack4WordsPerBlock : (two ? sdk::kStack2WordsPerBlock : sdk::kStackWordsPerBlock);
    int rc = ensure(c->stack, (size_t)grid * stack_words * sizeof(uint32_t));
    if (rc) return rc;
    rc = ensure(c->counter, 256);
    if (rc) return rc;
    // QUAD with per-XCD heads: the dequeue counter lives in the heads region after the heads.
    // Plain launches take a fresh region of a pool of kHeadRounds, cleared by one memset every
    // kHeadRounds launches (a per-launch memset is its own ~4 us dispatch in front of the
    // kernel); the split phase's region is cleared by its prep launch.  Otherwise the counter
    // is word 0 of c->counter (words 1.. belong to callers).
    const bool use_heads = four && c->xcd_heads && dn_phase != 2;
    uint32_t* heads = nullptr;
    if (use_heads) {
        if ((rc = ensure(c->heads, (size_t)kHeadRounds * sdk::kHeadWords * sizeof(uint32_t)))) return rc;
        uint32_t region = 0;
        if (dn_phase == 0) {
            region = c->heads_round++ % kHeadRounds;
            if (region == 0)
                HIPCALL(hipMemsetAsync(c->heads.p, 0, (size_t)kHeadRounds * sdk::kHeadWords * sizeof(uint32_t), c->stream));
        }
        heads = static_cast<uint32_t*>(c->heads.p) + (size_t)region * sdk::kHeadWords;
    } else if (dn_phase == 0) {
        HIPCALL(hipMemsetAsync(c->counter.p, 0, 8, c->stream));
    }
    sdk::SolveArgs a;
    a.in = d_in;
    a.mask = d_mask;
    a.out = d_out;
    a.status = d_status;
    a.work = d_work;
    a.n = n;
    a.next = use_heads ? heads + sdk::kHeadNext : static_cast<uint32_t*>(c->counter.p);
    a.stack = static_cast<uint32_t*>(c->stack.p);
    a.budget = node_budget;
    a.order = order >= 0 ? order : c->order;
    a.limit = limit;
    a.count = d_count;
    a.counts = d_counts;
    a.count_mode = count_mode;
    a.chunk = chunk;
    a.work_rounds = c->work_rounds;
    a.in_first = in_first;
    a.in_step = in_step;
    a.locked = c->locked;
    a.heads = nullptr;
    a.donate = nullptr;
    a.n_dev = n_dev;   // the plain and split launches of a prop32 fallback: the list's length
    a.save = nullptr;
    a.save_idx = nullptr;
    // a first-solution scan (frontier_first): the plain QUAD launch cancels boards above the lowest hit
    a.found = (four && !count_mode && dn_phase == 0) ? c->first_found : nullptr;
    a.budget_big = (four && dn_phase == 1) ? c->split_big : 0;   // the split phase of a device-counted batch
    if (dn_phase == 1 && c->dn_resume_now && four && !count_mode) {
        // the split phase leaves the stacks of the boards it stops (sdk::split_save4)
        a.save = c->dn_save.p;
        a.save_idx = static_cast<uint32_t*>(c->dn_save_idx.p);
    }
    unsigned grid_used = grid;
    if (four && !count_mode && dn_phase == 2) {
        // subtree donation: idle waves wait for items while any wave of the grid works, so the
        // grid is the resident one (its occupancy, not waves_per_cu2), whatever the batch size:
        // waves without a board of their own are the helpers
        if (c->dn_blocks_per_cu <= 0) {
            c->dn_blocks_per_cu = sdk::solve4_dn_blocks_per_cu();
            if (c->dn_blocks_per_cu <= 0) return fail(SDK_EHIP, "occupancy query for the donation kernel failed");
        }
        a.donate = c->dn_area;
        // the boards: a list length on the device (n bounds it), one per dequeue on the
        // area's own counter
        a.n_dev = n_dev;
        a.chunk = 1;
        a.next = &static_cast<sdk::DnCtl*>(c->dn_area)->next;
        // the resident grid, at most what the kernel keeps of it for n boards: n / 4 + 64 + helpers x
        // min(n, kDnHelpCap) (solve4_kernel; the list on the device may be shorter, then it keeps less)
        grid_used = (unsigned)std::max<uint64_t>(
            1, std::min<uint64_t>({(uint64_t)c->cus * (uint64_t)std::min(c->dn_blocks_per_cu, c->waves_per_cu2),
                                   (uint64_t)sdk::kDnMbox,
                                   ((uint64_t)n + 3) / 4 + 64ull +
                                       (uint64_t)c->dn_helpers * std::min<uint64_t>(n, sdk::kDnHelpCap)}));
        if (grid_used > grid) {
            rc = ensure(c->stack, (size_t)grid_used * stack_words * sizeof(uint32_t));
            if (rc) return rc;
            a.stack = static_cast<uint32_t*>(c->stack.p);
        }
    }
    if (use_heads) a.heads = heads;
    hipEvent_t stop;
    rc = timer_begin(c, &stop);
    if (rc) return rc;
    if (four) {
        HIPCALL(sdk::launch_solve4(a, grid_used, c->stream));
    } else if (two) {
        HIPCALL(sdk::launch_solve2(a, grid, c->stream));
    } else {
        sdk::solve_kernel<<<grid, 64, 0, c->stream>>>(a);
    }
    HIPCALL(hipGetLastError());
    if ((rc = timer_end(c, stop))) return rc;
    return SDK_OK;
}

// Solve launch.  QUAD solves with SDK_OPT_DONATE (LEX, or MRV_UNIQUE: its split phase counts to
// two completions and re-searches in LEX within the slot, like the plain launch) run in phases:
// every board first in
// the plain kernel with at most `split` search nodes (the C4/C2 path is that launch alone);
// the few boards that need more -- the launch's tail -- are gathered and solved again by
// solve4_kernel<true> on the full resident grid, where idle waves take subtrees of the
// heavy boards (subtree donation, solve4_kernel.h), and scattered back.  That second launch
// is exhaustive: MRV branching, at most two completions per board, every donated subtree
// needed work; a unique completion is the lex-first one.  The boards it finds several
// completions for (or cannot decide within the budget) are solved a third time in LEX
// order with donation.  Results are the ones a single slot finds (same boards and
// statuses; `work` adds up the phases and parts).
//
// Every phase is enqueued at once, without the host: the lists of boards a phase passes
// on live on the device (length word first), and the gather, donation and scatter kernels
// read their lengths there (an empty list costs a few microseconds of launches).  The
// phase buffers are sized for every board of the call, up to kDnCapBoards boards per
// phased pass; larger calls run in passes of that many.
constexpr uint64_t kDnCapBoards = 1ull << 24;

// list the boards of status[0, n) (n bounded by *n_dev when given) that carry `code` into
// `list` (its length zeroed by the prep launch), copying them to (buf_in, buf_mask)
// resume: the split phase's list -- boards with saved stacks go to the seed list, and
// dn_seed_kernel lists them after the restarted ones (donation area 0)
int dn_collect(sdk_ctx* c, const int8_t* d_status, uint64_t n, const uint32_t* n_dev, int8_t code, DevBuf& list,
               int stat, const uint8_t* d_in, const uint16_t* d_mask, uint64_t in_first, uint64_t in_step,
               DevBuf& buf_in, DevBuf& buf_mask, bool resume = false) {
    int rc;
    if ((rc = ensure(buf_in, (size_t)n * 81)) || (d_mask && (rc = ensure(buf_mask, (size_t)n * 2)))) return rc;
    sdk::DnResume rs{};
    if (resume) {
        rs.save = static_cast<const sdk::SplitSave*>(c->dn_save.p);
        rs.save_idx = static_cast<const uint32_t*>(c->dn_save_idx.p);
        rs.ctl = static_cast<sdk::DnCtl*>(c->dn.p);
        rs.seeds = static_cast<uint32_t*>(c->dn_seeds.p);
    }
    uint32_t* lst = static_cast<uint32_t*>(list.p);
    uint32_t* total = static_cast<uint32_t*>(c->dn_stat.p) + stat;
    uint8_t* bin = static_cast<uint8_t*>(buf_in.p);
    uint16_t* bmask = static_cast<uint16_t*>(d_mask ? buf_mask.p : nullptr);
    sdk::dn_collect_kernel<<<(unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, (uint64_t)c->cus * 8)),
                             256, 0, c->stream>>>(d_status, n, n_dev, code, lst, total, d_in, d_mask, in_first, in_step,
                                                  bin, bmask, rs);
    HIPCALL(hipGetLastError());
    if (resume) {
        sdk::dn_seed_kernel<<<(unsigned)std::min<uint64_t>(sdk::kSeedBoards, (uint64_t)c->cus * 4), 64, 0, c->stream>>>(
            rs.seeds, rs.save, lst, total, d_in, d_mask, in_first, in_step, bin, bmask, rs.ctl);
        HIPCALL(hipGetLastError());
    }
    return SDK_OK;
}

// solve the (at most cap) boards `list` collected into buf_in/buf_mask with the donation
// kernel (order) in donation area `area`, scatter the answers into (d_out, d_status, d_work)
// (n_dev: the boards the donation launch dequeues -- the list's length, or with resumed boards
// the restarted ones alone)
int dn_resolve(sdk_ctx* c, uint64_t cap, const DevBuf& list, int area, bool has_mask, uint8_t* d_out,
               int8_t* d_status, uint64_t* d_work, int order, int64_t budget, DevBuf& buf_in, DevBuf& buf_mask,
               DevBuf& buf_out, DevBuf& buf_st, DevBuf& buf_work, const uint32_t* n_dev = nullptr) {
    int rc;
    if ((rc = ensure(buf_out, (size_t)cap * 81)) || (rc = ensure(buf_st, cap)) ||
        (d_work && (rc = ensure(buf_work, (size_t)cap * 8))))
        return rc;
    const uint32_t* lst = static_cast<const uint32_t*>(list.p);
    uint8_t* in = static_cast<uint8_t*>(buf_in.p);
    uint16_t* mask = has_mask ? static_cast<uint16_t*>(buf_mask.p) : nullptr;
    uint8_t* out = static_cast<uint8_t*>(buf_out.p);
    int8_t* st = static_cast<int8_t*>(buf_st.p);
    uint64_t* work = d_work ? static_cast<uint64_t*>(buf_work.p) : nullptr;
    c->dn_area = static_cast<char*>(c->dn.p) + (size_t)area * sdk::kDnBytes;
    if ((rc = launch_solve_once(c, in, mask, out, st, work, cap, 0, 0, nullptr, nullptr, 0, 1, order, budget, 2,
                                n_dev ? n_dev : lst)))
        return rc;
    if (order == SDK_ORDER_MRV_UNIQUE) {
        // boards with several completions (or undecided): LEX order, donation again
        if ((rc = dn_collect(c, st, cap, lst, (int8_t)sdk::kDnRetryLex, c->dn3_list, 1, in, mask, 0, 1, c->dn3_in,
                             c->dn3_mask)) ||
            (rc = dn_resolve(c, cap, c->dn3_list, 1, has_mask, out, st, work, SDK_ORDER_LEX, budget, c->dn3_in,
                             c->dn3_mask, c->dn3_out, c->dn3_st, c->dn3_work)))
            return rc;
    }
    const unsigned g = (unsigned)std::min<uint64_t>(cap, (uint64_t)c->cus * 16);
    sdk::dn_scatter_kernel<<<g, 128, 0, c->stream>>>(lst, out, st, work, c->work_rounds == SDK_WORK_DEPTH, d_out,
                                                     d_status, d_work);
    HIPCALL(hipGetLastError());
    return SDK_OK;
}

// zero a phased pass's control words in one launch (sdk::dn_prep_kernel)
int dn_prep(sdk_ctx* c, uint64_t cap, bool first_pass) {
    int rc;
    if (c->dn.bytes < 2 * sdk::kDnBytes || c->dn_epoch > 0xFFFFFF00u) {
        // entries of epoch 0 (and, after 2^32 launches, the stale ones cleared once)
        if ((rc = ensure(c->dn, 2 * sdk::kDnBytes))) return rc;
        HIPCALL(hipMemsetAsync(c->dn.p, 0, 2 * sdk::kDnBytes, c->stream));
        c->dn_epoch = 0;
    }
    if ((rc = ensure(c->dn_stat, 256)) || (rc = ensure(c->counter, 256)) ||
        (rc = ensure(c->heads, (size_t)kHeadRounds * sdk::kHeadWords * sizeof(uint32_t))) ||
        (rc = ensure(c->dn_list, (cap + 1) * sizeof(uint32_t))) || (rc = ensure(c->dn3_list, (cap + 1) * sizeof(uint32_t))))
        return rc;
    sdk::DnPrep p{};
    p.counter = static_cast<uint32_t*>(c->counter.p);
    p.heads = c->xcd_heads ? static_cast<uint32_t*>(c->heads.p) : nullptr;
    p.heads_words = sdk::kHeadWords;   // the heads and the dequeue counter after them
    p.stat = first_pass ? static_cast<uint32_t*>(c->dn_stat.p) : nullptr;   // statistics add up over passes
    for (int k = 0; k < 2; ++k) {
        p.ctl[k] = reinterpret_cast<uint32_t*>(static_cast<char*>(c->dn.p) + (size_t)k * sdk::kDnBytes);
        p.epoch[k] = ++c->dn_epoch;
    }
    p.fault = c->dn_fault ? 1u : 0u;
    p.helpers = (uint32_t)c->dn_helpers;
    p.list[0] = static_cast<uint32_t*>(c->dn_list.p);
    p.list[1] = static_cast<uint32_t*>(c->dn3_list.p);
    if (c->dn_resume_now) {
        if ((rc = ensure(c->dn_save, sizeof(sdk::SplitSave))) || (rc = ensure(c->dn_save_idx, (size_t)cap * 4)) ||
            (rc = ensure(c->dn_seeds, (2 + 2 * (size_t)sdk::kSeedBoards) * 4)))
            return rc;
        p.seeds = static_cast<uint32_t*>(c->dn_seeds.p);
        p.save = static_cast<uint32_t*>(c->dn_save.p);
    }
    sdk::dn_prep_kernel<<<1, 256, 0, c->stream>>>(p);
    HIPCALL(hipGetLastError());
    return SDK_OK;
}

int launch_prop32_solve(sdk_ctx* c, const uint8_t* d_in, uint8_t* d_out, int8_t* d_status, size_t n, int order,
                        int64_t budget, int64_t donate);

int launch_solve(sdk_ctx* c, const uint8_t* d_in, const uint16_t* d_mask, uint8_t* d_out, int8_t* d_status,
                 uint64_t* d_work, size_t n, int count_mode, uint64_t limit, unsigned long long* d_count,
                 unsigned long long* d_counts = nullptr, uint64_t in_first = 0, uint64_t in_step = 1,
                 int order = -1, int64_t budget = -1, int64_t donate = -1, const uint32_t* n_dev = nullptr) {
    // donate: SDK_OPT_DONATE for this call (-1 = the context's); n_dev: the batch's length on the
    // device (n bounds it; the prop32 fallback)
    const int eff_order = order >= 0 ? order : c->order;
    const uint64_t node_budget = budget >= 0 ? (uint64_t)budget : c->budget;
    if (!n_dev) c->prop32_ran = false;
    // the bit-sliced root propagation pass first (prop32_kernel.h): plain solves of whole batches
    // (no first-cell masks, work counters, strided inputs or first-solution scans), 16-byte
    // aligned, at least prop32_min boards; a budget of 1 node is left to solve4 (a board solved at
    // its root takes one); prop32 always runs locked-candidates passes, so with SDK_OPT_LOCKED 0
    // it only runs where no budget can tell the difference
    if (!n_dev && c->prop32 && c->solver == SDK_SOLVER_QUAD && !count_mode && d_out && d_status && !d_work &&
        !d_mask && in_first == 0 && in_step <= 1 && !c->first_found &&
        (node_budget == 0 || (node_budget >= 2 && c->locked)) &&
        (int64_t)n >= c->prop32_min && n <= kDnCapBoards &&
        ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out)) & 15u) == 0)
        return launch_prop32_solve(c, d_in, d_out, d_status, n, order, budget, donate);
    const int64_t dn = donate >= 0 ? donate : (int64_t)c->donate;
    // the default split budget doubles above 2^19 SEARCHED boards (sdk::kBudgetBigBoards; a prop32
    // fallback batch's count is on the device, so its split launch picks the budget there): with ~30
    // boards per slot a heavy board's extra nodes overlap the bulk, and fewer boards reach the
    // donation launch (1M hard boards, 880k searched, LEX: 6.88 ms at 128, 6.14 at 256, 6.39 at 384;
    // 1M minimal, 460k searched: 2.68 ms at 128, 2.93 at 256; profiles/r05/sweep_phased_hard_r05s.log,
    // ab_lc_r05t.log)
    const bool split_auto = dn == 1;
    const uint64_t split = split_auto ? (!n_dev && n > sdk::kBudgetBigBoards ? 2 * kDnSplitDefault : kDnSplitDefault)
                                      : (uint64_t)dn;
    // (only where the node budget leaves room for it: with a budget B <= 256 a board needing
    // more than B nodes must end as a budget hit, which the split phase at 256 would solve)
    c->split_big = split_auto && n_dev && (node_budget == 0 || node_budget > 2 * kDnSplitDefault)
                       ? 2 * kDnSplitDefault : 0;
    const bool two_phase = n > 0 && !count_mode && dn && c->solver == SDK_SOLVER_QUAD &&
                           (eff_order == SDK_ORDER_LEX || eff_order == SDK_ORDER_MRV_UNIQUE) && d_out && d_status &&
                           (node_budget == 0 || node_budget > split) &&
                           // a prop32 fallback batch (n_dev) holds only boards propagation left open:
                           // phased at any size (1M hard boards: 6.8 ms phased vs 8.3 in one launch,
                           // profiles/r05/ab_dnmax_r05r.log)
                           (c->dn_max == 0 || (int64_t)n <= c->dn_max || n_dev);
    c->dn_ran = two_phase;
    if (two_phase) c->dn_err_check = true;
    // resumed items keep the split phase's branching, so only MRV stacks resume, into the
    // exhaustive (MRV) donation launch: LEX items there cost more nodes than a restart in MRV
    // order (heavy 1000: 80k vs 61k nodes, 1.56 vs 1.30 ms), and LEX acceptance in a LEX
    // donation launch would need the closed prefixes MRV stacks do not have
    c->dn_resume_now = two_phase && c->dn_resume && c->dn_exhaustive && eff_order == SDK_ORDER_MRV_UNIQUE;
    if (!two_phase)
        return launch_solve_once(c, d_in, d_mask, d_out, d_status, d_work, n, count_mode, limit, d_count, d_counts,
                                 in_first, in_step, order, budget, 0, n_dev);
    if (n_dev && n > kDnCapBoards) return fail(SDK_EINVAL, "a device-counted batch is solved in one pass");
    // SDK_OPT_TIMING: the phases of one solve are one timed span
    hipEvent_t stop;
    int rc = timer_begin(c, &stop);
    if (rc) return rc;
    c->timer_hold = true;
    const uint64_t step = in_step ? in_step : 1;
    for (uint64_t b0 = 0; b0 < n && !rc; b0 += kDnCapBoards) {
        const uint64_t m = std::min<uint64_t>(n - b0, kDnCapBoards);
        uint8_t* out = d_out + b0 * 81;
        int8_t* st = d_status + b0;
        uint64_t* work = d_work ? d_work + b0 : nullptr;
        const uint16_t* mask = d_mask ? d_mask + b0 : nullptr;
        const uint64_t first = in_first + b0 * step;
        (void)((rc = dn_prep(c, m, b0 == 0)) ||
               (rc = launch_solve_once(c, d_in, mask, out, st, work, m, 0, 0, nullptr, nullptr, first, step, order,
                                       (int64_t)split, 1, n_dev)) ||
               (rc = dn_collect(c, st, m, n_dev, (int8_t)-2, c->dn_list, 0, d_in, mask, first, step, c->dn_in,
                                c->dn_mask, c->dn_resume_now)) ||
               (rc = dn_resolve(c, m, c->dn_list, 0, mask != nullptr, out, st, work,
                                c->dn_exhaustive ? SDK_ORDER_MRV_UNIQUE : SDK_ORDER_LEX, (int64_t)node_budget, c->dn_in,
                                c->dn_mask, c->dn_out, c->dn_st, c->dn_work,
                                c->dn_resume_now ? static_cast<uint32_t*>(c->dn_seeds.p) + 1 : nullptr)));
    }
    c->timer_hold = false;
    if (rc) return rc;
    return timer_end(c, stop);
}

// The prop32 pass (prop32_kernel.h) over the batch, then the boards it leaves undecided -- listed
// with their inputs on the device -- solved by the usual path (solve4, phased with donation when
// that applies) with the list's length read on the device, and their answers scattered back.
// Every launch is enqueued at once; an empty list costs the fallback's launches a few microseconds.
int launch_prop32_solve(sdk_ctx* c, const uint8_t* d_in, uint8_t* d_out, int8_t* d_status, size_t n, int order,
                        int64_t budget, int64_t donate) {
    int rc;
    constexpr size_t kCtlBytes = (size_t)sdk::kP32Heads * sdk::kP32HeadStride * 4;
    if ((rc = ensure(c->p32_ctl, kCtlBytes)) || (rc = ensure(c->p32_list, (n + 1) * 4)) ||
        (rc = ensure(c->p32_in, n * 81)) || (rc = ensure(c->p32_out, n * 81)) || (rc = ensure(c->p32_st, n)))
        return rc;
    HIPCALL(hipMemsetAsync(c->p32_ctl.p, 0, kCtlBytes, c->stream));
    HIPCALL(hipMemsetAsync(c->p32_list.p, 0, 4, c->stream));
    // SDK_OPT_TIMING: two spans, the pass itself and its fallback (search + scatter) as one
    hipEvent_t stop;
    if ((rc = timer_begin(c, &stop))) return rc;
    sdk::Prop32Args a{};
    a.in = d_in;
    a.out = d_out;
    a.status = d_status;
    a.n = n;
    a.heads = static_cast<uint32_t*>(c->p32_ctl.p);
    a.list = static_cast<uint32_t*>(c->p32_list.p);
    a.list_in = static_cast<uint8_t*>(c->p32_in.p);
    a.lc_every = (uint32_t)std::max(1, c->prop32_lc & 0xFF);
    a.lc_first = (c->prop32_lc >> 8) ? (uint32_t)(c->prop32_lc >> 8) : a.lc_every;
    a.max_steps = 96;
    // the search continues from the propagated grids when no node budget applies (a budget counts
    // nodes from the input, so the statuses of budget hits would differ)
    const uint64_t node_budget = budget >= 0 ? (uint64_t)budget : c->budget;
    a.handover = (c->prop32_handover && node_budget == 0) ? 1 : 0;
    a.tail_live = a.handover ? (uint32_t)c->prop32_tail_live : 0u;
    a.tail_step = (uint32_t)c->prop32_tail_step;
    const uint64_t groups = (n + 63) / 64;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(groups, (uint64_t)c->cus * 20));
    uint64_t* stamps = nullptr;
    if (c->clock_probe) {      // the diagnostic twin (sdk_debug_clock_arm)
        if ((rc = ensure(c->p32_stamps, (size_t)grid * 32))) return rc;
        stamps = static_cast<uint64_t*>(c->p32_stamps.p);
        c->p32_stamp_wgs = grid;
    }
    HIPCALL(sdk::launch_prop32(a, grid, c->stream, stamps));
    if ((rc = timer_end(c, stop)) || (rc = timer_begin(c, &stop))) return rc;
    c->timer_hold = true;
    c->prop32_ran = true;
    const uint32_t* lst = static_cast<const uint32_t*>(c->p32_list.p);
    rc = launch_solve(c, static_cast<uint8_t*>(c->p32_in.p), nullptr, static_cast<uint8_t*>(c->p32_out.p),
                      static_cast<int8_t*>(c->p32_st.p), nullptr, n, 0, 0, nullptr, nullptr, 0, 1, order, budget,
                      donate, lst);
    if (!rc) {
        // one thread per 4 bytes of the list's boards (its length is on the device: sized for all n)
        const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n * 81 + 1023) / 1024, (uint64_t)c->cus * 8));
        if (sdk::launch_p32_scatter(lst, static_cast<uint8_t*>(c->p32_out.p), static_cast<int8_t*>(c->p32_st.p), d_in,
                                    d_out, d_status, g, c->stream) != hipSuccess)
            rc = fail(SDK_EHIP, "prop32 scatter launch failed");
    }
    c->timer_hold = false;
    if (rc) return rc;
    return timer_end(c, stop);
}

// Deterministic breadth-first frontier of one board, left in c->fr_a.
// Every rank that builds it from the same board gets the same boards in the same
// order, so ranks can split it without exchanging boards.
//   SDK_FRONTIER_COUNT: MRV branching; solved leaves are counted (fr_leaves) and dropped.
//   SDK_FRONTIER_FIRST: lex branching, solved leaves kept in place, so the frontier is
//                       in lex order of completions (see frontier_kernel.h).
// Expansion stops once the frontier holds >= target boards (or nothing branches).
// Breadth-first expansion of the frontier in fr_a (m0 boards; level 0 applies the
// first-cell mask in fr_mask when `use_mask`) until it reaches `target` boards.  Buffers
// are sized once for the whole build, so the levels are enqueued without the host: a level
// is expanded only while the frontier is below `target` (or at level 0), and a level with
// more than `cap` children is rejected.
constexpr uint64_t kFrontierCap = 1ull << 25;  // 32M boards (2.6 GB) per frontier buffer

// boards a frontier buffer must hold for a build from m0 boards towards `target`
uint64_t frontier_capacity(uint64_t m0, uint64_t target) {
    const uint64_t m_exp = std::max<uint64_t>(m0, std::min(target, kFrontierCap));
    return std::max<uint64_t>(1, std::min(kFrontierCap, 9 * m_exp));
}

// The caller has put the m0 boards in fr_a, sized for frontier_capacity(m0, target) boards
// BEFORE seeding it (a later grow would drop them).
// use_mask: fr_mask holds one first-cell mask per seed board (level 0 applies them);
// force0: level 0 is expanded whatever the seed count (a seed board's mask lives only in that
// level, and sdk_expand_boards always wants at least one level).
int run_frontier_levels(sdk_ctx* c, uint64_t m0, bool use_mask, int mode, uint64_t target, bool force0) {
    int rc;
    const bool first = mode == SDK_FRONTIER_FIRST;
    const uint64_t m_exp = std::max<uint64_t>(m0, std::min(target, kFrontierCap));
    const uint64_t c_out = frontier_capacity(m0, target);
    const uint64_t tiles = (m_exp + sdk::kScanTile - 1) / sdk::kScanTile;
    if (c->fr_a.bytes < c_out * 81) return fail(SDK_EINVAL, "frontier buffer not sized before seeding");
    if ((rc = ensure(c->fr_b, c_out * 81)) || (rc = ensure(c->fr_mask, 16)) ||
        (rc = ensure(c->prop, m_exp * 81)) || (rc = ensure(c->bcell, m_exp)) || (rc = ensure(c->bmask, m_exp * 2)) ||
        (rc = ensure(c->nchild, m_exp * 4)) || (rc = ensure(c->offs, m_exp * 8)) || (rc = ensure(c->tsum, tiles * 8)) ||
        (rc = ensure(c->fr_ctl, sizeof(sdk::FrontierCtl))))
        return rc;
    sdk::FrontierCtl* ctl = static_cast<sdk::FrontierCtl*>(c->fr_ctl.p);
    sdk::FrontierCtl h{};
    h.m = m0;
    HIPCALL(hipMemcpyAsync(ctl, &h, sizeof h, hipMemcpyHostToDevice, c->stream));
    void* buf[2] = {c->fr_a.p, c->fr_b.p};
    const unsigned eg = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>((m_exp + sdk::kChunk - 1) / sdk::kChunk, (uint64_t)c->cus * c->waves_per_cu));
    const bool quad = c->solver == SDK_SOLVER_QUAD;
    const unsigned eg4 = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>((m_exp + 3) / 4, (uint64_t)c->cus * c->waves_per_cu2));
    const unsigned sg = (unsigned)std::min<uint64_t>(tiles, (uint64_t)c->cus * 4);
    const unsigned gg = (unsigned)std::min<uint64_t>(m_exp, (uint64_t)c->cus * 32);
    hipEvent_t stop;
    if ((rc = timer_begin(c, &stop))) return rc;
    constexpr int kLevelsPerSync = 4;
    for (int level = 0; level < 81; ++level) {
        const int in = level & 1;
        sdk::frontier_begin_kernel<<<1, 1, 0, c->stream>>>(ctl, target, level == 0 && force0 ? 1 : 0);
        sdk::ExpandArgs ea;
        ea.in = static_cast<const uint8_t*>(buf[in]);
        ea.ctl = ctl;
        ea.prop = static_cast<uint8_t*>(c->prop.p);
        ea.bcell = static_cast<uint8_t*>(c->bcell.p);
        ea.bmask = static_cast<uint16_t*>(c->bmask.p);
        ea.nchild = static_cast<uint32_t*>(c->nchild.p);
        ea.order = first ? sdk::ORDER_LEX : sdk::ORDER_MRV;
        ea.mask = (level == 0 && use_mask) ? static_cast<const uint16_t*>(c->fr_mask.p) : nullptr;
        ea.keep_leaves = first ? 1 : 0;
        if (quad)   // four boards per wave (expand4_kernel.h): the same frontier, byte for byte
            HIPCALL(sdk::launch_expand4(ea, eg4, c->stream));
        else
            sdk::expand_kernel<<<eg, 64, 0, c->stream>>>(ea);
        sdk::scan_tiles_kernel<<<sg, 1024, 0, c->stream>>>(static_cast<uint32_t*>(c->nchild.p),
                                                           static_cast<uint64_t*>(c->offs.p), ctl,
                                                           static_cast<uint64_t*>(c->tsum.p));
        sdk::scan_top_kernel<<<1, 1024, 0, c->stream>>>(static_cast<uint64_t*>(c->tsum.p), ctl, c_out);
        sdk::emit_kernel<<<gg, 64, 0, c->stream>>>(static_cast<uint8_t*>(c->prop.p), static_cast<uint8_t*>(c->bcell.p),
                                                   static_cast<uint16_t*>(c->bmask.p), static_cast<uint64_t*>(c->offs.p),
                                                   static_cast<uint64_t*>(c->tsum.p), ctl,
                                                   static_cast<uint8_t*>(buf[in ^ 1]));
        sdk::frontier_end_kernel<<<1, 1, 0, c->stream>>>(ctl, first ? 1 : 0);
        HIPCALL(hipGetLastError());
        if (level % kLevelsPerSync == kLevelsPerSync - 1 || level == 80) {
            HIPCALL(hipMemcpyAsync(&h, ctl, sizeof h, hipMemcpyDeviceToHost, c->stream));
            HIPCALL(hipStreamSynchronize(c->stream));
            if (h.done) break;
        }
    }
    if ((rc = timer_end(c, stop))) return rc;
    HIPCALL(hipStreamSynchronize(c->stream));
    if (h.level & 1) std::swap(c->fr_a, c->fr_b);   // the final frontier lives in fr_a
    c->fr_size = h.m;
    c->fr_leaves = h.leaves;
    c->fr_levels = h.level;
    c->fr_valid = true;
    return SDK_OK;
}

int build_frontier(sdk_ctx* c, const uint8_t* h_board, const uint16_t* h_mask, int mode, uint64_t target) {
    c->fr_valid = false;
    c->fr_mode = mode;
    if (target == 0) target = (uint64_t)c->cus * (uint64_t)c->waves_per_cu * 8ull;
    int rc;
    if ((rc = ensure(c->fr_a, frontier_capacity(1, target) * 81)) || (rc = ensure(c->fr_mask, 16))) return rc;
    HIPCALL(hipMemcpyAsync(c->fr_a.p, h_board, 81, hipMemcpyHostToDevice, c->stream));
    if (h_mask) HIPCALL(hipMemcpyAsync(c->fr_mask.p, h_mask, 2, hipMemcpyHostToDevice, c->stream));
    return run_frontier_levels(c, 1, h_mask != nullptr, mode, target, h_mask != nullptr);
}

// Keep frontier boards first, first+step, ... < end of the current (count-mode) frontier and
// expand them further, on this device alone, until they number `target`: the second,
// rank-local stage of a frontier split, so a rank's share of a replicated frontier can be
// small and cheap to build; with step 1 and a short range, a rank's last heavy subtrees
// split into second-level records for the rebalanced count.  The leaves reported are those
// met during this refinement.
int refine_frontier(sdk_ctx* c, uint64_t first, uint64_t step, uint64_t end, uint64_t target) {
    if (!c->fr_valid) return fail(SDK_EINVAL, "no frontier: call sdk_frontier_build first");
    if (step == 0) return fail(SDK_EINVAL, "step must be >= 1");
    const uint64_t m = std::min(end, c->fr_size);
    const uint64_t n = first < m ? (m - first + step - 1) / step : 0;
    c->fr_valid = false;
    target = std::max<uint64_t>(target, n);
    int rc;
    // fr_b takes the share and becomes fr_a: size it for the whole refinement now
    if ((rc = ensure(c->fr_b, frontier_capacity(std::max<uint64_t>(n, 1), target) * 81))) return rc;
    if (n) {
        const unsigned g = (unsigned)std::min<uint64_t>((n + 3) / 4, (uint64_t)c->cus * 16);
        sdk::gather_boards_kernel<<<g, 256, 0, c->stream>>>(static_cast<const uint8_t*>(c->fr_a.p), first, step, n,
                                                           static_cast<uint8_t*>(c->fr_b.p));
        HIPCALL(hipGetLastError());
    }
    std::swap(c->fr_a, c->fr_b);
    if (n == 0) {
        c->fr_size = 0;
        c->fr_leaves = 0;
        c->fr_levels = 0;
        c->fr_valid = true;
        return SDK_OK;
    }
    return run_frontier_levels(c, n, false, c->fr_mode, target, false);
}

// Boards [lo, mid) of the current frontier refined as refine_frontier does (step 1), followed by
// boards [mid, hi) unchanged: a first-solution search splits the one board that hit its node
// budget (mid = lo + 1) without expanding the rest of its live range.  In first mode the result
// is still sorted by completion (the refined boards' children keep their order and precede
// board mid's completions).
int refine_head(sdk_ctx* c, uint64_t lo, uint64_t mid, uint64_t hi, uint64_t target) {
    if (!c->fr_valid) return fail(SDK_EINVAL, "no frontier: call sdk_frontier_build first");
    hi = std::min(hi, c->fr_size);
    lo = std::min(lo, hi);
    mid = std::min(std::max(mid, lo), hi);
    const uint64_t tail = hi - mid;
    int rc;
    if (tail) {   // the kept boards go aside first: the refinement reuses both frontier buffers
        if ((rc = ensure(c->fr_tail, tail * 81))) return rc;
        HIPCALL(hipMemcpyAsync(c->fr_tail.p, static_cast<const char*>(c->fr_a.p) + mid * 81, tail * 81,
                               hipMemcpyDeviceToDevice, c->stream));
    }
    if ((rc = refine_frontier(c, lo, 1, mid, target))) return rc;
    if (!tail) return SDK_OK;
    const uint64_t h = c->fr_size;
    c->fr_valid = false;
    if (c->fr_a.bytes < (h + tail) * 81) {
        DevBuf nb;
        if ((rc = ensure(nb, (h + tail) * 81))) return rc;
        if (h) HIPCALL(hipMemcpyAsync(nb.p, c->fr_a.p, h * 81, hipMemcpyDeviceToDevice, c->stream));
        HIPCALL(hipStreamSynchronize(c->stream));
        c->fr_a.swap(nb);          // the old buffer goes with nb
    }
    HIPCALL(hipMemcpyAsync(static_cast<char*>(c->fr_a.p) + h * 81, c->fr_tail.p, tail * 81, hipMemcpyDeviceToDevice,
                           c->stream));
    c->fr_size = h + tail;
    c->fr_valid = true;
    return SDK_OK;
}

// Lex-ordered (SDK_FRONTIER_FIRST) breadth-first expansion of n seed boards, each with its own
// first-cell mask, at least one level deep and on until the frontier holds >= target boards;
// the frontier is copied to the host.  Children keep their parents' order, so the result is
// sorted by the completions below each board (see frontier_kernel.h): the worklist step of a
// resumable lex-first search (search.py), which expands the boards that hit the node budget.
int expand_boards(sdk_ctx* c, const uint8_t* h_in, const uint16_t* h_masks, uint64_t n, uint64_t target,
                  uint8_t* h_out, uint64_t cap, uint64_t* out_n) {
    c->fr_valid = false;
    c->fr_mode = SDK_FRONTIER_FIRST;
    *out_n = 0;
    if (n == 0) return SDK_OK;
    if (n > kFrontierCap) return fail(SDK_EINVAL, "at most %llu seed boards", (unsigned long long)kFrontierCap);
    int rc;
    if ((rc = ensure(c->fr_a, frontier_capacity(n, target) * 81)) || (rc = ensure(c->fr_mask, n * 2))) return rc;
    // through the pinned staging area (see HostBuf); run_frontier_levels synchronizes before returning
    char* st = static_cast<char*>(stage_host(c->stage, n * 83));
    if (st) {
        std::memcpy(st, h_in, n * 81);
        if (h_masks) std::memcpy(st + n * 81, h_masks, n * 2);
    }
    DrainOnError drain{c->stream, true};    // also covers the pageable path's output copy
    HIPCALL(hipMemcpyAsync(c->fr_a.p, st ? st : (const char*)h_in, n * 81, hipMemcpyHostToDevice, c->stream));
    if (h_masks)
        HIPCALL(hipMemcpyAsync(c->fr_mask.p, st ? st + n * 81 : (const char*)h_masks, n * 2, hipMemcpyHostToDevice,
                               c->stream));
    if ((rc = run_frontier_levels(c, n, h_masks != nullptr, SDK_FRONTIER_FIRST, target, true))) return rc;
    if (c->fr_size > cap)
        return fail(SDK_EINVAL, "frontier of %llu boards exceeds cap %llu (pass cap >= 9 * max(n, target))",
                    (unsigned long long)c->fr_size, (unsigned long long)cap);
    if (c->fr_size) {
        char* so = static_cast<char*>(stage_host(c->stage, c->fr_size * 81));
        HIPCALL(hipMemcpyAsync(so ? so : (char*)h_out, c->fr_a.p, c->fr_size * 81, hipMemcpyDeviceToHost, c->stream));
        HIPCALL(hipStreamSynchronize(c->stream));
        if (so) std::memcpy(h_out, so, c->fr_size * 81);
    }
    HIPCALL(hipStreamSynchronize(c->stream));
    drain.armed = false;
    *out_n = c->fr_size;
    return SDK_OK;
}

// Count the completions below frontier boards first, first+step, ... < end into
// d_result = {count (u64), boards that hit the node budget (u64)}.
int frontier_count(sdk_ctx* c, uint64_t first, uint64_t step, uint64_t end, uint64_t limit,
                   unsigned long long* d_result) {
    if (!c->fr_valid) return fail(SDK_EINVAL, "no frontier: call sdk_frontier_build first");
    if (step == 0) return fail(SDK_EINVAL, "step must be >= 1");
    end = std::min(end, c->fr_size);
    const uint64_t n = first < end ? (end - first + step - 1) / step : 0;
    int rc;
    if ((rc = ensure(c->counter, 256)) || (rc = ensure(c->fr_status, std::max<uint64_t>(n, 1)))) return rc;
    unsigned long long* d_count = static_cast<unsigned long long*>(c->counter.p) + 3;
    HIPCALL(hipMemsetAsync(d_count, 0, 8, c->stream));
    if (n) {
        rc = launch_solve(c, static_cast<uint8_t*>(c->fr_a.p), nullptr, nullptr, static_cast<int8_t*>(c->fr_status.p),
                          nullptr, n, 1, limit, d_count, nullptr, first, step);
        if (rc) return rc;
    }
    sdk::count_result_kernel<<<1, 256, 0, c->stream>>>(static_cast<int8_t*>(c->fr_status.p), n, d_count, d_result);
    HIPCALL(hipGetLastError());
    return SDK_OK;
}

// Lex-ordered scan step of a first-solution search: solve frontier boards [lo, hi)
// and leave the lowest hit in d_found / d_best (first_hit_kernel).
int frontier_first(sdk_ctx* c, uint64_t lo, uint64_t hi, long long* d_found, uint8_t* d_best) {
    if (!c->fr_valid) return fail(SDK_EINVAL, "no frontier: call sdk_frontier_build first");
    hi = std::min(hi, c->fr_size);
    const uint64_t n = lo < hi ? hi - lo : 0;
    int rc;
    if ((rc = ensure(c->out, std::max<uint64_t>(n, 1) * 81)) || (rc = ensure(c->status, std::max<uint64_t>(n, 1))))
        return rc;
    if (n) {
        // boards above the lowest hit are cancelled inside the launch (solve4_kernel<.., FS>):
        // d_found is its found word until first_hit_kernel writes the answer.  The plain kernel
        // (no subtree donation: a heavy board is split by the caller, shard.sharded_solve)
        sdk::first_init_kernel<<<1, 1, 0, c->stream>>>(d_found);
        HIPCALL(hipGetLastError());
        c->first_found = d_found;
        rc = launch_solve(c, static_cast<uint8_t*>(c->fr_a.p), nullptr, static_cast<uint8_t*>(c->out.p),
                          static_cast<int8_t*>(c->status.p), nullptr, n, 0, 0, nullptr, nullptr, lo, 1, -1, -1, 0);
        c->first_found = nullptr;
        if (rc) return rc;
    }
    sdk::first_hit_kernel<<<1, 256, 0, c->stream>>>(static_cast<int8_t*>(c->status.p),
                                                    static_cast<uint8_t*>(c->out.p), n, lo, d_found, d_best);
    HIPCALL(hipGetLastError());
    return SDK_OK;
}

// Single-process form of the frontier count (sdk_count_solutions[_slice]): this
// rank's contiguous slice; rank 0 adds the leaves met during expansion.
int count_slice(sdk_ctx* c, const uint8_t* h_board, uint64_t limit, int rank, int world, uint64_t* local_count,
                uint64_t* frontier_size, int8_t* status) {
    if (world < 1 || rank < 0 || rank >= world) return fail(SDK_EINVAL, "bad rank %d / world %d", rank, world);
    int rc = build_frontier(c, h_board, nullptr, SDK_FRONTIER_COUNT,
                            (uint64_t)c->cus * (uint64_t)c->waves_per_cu * 8ull * (uint64_t)world);
    if (rc) return rc;
    const uint64_t m = c->fr_size;
    const uint64_t lo = (rank * m) / world, hi = ((rank + 1) * m) / world;
    if ((rc = ensure(c->counter, 256))) return rc;   // before taking an address inside it
    unsigned long long* d_res = static_cast<unsigned long long*>(c->counter.p) + 6;
    if ((rc = frontier_count(c, lo, 1, hi, limit, d_res))) return rc;
    unsigned long long res[2] = {0, 0};
    HIPCALL(hipMemcpyAsync(res, d_res, sizeof res, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    uint64_t cnt = res[0] + (rank == 0 ? c->fr_leaves : 0);
    if (limit && cnt > limit) cnt = limit;
    *local_count = cnt;
    if (frontier_size) *frontier_size = m;
    *status = res[1] ? (int8_t)-2 : (cnt > 0 ? (int8_t)1 : (int8_t)0);
    return SDK_OK;
}

#define NCCLCALL(expr)                                                                        \
    do {                                                                                      \
        ncclResult_t r_ = (expr);                                                             \
        if (r_ != ncclSuccess)                                                                \
            return fail(SDK_ECOMM, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_), __FILE__, __LINE__); \
    } while (0)

}  // namespace

extern "C" {

int sdk_abi_version(void) { return SDK_ABI_VERSION; }

const char* sdk_last_error(void) { return g_last_error.c_str(); }

int sdk_device_count(int* count) {
    if (!count) return fail(SDK_EINVAL, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return SDK_OK;
}

int sdk_create(int device, sdk_ctx** out) {
    if (!out) return fail(SDK_EINVAL, "out is NULL");
    *out = nullptr;
    int n = 0;
    HIPCALL(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(SDK_EINVAL, "device %d out of range (%d devices)", device, n);
    HIPCALL(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCALL(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SDK_EINVAL, "device %d is %s; this library is built for gfx950 only", device, prop.gcnArchName);
    sdk_ctx* c = new (std::nothrow) sdk_ctx();
    if (!c) return fail(SDK_ENOMEM, "context allocation failed");
    c->device = device;
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(SDK_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    (void)stage_host(c->stage, kStageInit);   // best effort: a failure leaves the pageable path
    *out = c;
    return SDK_OK;
}

int sdk_destroy(sdk_ctx* c) {
    if (!c) return SDK_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    // every DevBuf member frees itself in `delete c` below (on this device)
    if (c->stage.p) (void)hipHostFree(c->stage.p);
    for (auto& pr : c->events) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    (void)hipStreamDestroy(c->stream);
    delete c;
    return SDK_OK;
}

int sdk_set_option(sdk_ctx* c, int key, int64_t value) {
    if (!c) return fail(SDK_EINVAL, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    switch (key) {
        case SDK_OPT_ORDER:
            if (value != SDK_ORDER_MRV_UNIQUE && value != SDK_ORDER_LEX) return fail(SDK_EINVAL, "bad order %lld", (long long)value);
            c->order = (int)value;
            return SDK_OK;
        case SDK_OPT_NODE_BUDGET:
            if (value < 0) return fail(SDK_EINVAL, "budget must be >= 0");
            c->budget = (uint64_t)value;
            return SDK_OK;
        case SDK_OPT_WAVES_PER_CU:
            if (value < 1 || value > 32) return fail(SDK_EINVAL, "waves per CU must be 1..32");
            c->waves_per_cu = (int)value;
            return SDK_OK;
        case SDK_OPT_CHECK_BLOCKS_PER_CU:
            if (value < 1 || value > 16) return fail(SDK_EINVAL, "check blocks per CU must be 1..16");
            c->check_blocks_per_cu = (int)value;
            return SDK_OK;
        case SDK_OPT_WORK_COUNTER:
            if (value != SDK_WORK_NODES && value != SDK_WORK_ROUNDS && value != SDK_WORK_DEPTH)
                return fail(SDK_EINVAL, "bad work counter %lld", (long long)value);
            c->work_rounds = (int)value;
            return SDK_OK;
        case SDK_OPT_DEVICE_CUS:
            return fail(SDK_EINVAL, "SDK_OPT_DEVICE_CUS is read-only");
        case SDK_OPT_TIMER_EVENTS:
            return fail(SDK_EINVAL, "SDK_OPT_TIMER_EVENTS is read-only");
        case SDK_OPT_TIMING:
            if (value != 0 && value != 1) return fail(SDK_EINVAL, "timing must be 0 or 1");
            c->timing = value != 0;
            return SDK_OK;
        case SDK_OPT_SOLVER:
            if (value != SDK_SOLVER_WAVE && value != SDK_SOLVER_HALFWAVE && value != SDK_SOLVER_QUAD &&
                value != SDK_SOLVER_LANE)
                return fail(SDK_EINVAL, "bad solver %lld", (long long)value);
            c->solver = (int)value;
            return SDK_OK;
        case SDK_OPT_WAVES_PER_CU2:
            if (value < 1 || value > 32) return fail(SDK_EINVAL, "waves per CU must be 1..32");
            c->waves_per_cu2 = (int)value;
            return SDK_OK;
        case SDK_OPT_SOLVE_CHUNK:
            if (value < 0 || value > 4096) return fail(SDK_EINVAL, "solve chunk must be 0..4096");
            c->solve_chunk = (int)value;
            return SDK_OK;
        case SDK_OPT_LOCKED:
            if (value < 0 || value > 2) return fail(SDK_EINVAL, "locked must be 0, 1 or 2");
            c->locked = (int)value;
            return SDK_OK;
        case SDK_OPT_DONATED:
            return fail(SDK_EINVAL, "SDK_OPT_DONATED is read-only");
        case SDK_OPT_SPLIT_BOARDS:
            return fail(SDK_EINVAL, "SDK_OPT_SPLIT_BOARDS is read-only");
        case SDK_OPT_RESUMED:
            return fail(SDK_EINVAL, "SDK_OPT_RESUMED is read-only");
        case SDK_OPT_LEX_BOARDS:
            return fail(SDK_EINVAL, "SDK_OPT_LEX_BOARDS is read-only");
        case SDK_OPT_DONATE_MAX:
            if (value < 0) return fail(SDK_EINVAL, "SDK_OPT_DONATE_MAX must be >= 0");
            c->dn_max = value;
            return SDK_OK;
        case SDK_OPT_DN_FAULT:
            if (value != 0 && value != 1) return fail(SDK_EINVAL, "SDK_OPT_DN_FAULT must be 0 or 1");
            c->dn_fault = (int)value;
            return SDK_OK;
        case SDK_OPT_DONATE_HELPERS:
            if (value < 1 || value > 4096) return fail(SDK_EINVAL, "SDK_OPT_DONATE_HELPERS must be 1..4096");
            c->dn_helpers = (int)value;
            return SDK_OK;
        case SDK_OPT_DONATE_RESUME:
            if (value != 0 && value != 1) return fail(SDK_EINVAL, "SDK_OPT_DONATE_RESUME must be 0 or 1");
            c->dn_resume = (int)value;
            return SDK_OK;
        case SDK_OPT_DONATE_MODE:
            if (value != 0 && value != 1) return fail(SDK_EINVAL, "donate mode must be 0 (LEX) or 1 (exhaustive)");
            c->dn_exhaustive = (int)value;
            return SDK_OK;
        case SDK_OPT_DONATE:
            if (value < 0 || value > (1 << 30)) return fail(SDK_EINVAL, "donate must be 0, 1 or a split budget >= 2");
            c->donate = (int)value;
            return SDK_OK;
        case SDK_OPT_PROP32:
            if (value != 0 && value != 1) return fail(SDK_EINVAL, "SDK_OPT_PROP32 is 0 or 1");
            c->prop32 = (int)value;
            return SDK_OK;
        case SDK_OPT_PROP32_LC:
            if ((value & 0xFF) < 1 || (value & 0xFF) > 64 || (value >> 8) > 64)
                return fail(SDK_EINVAL, "SDK_OPT_PROP32_LC: period 1..64 | first step 0..64 << 8");
            c->prop32_lc = (int)value;
            return SDK_OK;
        case SDK_OPT_PROP32_MIN:
            if (value < 1) return fail(SDK_EINVAL, "SDK_OPT_PROP32_MIN must be >= 1");
            c->prop32_min = value;
            return SDK_OK;
        case SDK_OPT_PROP32_HANDOVER:
            if (value != 0 && value != 1) return fail(SDK_EINVAL, "SDK_OPT_PROP32_HANDOVER is 0 or 1");
            c->prop32_handover = (int)value;
            return SDK_OK;
        case SDK_OPT_PROP32_TAIL:
            if (value < 0 || (value & 0xFF) > 64 || (value >> 8) > 96) return fail(SDK_EINVAL, "SDK_OPT_PROP32_TAIL out of range");
            c->prop32_tail_live = (int)(value & 0xFF);
            c->prop32_tail_step = (int)(value >> 8);
            return SDK_OK;
        case SDK_OPT_XCD_HEADS:
            if (value != 0 && value != 1) return fail(SDK_EINVAL, "xcd heads must be 0 or 1");
            c->xcd_heads = (int)value;
            return SDK_OK;
        case SDK_OPT_CHECK_VARIANT:
            if (value < SDK_CHECK_REG1 || value > SDK_CHECK_WAVE2) return fail(SDK_EINVAL, "bad check variant %lld", (long long)value);
            c->check_variant = (int)value;
            return SDK_OK;
        default:
            return fail(SDK_EINVAL, "unknown option %d", key);
    }
}

// diagnostics (not in the header): the donation control block of the last donating launch
extern "C" int sdk_debug_dn_ctl(sdk_ctx* c, uint32_t* out16) {
    if (!c || !out16) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    std::memset(out16, 0, 64);
    if (!c->dn.p) return SDK_OK;
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipMemcpyAsync(out16, c->dn.p, 64, hipMemcpyDeviceToHost, c->stream));   // the global words
    HIPCALL(hipStreamSynchronize(c->stream));
    return SDK_OK;
}

// diagnostics (not in the header): the in-kernel clock of the prop32 pass.  Armed, the context's
// prop32 passes run prop32_clock_kernel, which stamps s_memtime / s_memrealtime at each workgroup's
// entry and exit; _read waits for the last such pass and returns the shader clock of its workgroups
// (GHz: shader ticks per 10 ns of the 100 MHz real-time counter) as median, 10th and 90th percentile
// and mean (out4), and how many workgroups it had.  (MI355X_MICROARCH.md, "DVFS give-back" item 6.)
extern "C" int sdk_debug_clock_arm(sdk_ctx* c, int on) {
    if (!c) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    c->clock_probe = on ? 1 : 0;
    return SDK_OK;
}

extern "C" int sdk_debug_clock_read(sdk_ctx* c, double* out4, int64_t* workgroups) {
    if (!c || !out4 || !workgroups) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    *workgroups = 0;
    for (int i = 0; i < 4; ++i) out4[i] = 0.0;
    if (!c->p32_stamp_wgs || !c->p32_stamps.p) return SDK_OK;
    HIPCALL(hipSetDevice(c->device));
    std::vector<uint64_t> h((size_t)c->p32_stamp_wgs * 4);
    HIPCALL(hipMemcpyAsync(h.data(), c->p32_stamps.p, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    std::vector<double> ghz;
    ghz.reserve(c->p32_stamp_wgs);
    for (size_t w = 0; w < c->p32_stamp_wgs; ++w) {
        const uint64_t dt = h[4 * w + 2] - h[4 * w], dr = h[4 * w + 3] - h[4 * w + 1];
        if (dr >= 10 && h[4 * w + 2] > h[4 * w]) ghz.push_back((double)dt / (double)dr / 10.0);   // >= 0.1 us
    }
    if (ghz.empty()) return SDK_OK;
    std::sort(ghz.begin(), ghz.end());
    double sum = 0.0;
    for (double v : ghz) sum += v;
    out4[0] = ghz[ghz.size() / 2];
    out4[1] = ghz[ghz.size() / 10];
    out4[2] = ghz[(ghz.size() * 9) / 10];
    out4[3] = sum / (double)ghz.size();
    *workgroups = (int64_t)ghz.size();
    return SDK_OK;
}

namespace {
// a phased solve's board counts (dn_stat) wait for it on the context's stream
int read_dn_stat(sdk_ctx* c, int k, int64_t* value) {
    *value = 0;
    if (!c->dn_ran || !c->dn_stat.p) return SDK_OK;
    HIPCALL(hipSetDevice(c->device));
    uint32_t v = 0;
    HIPCALL(hipMemcpyAsync(&v, static_cast<uint32_t*>(c->dn_stat.p) + k, sizeof v, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    *value = v;
    return SDK_OK;
}

// The sticky error words of the two donation areas (a bounded wait on another wave inside a
// donation launch ran out, solve4_kernel.h kDnWaitTicks): read once after a phased solve,
// cleared, and turned into SDK_EHIP -- the solve's boards are then not valid.
int dn_check_error(sdk_ctx* c) {
    if (!c->dn_err_check || !c->dn.p) return SDK_OK;
    c->dn_err_check = false;
    uint32_t e[2] = {0u, 0u};
    for (int k = 0; k < 2; ++k)
        HIPCALL(hipMemcpyAsync(&e[k], static_cast<char*>(c->dn.p) + (size_t)k * sdk::kDnBytes + offsetof(sdk::DnCtl, err),
                               sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    const uint32_t err = e[0] | e[1];
    if (err == 0u) return SDK_OK;
    for (int k = 0; k < 2; ++k)
        HIPCALL(hipMemsetAsync(static_cast<char*>(c->dn.p) + (size_t)k * sdk::kDnBytes + offsetof(sdk::DnCtl, err), 0,
                               sizeof(uint32_t), c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    if (err & sdk::kDnErrSeed)
        return fail(SDK_EHIP, "donation launch: a resumed board's items disagree with their reservation; the "
                    "solve's boards are not valid");
    return fail(SDK_EHIP, "donation launch: a bounded wait on another wave ran out (%s%s); the solve's boards are "
                "not valid", (err & sdk::kDnErrReg) ? "registration entry never written " : "",
                (err & sdk::kDnErrLock) ? "record lock never released" : "");
}
}  // namespace

int sdk_get_option(sdk_ctx* c, int key, int64_t* value) {
    if (!c || !value) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    switch (key) {
        case SDK_OPT_ORDER: *value = c->order; return SDK_OK;
        case SDK_OPT_NODE_BUDGET: *value = (int64_t)c->budget; return SDK_OK;
        case SDK_OPT_WAVES_PER_CU: *value = c->waves_per_cu; return SDK_OK;
        case SDK_OPT_CHECK_BLOCKS_PER_CU: *value = c->check_blocks_per_cu; return SDK_OK;
        case SDK_OPT_WORK_COUNTER: *value = c->work_rounds; return SDK_OK;
        case SDK_OPT_DEVICE_CUS: *value = c->cus; return SDK_OK;
        case SDK_OPT_SOLVER: *value = c->solver; return SDK_OK;
        case SDK_OPT_WAVES_PER_CU2: *value = c->waves_per_cu2; return SDK_OK;
        case SDK_OPT_CHECK_VARIANT: *value = c->check_variant; return SDK_OK;
        case SDK_OPT_SOLVE_CHUNK: *value = c->solve_chunk; return SDK_OK;
        case SDK_OPT_TIMING: *value = c->timing ? 1 : 0; return SDK_OK;
        case SDK_OPT_LOCKED: *value = c->locked; return SDK_OK;
        case SDK_OPT_XCD_HEADS: *value = c->xcd_heads; return SDK_OK;
        case SDK_OPT_PROP32: *value = c->prop32; return SDK_OK;
        case SDK_OPT_PROP32_LC: *value = c->prop32_lc; return SDK_OK;
        case SDK_OPT_PROP32_MIN: *value = c->prop32_min; return SDK_OK;
        case SDK_OPT_PROP32_HANDOVER: *value = c->prop32_handover; return SDK_OK;
        case SDK_OPT_PROP32_TAIL: *value = c->prop32_tail_live | (c->prop32_tail_step << 8); return SDK_OK;
        case SDK_OPT_PROP32_UNDECIDED: {
            *value = 0;
            if (!c->prop32_ran) return SDK_OK;
            HIPCALL(hipSetDevice(c->device));
            uint32_t v = 0;
            HIPCALL(hipMemcpyAsync(&v, c->p32_list.p, sizeof v, hipMemcpyDeviceToHost, c->stream));
            HIPCALL(hipStreamSynchronize(c->stream));
            *value = v;
            return SDK_OK;
        }
        case SDK_OPT_DONATE: *value = c->donate; return SDK_OK;
        case SDK_OPT_SPLIT_BOARDS: return read_dn_stat(c, 0, value);
        case SDK_OPT_DONATE_MODE: *value = c->dn_exhaustive; return SDK_OK;
        case SDK_OPT_LEX_BOARDS: return read_dn_stat(c, 1, value);
        case SDK_OPT_DONATE_MAX: *value = c->dn_max; return SDK_OK;
        case SDK_OPT_DN_FAULT: *value = c->dn_fault; return SDK_OK;
        case SDK_OPT_DONATE_HELPERS: *value = c->dn_helpers; return SDK_OK;
        case SDK_OPT_DONATE_RESUME: *value = c->dn_resume; return SDK_OK;
        case SDK_OPT_DONATED: {
            // items handed out by the last phased solve's donation launches (of its last
            // kDnCapBoards-board pass; waits for it on the context's stream)
            *value = 0;
            if (!c->dn.p || c->dn_epoch == 0 || !c->dn_ran) return SDK_OK;
            HIPCALL(hipSetDevice(c->device));
            sdk::DnCtl h[2];
            for (int k = 0; k < 2; ++k)
                HIPCALL(hipMemcpyAsync(&h[k], static_cast<char*>(c->dn.p) + (size_t)k * sdk::kDnBytes, sizeof h[k],
                                       hipMemcpyDeviceToHost, c->stream));
            HIPCALL(hipStreamSynchronize(c->stream));
            *value = (int64_t)h[0].delivered + (int64_t)h[1].delivered;
            return SDK_OK;
        }
        case SDK_OPT_RESUMED: {
            // boards the last phased solve resumed (donation area 0; waits for the solve)
            *value = 0;
            if (!c->dn.p || c->dn_epoch == 0 || !c->dn_ran) return SDK_OK;
            HIPCALL(hipSetDevice(c->device));
            sdk::DnSeed h;
            HIPCALL(hipMemcpyAsync(&h, static_cast<char*>(c->dn.p) + offsetof(sdk::DnCtl, seed), sizeof h,
                                   hipMemcpyDeviceToHost, c->stream));
            HIPCALL(hipStreamSynchronize(c->stream));
            *value = (int64_t)h.boards;
            return SDK_OK;
        }
        case SDK_OPT_TIMER_EVENTS: *value = (int64_t)c->events.size(); return SDK_OK;
        default: return fail(SDK_EINVAL, "unknown option %d", key);
    }
}

int sdk_dev_alloc(sdk_ctx* c, size_t bytes, void** dptr) {
    if (!c || !dptr) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipMalloc(dptr, std::max(bytes, (size_t)16)));
    return SDK_OK;
}

int sdk_dev_free(sdk_ctx* c, void* dptr) {
    if (!c) return fail(SDK_EINVAL, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipStreamSynchronize(c->stream));
    if (dptr) HIPCALL(hipFree(dptr));
    return SDK_OK;
}

int sdk_memcpy_h2d(sdk_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c || (!dst && bytes) || (!src && bytes)) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    return SDK_OK;
}

int sdk_memcpy_d2h(sdk_ctx* c, void* dst, const void* src, size_t bytes) {
    if (!c || (!dst && bytes) || (!src && bytes)) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    return dn_check_error(c);
}

int sdk_synchronize(sdk_ctx* c) {
    if (!c) return fail(SDK_EINVAL, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipStreamSynchronize(c->stream));
    return dn_check_error(c);
}

int sdk_timer_reset(sdk_ctx* c) {
    if (!c) return fail(SDK_EINVAL, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipStreamSynchronize(c->stream));
    c->events_used = 0;
    return SDK_OK;
}

int sdk_timer_read(sdk_ctx* c, double* total_ms, int64_t* launches) {
    if (!c || !total_ms || !launches) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    double tot = 0;
    for (size_t i = 0; i < c->events_used; ++i) {
        float ms = 0.f;
        HIPCALL(hipEventElapsedTime(&ms, c->events[i].first, c->events[i].second));
        tot += ms;
    }
    *total_ms = tot;
    *launches = (int64_t)c->events_used;
    return SDK_OK;
}

// diagnostics (not in the header): durations of the timed launches since sdk_timer_reset
extern "C" int sdk_debug_timer_list(sdk_ctx* c, double* ms, int64_t cap, int64_t* n) {
    if (!c || !ms || !n) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    *n = (int64_t)c->events_used;
    for (size_t i = 0; i < c->events_used && (int64_t)i < cap; ++i) {
        float v = 0.f;
        HIPCALL(hipEventElapsedTime(&v, c->events[i].first, c->events[i].second));
        ms[i] = v;
    }
    return SDK_OK;
}

int sdk_check_batch_dev(sdk_ctx* c, const void* d_boards, void* d_verdict, size_t n) {
    if (!c || (n && (!d_boards || !d_verdict))) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return launch_check(c, static_cast<const uint8_t*>(d_boards), static_cast<uint8_t*>(d_verdict), n);
}

int sdk_solve_batch_dev(sdk_ctx* c, const void* d_in, const void* d_mask, void* d_out, void* d_status,
                        void* d_work, size_t n) {
    if (!c || (n && (!d_in || !d_out || !d_status))) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return launch_solve(c, static_cast<const uint8_t*>(d_in), static_cast<const uint16_t*>(d_mask),
                        static_cast<uint8_t*>(d_out), static_cast<int8_t*>(d_status), static_cast<uint64_t*>(d_work),
                        n, 0, 0, nullptr);
}

int sdk_check_batch(sdk_ctx* c, const uint8_t* boards, uint8_t* verdict, size_t n) {
    if (!c || (n && (!boards || !verdict))) return fail(SDK_EINVAL, "NULL argument");
    if (n == 0) return SDK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c->in, n * 81)) || (rc = ensure(c->verdict, n))) return rc;
    HIPCALL(hipMemcpyAsync(c->in.p, boards, n * 81, hipMemcpyHostToDevice, c->stream));
    if ((rc = launch_check(c, static_cast<uint8_t*>(c->in.p), static_cast<uint8_t*>(c->verdict.p), n))) return rc;
    HIPCALL(hipMemcpyAsync(verdict, c->verdict.p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    return SDK_OK;
}

int sdk_check_batch_i64(sdk_ctx* c, const int64_t* boards, uint8_t* verdict, size_t n) {
    if (!c || (n && (!boards || !verdict))) return fail(SDK_EINVAL, "NULL argument");
    if (n == 0) return SDK_OK;
    for (size_t k = 0; k < n * 81; ++k)
        if (boards[k] >= (1ll << 59) || boards[k] <= -(1ll << 59))
            return fail(SDK_EINVAL, "cell value %lld out of the checker's range (|v| < 2^59)", (long long)boards[k]);
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c->in, n * 81 * sizeof(int64_t))) || (rc = ensure(c->verdict, n))) return rc;
    HIPCALL(hipMemcpyAsync(c->in.p, boards, n * 81 * sizeof(int64_t), hipMemcpyHostToDevice, c->stream));
    hipEvent_t stop;
    if ((rc = timer_begin(c, &stop))) return rc;
    const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, (uint64_t)c->cus * 8);
    sdk::check_kernel_i64<<<grid, 256, 0, c->stream>>>(static_cast<const int64_t*>(c->in.p),
                                                      static_cast<uint8_t*>(c->verdict.p), (uint64_t)n);
    HIPCALL(hipGetLastError());
    if ((rc = timer_end(c, stop))) return rc;
    HIPCALL(hipMemcpyAsync(verdict, c->verdict.p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    return SDK_OK;
}

int sdk_solve_batch(sdk_ctx* c, const uint8_t* in, const uint16_t* first_cell_mask, uint8_t* out, int8_t* status,
                    uint64_t* work, size_t n) {
    return sdk_solve_batch_budget(c, in, first_cell_mask, out, status, work, n, SDK_BUDGET_CONTEXT);
}

int sdk_solve_batch_budget(sdk_ctx* c, const uint8_t* in, const uint16_t* first_cell_mask, uint8_t* out,
                           int8_t* status, uint64_t* work, size_t n, uint64_t node_budget) {
    return sdk_solve_batch_ex(c, in, first_cell_mask, out, status, work, n, node_budget, SDK_DONATE_CONTEXT);
}

int sdk_solve_batch_ex(sdk_ctx* c, const uint8_t* in, const uint16_t* first_cell_mask, uint8_t* out, int8_t* status,
                       uint64_t* work, size_t n, uint64_t node_budget, int64_t donate) {
    if (!c || (n && (!in || !out || !status))) return fail(SDK_EINVAL, "NULL argument");
    if (node_budget != SDK_BUDGET_CONTEXT && node_budget > (uint64_t)INT64_MAX)
        return fail(SDK_EINVAL, "node budget out of range");
    if (donate < SDK_DONATE_CONTEXT || donate > (1 << 30))
        return fail(SDK_EINVAL, "donate must be SDK_DONATE_CONTEXT, 0, 1 or a split budget >= 2");
    if (n == 0) return SDK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c->in, n * 81)) || (rc = ensure(c->out, n * 81)) || (rc = ensure(c->status, n))) return rc;
    if (first_cell_mask && (rc = ensure(c->mask, n * 2))) return rc;
    if (work && (rc = ensure(c->work, n * 8))) return rc;
    // staging layout: work (n x 8), masks (n x 2), in / out boards (n x 81), status (n)
    char* st = static_cast<char*>(stage_host(c->stage, n * (8 + 2 + 81 + 1)));
    uint64_t* s_work = reinterpret_cast<uint64_t*>(st);
    uint16_t* s_mask = st ? reinterpret_cast<uint16_t*>(st + n * 8) : nullptr;
    uint8_t* s_io = st ? reinterpret_cast<uint8_t*>(st + n * 10) : nullptr;
    int8_t* s_st = st ? reinterpret_cast<int8_t*>(st + n * 91) : nullptr;
    if (st) {
        std::memcpy(s_io, in, n * 81);
        if (first_cell_mask) std::memcpy(s_mask, first_cell_mask, n * 2);
    }
    DrainOnError drain{c->stream, st != nullptr};
    HIPCALL(hipMemcpyAsync(c->in.p, st ? s_io : in, n * 81, hipMemcpyHostToDevice, c->stream));
    if (first_cell_mask)
        HIPCALL(hipMemcpyAsync(c->mask.p, st ? s_mask : first_cell_mask, n * 2, hipMemcpyHostToDevice, c->stream));
    rc = launch_solve(c, static_cast<uint8_t*>(c->in.p), first_cell_mask ? static_cast<uint16_t*>(c->mask.p) : nullptr,
                      static_cast<uint8_t*>(c->out.p), static_cast<int8_t*>(c->status.p),
                      work ? static_cast<uint64_t*>(c->work.p) : nullptr, n, 0, 0, nullptr, nullptr, 0, 1, -1,
                      node_budget == SDK_BUDGET_CONTEXT ? -1 : (int64_t)node_budget, donate);
    if (rc) return rc;
    HIPCALL(hipMemcpyAsync(st ? s_io : out, c->out.p, n * 81, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipMemcpyAsync(st ? s_st : status, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
    if (work) HIPCALL(hipMemcpyAsync(st ? s_work : work, c->work.p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    drain.armed = false;
    if (st) {
        std::memcpy(out, s_io, n * 81);
        std::memcpy(status, s_st, n);
        if (work) std::memcpy(work, s_work, n * 8);
    }
    return dn_check_error(c);
}

int sdk_count_solutions(sdk_ctx* c, const uint8_t* board, uint64_t limit, uint64_t* count, int8_t* status) {
    if (!c || !board || !count || !status) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return count_slice(c, board, limit, 0, 1, count, nullptr, status);
}

int sdk_count_solutions_slice(sdk_ctx* c, const uint8_t* board, uint64_t limit, int rank, int world,
                              uint64_t* count, uint64_t* frontier_size, int8_t* status) {
    if (!c || !board || !count || !status) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return count_slice(c, board, limit, rank, world, count, frontier_size, status);
}

int sdk_frontier_build(sdk_ctx* c, const uint8_t* board, const uint16_t* first_cell_mask, int mode, uint64_t target,
                       uint64_t* size, uint64_t* leaves) {
    if (!c || !board) return fail(SDK_EINVAL, "NULL argument");
    if (mode != SDK_FRONTIER_COUNT && mode != SDK_FRONTIER_FIRST) return fail(SDK_EINVAL, "bad frontier mode %d", mode);
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc = build_frontier(c, board, first_cell_mask, mode, target);
    if (rc) return rc;
    if (size) *size = c->fr_size;
    if (leaves) *leaves = c->fr_leaves;
    return SDK_OK;
}

int sdk_expand_boards(sdk_ctx* c, const uint8_t* boards, const uint16_t* first_cell_masks, size_t n,
                      uint64_t target, uint8_t* out, size_t cap, uint64_t* out_n) {
    if (!c || !out_n || (n && (!boards || !out))) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return expand_boards(c, boards, first_cell_masks, n, target, out, cap, out_n);
}

int sdk_frontier_refine(sdk_ctx* c, uint64_t first, uint64_t step, uint64_t target, uint64_t* size,
                        uint64_t* leaves) {
    if (!c) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc = refine_frontier(c, first, step, UINT64_MAX, target);
    if (rc) return rc;
    if (size) *size = c->fr_size;
    if (leaves) *leaves = c->fr_leaves;
    return SDK_OK;
}

int sdk_frontier_refine_range(sdk_ctx* c, uint64_t lo, uint64_t hi, uint64_t target, uint64_t* size,
                              uint64_t* leaves) {
    if (!c) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc = refine_frontier(c, lo, 1, hi, target);
    if (rc) return rc;
    if (size) *size = c->fr_size;
    if (leaves) *leaves = c->fr_leaves;
    return SDK_OK;
}

int sdk_frontier_refine_head(sdk_ctx* c, uint64_t lo, uint64_t mid, uint64_t hi, uint64_t target, uint64_t* size,
                             uint64_t* leaves) {
    if (!c) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc = refine_head(c, lo, mid, hi, target);
    if (rc) return rc;
    if (size) *size = c->fr_size;
    if (leaves) *leaves = c->fr_leaves;
    return SDK_OK;
}

int sdk_frontier_boards_dev(sdk_ctx* c, void** d_boards, uint64_t* size) {
    if (!c || !d_boards || !size) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->fr_valid) return fail(SDK_EINVAL, "no frontier: call sdk_frontier_build first");
    *d_boards = c->fr_a.p;
    *size = c->fr_size;
    return SDK_OK;
}

int sdk_frontier_load_dev(sdk_ctx* c, const void* d_boards, uint64_t n) {
    if (!c || (n && !d_boards)) return fail(SDK_EINVAL, "NULL argument");
    if (n > kFrontierCap) return fail(SDK_EINVAL, "at most %llu frontier boards", (unsigned long long)kFrontierCap);
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    c->fr_valid = false;
    const char* src = static_cast<const char*>(d_boards);
    const char* a0 = static_cast<const char*>(c->fr_a.p);
    if (n && src == a0) {
        c->fr_size = n;                     // already in place
    } else if (n && a0 && src > a0 && src < a0 + c->fr_a.bytes) {
        // a range of the current frontier (overlapping copy): through fr_b
        int rc;
        if ((rc = ensure(c->fr_b, n * 81))) return rc;
        HIPCALL(hipMemcpyAsync(c->fr_b.p, d_boards, n * 81, hipMemcpyDeviceToDevice, c->stream));
        std::swap(c->fr_a, c->fr_b);
        c->fr_size = n;
    } else {
        int rc;
        if ((rc = ensure(c->fr_a, std::max<uint64_t>(n, 1) * 81))) return rc;
        if (n) HIPCALL(hipMemcpyAsync(c->fr_a.p, d_boards, n * 81, hipMemcpyDeviceToDevice, c->stream));
        c->fr_size = n;
    }
    c->fr_leaves = 0;
    c->fr_levels = 0;
    c->fr_valid = true;
    return SDK_OK;
}

int sdk_frontier_count_dev(sdk_ctx* c, uint64_t first, uint64_t step, uint64_t end, uint64_t limit, void* d_result) {
    if (!c || !d_result) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return frontier_count(c, first, step, end, limit, static_cast<unsigned long long*>(d_result));
}

int sdk_frontier_first_dev(sdk_ctx* c, uint64_t lo, uint64_t hi, void* d_found, void* d_best) {
    if (!c || !d_found || !d_best) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return frontier_first(c, lo, hi, static_cast<long long*>(d_found), static_cast<uint8_t*>(d_best));
}

int sdk_comm_unique_id(uint8_t* id) {
    if (!id) return fail(SDK_EINVAL, "NULL argument");
    ncclUniqueId u;
    NCCLCALL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, SDK_COMM_ID_BYTES);
    return SDK_OK;
}

int sdk_comm_init(sdk_ctx* c, const uint8_t* id, int rank, int world) {
    if (!c || !id) return fail(SDK_EINVAL, "NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return fail(SDK_EINVAL, "bad rank %d / world %d", rank, world);
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->comm) return fail(SDK_EINVAL, "context already has a communicator");
    HIPCALL(hipSetDevice(c->device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, SDK_COMM_ID_BYTES);
    NCCLCALL(ncclCommInitRank(&c->comm, world, u, rank));
    c->comm_rank = rank;
    c->comm_world = world;
    return SDK_OK;
}

int sdk_comm_init_all(const int* devices, int ndev, sdk_ctx** ctxs) {
    if (!devices || !ctxs || ndev < 1) return fail(SDK_EINVAL, "need ndev >= 1 devices and contexts");
    for (int k = 0; k < ndev; ++k) {
        ctxs[k] = nullptr;
        for (int j = 0; j < k; ++j)
            if (devices[j] == devices[k]) return fail(SDK_EINVAL, "device %d listed twice", devices[k]);
    }
    int rc = SDK_OK;
    for (int k = 0; k < ndev && rc == SDK_OK; ++k) rc = sdk_create(devices[k], &ctxs[k]);
    std::vector<ncclComm_t> comms(ndev, nullptr);
    if (rc == SDK_OK) {
        const ncclResult_t r = ncclCommInitAll(comms.data(), ndev, devices);
        if (r != ncclSuccess) rc = fail(SDK_ECOMM, "ncclCommInitAll: %s", ncclGetErrorString(r));
    }
    if (rc != SDK_OK) {
        const std::string msg = g_last_error;
        for (int k = 0; k < ndev; ++k) {
            if (ctxs[k]) (void)sdk_destroy(ctxs[k]);
            ctxs[k] = nullptr;
        }
        g_last_error = msg;
        return rc;
    }
    for (int k = 0; k < ndev; ++k) {
        ctxs[k]->comm = comms[k];
        ctxs[k]->comm_rank = k;
        ctxs[k]->comm_world = ndev;
    }
    return SDK_OK;
}

int sdk_comm_destroy(sdk_ctx* c) {
    if (!c) return fail(SDK_EINVAL, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->comm) return SDK_OK;
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipStreamSynchronize(c->stream));
    ncclComm_t comm = c->comm;
    c->comm = nullptr;
    c->comm_rank = 0;
    c->comm_world = 1;
    NCCLCALL(ncclCommDestroy(comm));
    return SDK_OK;
}

int sdk_comm_allreduce_dev(sdk_ctx* c, void* d_buf, size_t count, int dtype, int op) {
    if (!c || (count && !d_buf)) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->comm) return fail(SDK_EINVAL, "no communicator: call sdk_comm_init first");
    ncclDataType_t t;
    switch (dtype) {
        case SDK_COMM_U64: t = ncclUint64; break;
        case SDK_COMM_I64: t = ncclInt64; break;
        case SDK_COMM_U8: t = ncclUint8; break;
        default: return fail(SDK_EINVAL, "bad dtype %d", dtype);
    }
    ncclRedOp_t o;
    switch (op) {
        case SDK_COMM_SUM: o = ncclSum; break;
        case SDK_COMM_MIN: o = ncclMin; break;
        case SDK_COMM_MAX: o = ncclMax; break;
        default: return fail(SDK_EINVAL, "bad op %d", op);
    }
    HIPCALL(hipSetDevice(c->device));
    NCCLCALL(ncclAllReduce(d_buf, d_buf, count, t, o, c->comm, c->stream));
    return SDK_OK;
}

int sdk_comm_broadcast_dev(sdk_ctx* c, void* d_buf, size_t bytes, int root) {
    if (!c || (bytes && !d_buf)) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->comm) return fail(SDK_EINVAL, "no communicator: call sdk_comm_init first");
    if (root < 0 || root >= c->comm_world) return fail(SDK_EINVAL, "bad root %d", root);
    HIPCALL(hipSetDevice(c->device));
    NCCLCALL(ncclBroadcast(d_buf, d_buf, bytes, ncclUint8, root, c->comm, c->stream));
    return SDK_OK;
}

int sdk_comm_p2p_dev(sdk_ctx* c, int nops, const int* ops, const int* peers, void* const* bufs, const size_t* bytes) {
    if (!c || nops < 0 || (nops && (!ops || !peers || !bufs || !bytes))) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->comm) return fail(SDK_EINVAL, "no communicator: call sdk_comm_init first");
    for (int k = 0; k < nops; ++k) {
        if (ops[k] != SDK_COMM_SEND && ops[k] != SDK_COMM_RECV) return fail(SDK_EINVAL, "bad p2p op %d", ops[k]);
        if (peers[k] < 0 || peers[k] >= c->comm_world || peers[k] == c->comm_rank)
            return fail(SDK_EINVAL, "bad p2p peer %d (rank %d of %d)", peers[k], c->comm_rank, c->comm_world);
        if (bytes[k] && !bufs[k]) return fail(SDK_EINVAL, "NULL p2p buffer");
    }
    HIPCALL(hipSetDevice(c->device));
    NCCLCALL(ncclGroupStart());
    ncclResult_t r = ncclSuccess;
    for (int k = 0; k < nops && r == ncclSuccess; ++k) {
        if (!bytes[k]) continue;   // both sides of a pair agree on the size, so both skip
        r = ops[k] == SDK_COMM_SEND ? ncclSend(bufs[k], bytes[k], ncclUint8, peers[k], c->comm, c->stream)
                                    : ncclRecv(bufs[k], bytes[k], ncclUint8, peers[k], c->comm, c->stream);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess) return fail(SDK_ECOMM, "ncclSend/ncclRecv: %s", ncclGetErrorString(r));
    if (r2 != ncclSuccess) return fail(SDK_ECOMM, "ncclGroupEnd: %s", ncclGetErrorString(r2));
    return SDK_OK;
}

int sdk_comm_send_dev(sdk_ctx* c, const void* d_buf, size_t bytes, int peer) {
    const int op = SDK_COMM_SEND;
    void* buf = const_cast<void*>(d_buf);
    return sdk_comm_p2p_dev(c, 1, &op, &peer, &buf, &bytes);
}

int sdk_comm_recv_dev(sdk_ctx* c, void* d_buf, size_t bytes, int peer) {
    const int op = SDK_COMM_RECV;
    return sdk_comm_p2p_dev(c, 1, &op, &peer, &d_buf, &bytes);
}

int sdk_comm_allgather_dev(sdk_ctx* c, const void* d_send, void* d_recv, size_t bytes) {
    if (!c || (bytes && (!d_send || !d_recv))) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    if (!c->comm) return fail(SDK_EINVAL, "no communicator: call sdk_comm_init first");
    HIPCALL(hipSetDevice(c->device));
    NCCLCALL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, c->comm, c->stream));
    return SDK_OK;
}

}  // extern "C"
