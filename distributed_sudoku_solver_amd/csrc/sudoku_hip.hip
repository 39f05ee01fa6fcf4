// sudoku_hip.hip -- libsudoku_hip.so: C-ABI (include/sudoku_hip.h) over the gfx950 kernels.
//
// Host side is deliberately thin: a context = (device, stream, grow-only device
// workspaces, HIP event pairs for kernel timing, options) behind a mutex.  No
// CPU compute path exists: every board is checked / solved by a HIP kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
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

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

struct sdk_ctx {
    int device = 0;
    int cus = 256;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // options
    int order = SDK_ORDER_MRV_UNIQUE;
    uint64_t budget = 0;
    int waves_per_cu = 32;
    int check_blocks_per_cu = 3;
    // workspaces
    DevBuf stack, counter, in, mask, out, status, work, verdict;
    DevBuf fr_a, fr_b, prop, bcell, bmask, nchild, offs, fr_status;
    // timing
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    size_t events_used = 0;
};

namespace {

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

int timer_begin(sdk_ctx* c, hipEvent_t* stop_out) {
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

int launch_check(sdk_ctx* c, const uint8_t* d_in, uint8_t* d_out, size_t n) {
    if (n == 0) return SDK_OK;
    if (reinterpret_cast<uintptr_t>(d_in) & 15) return fail(SDK_EINVAL, "device boards must be 16-byte aligned");
    const uint64_t tiles = (n + sdk::kCheckThreads - 1) / sdk::kCheckThreads;
    const unsigned grid = (unsigned)std::min<uint64_t>(tiles, (uint64_t)c->cus * c->check_blocks_per_cu);
    hipEvent_t stop;
    int rc = timer_begin(c, &stop);
    if (rc) return rc;
    sdk::check_kernel<<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n);
    HIPCALL(hipGetLastError());
    HIPCALL(hipEventRecord(stop, c->stream));
    return SDK_OK;
}

int launch_solve(sdk_ctx* c, const uint8_t* d_in, const uint16_t* d_mask, uint8_t* d_out, int8_t* d_status,
                 uint64_t* d_work, size_t n, int count_mode, uint64_t limit, unsigned long long* d_count,
                 unsigned long long* d_counts = nullptr) {
    if (n == 0) return SDK_OK;
    if (n > 0x7FFFFFFFull) return fail(SDK_EINVAL, "at most 2^31-1 boards per call");
    const uint64_t slots = (uint64_t)c->cus * c->waves_per_cu;
    // ~16 dequeues per wave over the launch, 1..64 boards each; count mode uses
    // single boards (subtrees differ by orders of magnitude)
    const uint32_t chunk = count_mode ? 1u : (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, n / (slots * 16)));
    const uint64_t want = (n + chunk - 1) / chunk;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, slots));
    int rc = ensure(c->stack, (size_t)grid * sdk::kStackWordsPerBlock * sizeof(uint32_t));
    if (rc) return rc;
    rc = ensure(c->counter, 256);
    if (rc) return rc;
    HIPCALL(hipMemsetAsync(c->counter.p, 0, 8, c->stream));  // word 0 = work counter; words 1.. belong to callers
    sdk::SolveArgs a;
    a.in = d_in;
    a.mask = d_mask;
    a.out = d_out;
    a.status = d_status;
    a.work = d_work;
    a.n = n;
    a.next = static_cast<uint32_t*>(c->counter.p);
    a.stack = static_cast<uint32_t*>(c->stack.p);
    a.budget = c->budget;
    a.order = c->order;
    a.limit = limit;
    a.count = d_count;
    a.counts = d_counts;
    a.count_mode = count_mode;
    a.chunk = chunk;
    hipEvent_t stop;
    rc = timer_begin(c, &stop);
    if (rc) return rc;
    sdk::solve_kernel<<<grid, 64, 0, c->stream>>>(a);
    HIPCALL(hipGetLastError());
    HIPCALL(hipEventRecord(stop, c->stream));
    return SDK_OK;
}

// Whole-tree solution count with a replicated, deterministic BFS frontier.
// Every rank expands the same frontier (no exchange), counts the subtrees of its
// contiguous slice with the batched count kernel; rank 0 also owns the leaves
// solved during expansion.  The caller sums the per-rank counts.
int count_frontier(sdk_ctx* c, const uint8_t* h_board, uint64_t limit, int rank, int world, uint64_t* local_count,
                   uint64_t* frontier_size, int8_t* status) {
    if (world < 1 || rank < 0 || rank >= world) return fail(SDK_EINVAL, "bad rank %d / world %d", rank, world);
    int rc;
    // counters: [0] next (u32), [1] leaves (u64), [2] scan total (u64), [3] count total (u64)
    if ((rc = ensure(c->counter, 256)) || (rc = ensure(c->fr_a, 81))) return rc;
    unsigned long long* ctr = static_cast<unsigned long long*>(c->counter.p);
    unsigned long long* d_leaves = ctr + 1;
    unsigned long long* d_total = ctr + 2;
    unsigned long long* d_count = ctr + 3;
    HIPCALL(hipMemsetAsync(c->counter.p, 0, 256, c->stream));
    HIPCALL(hipMemcpyAsync(c->fr_a.p, h_board, 81, hipMemcpyHostToDevice, c->stream));
    const uint64_t target = (uint64_t)c->cus * (uint64_t)c->waves_per_cu * 8ull * (uint64_t)world;
    const uint64_t cap = 1ull << 25;  // 32M boards (2.6 GB) per frontier buffer
    uint64_t m = 1;
    int level = 0;
    while (m > 0 && m < target && level < 81) {
        if ((rc = ensure(c->prop, m * 81)) || (rc = ensure(c->bcell, m)) || (rc = ensure(c->bmask, m * 2)) ||
            (rc = ensure(c->nchild, m * 4)) || (rc = ensure(c->offs, m * 8)))
            return rc;
        HIPCALL(hipMemsetAsync(c->counter.p, 0, 4, c->stream));
        sdk::ExpandArgs ea;
        ea.in = static_cast<const uint8_t*>(c->fr_a.p);
        ea.m = m;
        ea.prop = static_cast<uint8_t*>(c->prop.p);
        ea.bcell = static_cast<uint8_t*>(c->bcell.p);
        ea.bmask = static_cast<uint16_t*>(c->bmask.p);
        ea.nchild = static_cast<uint32_t*>(c->nchild.p);
        ea.leaves = d_leaves;
        ea.next = static_cast<uint32_t*>(c->counter.p);
        ea.order = sdk::ORDER_MRV;
        const unsigned eg = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((m + sdk::kChunk - 1) / sdk::kChunk,
                                                                               (uint64_t)c->cus * c->waves_per_cu));
        hipEvent_t stop;
        if ((rc = timer_begin(c, &stop))) return rc;
        sdk::expand_kernel<<<eg, 64, 0, c->stream>>>(ea);
        HIPCALL(hipGetLastError());
        sdk::scan_kernel<<<1, 1024, 0, c->stream>>>(static_cast<uint32_t*>(c->nchild.p),
                                                    static_cast<uint64_t*>(c->offs.p), m, d_total);
        HIPCALL(hipGetLastError());
        unsigned long long total = 0;
        HIPCALL(hipMemcpyAsync(&total, d_total, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCALL(hipStreamSynchronize(c->stream));
        if (total > cap) {
            HIPCALL(hipEventRecord(stop, c->stream));
            break;  // keep the current frontier: it is already big enough to split
        }
        if (total && (rc = ensure(c->fr_b, total * 81))) return rc;
        if (total) {
            const unsigned gg = (unsigned)std::min<uint64_t>(m, (uint64_t)c->cus * 32);
            sdk::emit_kernel<<<gg, 64, 0, c->stream>>>(static_cast<uint8_t*>(c->prop.p), static_cast<uint8_t*>(c->bcell.p),
                                                       static_cast<uint16_t*>(c->bmask.p),
                                                       static_cast<uint64_t*>(c->offs.p), m,
                                                       static_cast<uint8_t*>(c->fr_b.p));
            HIPCALL(hipGetLastError());
        }
        HIPCALL(hipEventRecord(stop, c->stream));
        std::swap(c->fr_a, c->fr_b);
        m = total;
        ++level;
    }
    // count this rank's slice of the final frontier
    const uint64_t lo = (rank * m) / world, hi = ((rank + 1) * m) / world;
    int8_t st = 1;
    uint64_t cnt = 0;
    if (hi > lo) {
        if ((rc = ensure(c->fr_status, hi - lo))) return rc;
        rc = launch_solve(c, static_cast<uint8_t*>(c->fr_a.p) + lo * 81, nullptr, nullptr,
                          static_cast<int8_t*>(c->fr_status.p), nullptr, hi - lo, 1, limit, d_count, nullptr);
        if (rc) return rc;
        std::vector<int8_t> sts(hi - lo);
        HIPCALL(hipMemcpyAsync(sts.data(), c->fr_status.p, hi - lo, hipMemcpyDeviceToHost, c->stream));
        unsigned long long tot = 0;
        HIPCALL(hipMemcpyAsync(&tot, d_count, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCALL(hipStreamSynchronize(c->stream));
        cnt = tot;
        for (int8_t x : sts)
            if (x == -2) st = -2;
    }
    unsigned long long leaves = 0;
    HIPCALL(hipMemcpyAsync(&leaves, d_leaves, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    if (rank == 0) cnt += leaves;
    if (limit && cnt > limit) cnt = limit;
    if (st != -2) st = cnt > 0 ? 1 : 0;
    *local_count = cnt;
    if (frontier_size) *frontier_size = m;
    *status = st;
    return SDK_OK;
}

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
    *out = c;
    return SDK_OK;
}

int sdk_destroy(sdk_ctx* c) {
    if (!c) return SDK_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (DevBuf* b : {&c->stack, &c->counter, &c->in, &c->mask, &c->out, &c->status, &c->work, &c->verdict,
                      &c->fr_a, &c->fr_b, &c->prop, &c->bcell, &c->bmask, &c->nchild, &c->offs, &c->fr_status})
        if (b->p) (void)hipFree(b->p);
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
        default:
            return fail(SDK_EINVAL, "unknown option %d", key);
    }
}

int sdk_get_option(sdk_ctx* c, int key, int64_t* value) {
    if (!c || !value) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    switch (key) {
        case SDK_OPT_ORDER: *value = c->order; return SDK_OK;
        case SDK_OPT_NODE_BUDGET: *value = (int64_t)c->budget; return SDK_OK;
        case SDK_OPT_WAVES_PER_CU: *value = c->waves_per_cu; return SDK_OK;
        case SDK_OPT_CHECK_BLOCKS_PER_CU: *value = c->check_blocks_per_cu; return SDK_OK;
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
    return SDK_OK;
}

int sdk_synchronize(sdk_ctx* c) {
    if (!c) return fail(SDK_EINVAL, "ctx is NULL");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    HIPCALL(hipStreamSynchronize(c->stream));
    return SDK_OK;
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

int sdk_solve_batch(sdk_ctx* c, const uint8_t* in, const uint16_t* first_cell_mask, uint8_t* out, int8_t* status,
                    uint64_t* work, size_t n) {
    if (!c || (n && (!in || !out || !status))) return fail(SDK_EINVAL, "NULL argument");
    if (n == 0) return SDK_OK;
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c->in, n * 81)) || (rc = ensure(c->out, n * 81)) || (rc = ensure(c->status, n))) return rc;
    if (first_cell_mask && (rc = ensure(c->mask, n * 2))) return rc;
    if (work && (rc = ensure(c->work, n * 8))) return rc;
    HIPCALL(hipMemcpyAsync(c->in.p, in, n * 81, hipMemcpyHostToDevice, c->stream));
    if (first_cell_mask) HIPCALL(hipMemcpyAsync(c->mask.p, first_cell_mask, n * 2, hipMemcpyHostToDevice, c->stream));
    rc = launch_solve(c, static_cast<uint8_t*>(c->in.p), first_cell_mask ? static_cast<uint16_t*>(c->mask.p) : nullptr,
                      static_cast<uint8_t*>(c->out.p), static_cast<int8_t*>(c->status.p),
                      work ? static_cast<uint64_t*>(c->work.p) : nullptr, n, 0, 0, nullptr);
    if (rc) return rc;
    HIPCALL(hipMemcpyAsync(out, c->out.p, n * 81, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipMemcpyAsync(status, c->status.p, n, hipMemcpyDeviceToHost, c->stream));
    if (work) HIPCALL(hipMemcpyAsync(work, c->work.p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    return SDK_OK;
}

int sdk_count_solutions(sdk_ctx* c, const uint8_t* board, uint64_t limit, uint64_t* count, int8_t* status) {
    if (!c || !board || !count || !status) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return count_frontier(c, board, limit, 0, 1, count, nullptr, status);
}

int sdk_count_solutions_slice(sdk_ctx* c, const uint8_t* board, uint64_t limit, int rank, int world,
                              uint64_t* count, uint64_t* frontier_size, int8_t* status) {
    if (!c || !board || !count || !status) return fail(SDK_EINVAL, "NULL argument");
    std::lock_guard<std::mutex> lk(c->mu);
    HIPCALL(hipSetDevice(c->device));
    return count_frontier(c, board, limit, rank, world, count, frontier_size, status);
}

}  // extern "C"
