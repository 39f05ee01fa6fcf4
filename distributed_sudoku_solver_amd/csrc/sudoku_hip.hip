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
    int waves_per_cu = 16;
    // workspaces
    DevBuf stack, counter, in, mask, out, status, work, verdict;
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
    const unsigned grid = (unsigned)std::min<uint64_t>(tiles, (uint64_t)c->cus * 8);
    hipEvent_t stop;
    int rc = timer_begin(c, &stop);
    if (rc) return rc;
    sdk::check_kernel<<<grid, sdk::kCheckThreads, 0, c->stream>>>(d_in, d_out, (uint64_t)n);
    HIPCALL(hipGetLastError());
    HIPCALL(hipEventRecord(stop, c->stream));
    return SDK_OK;
}

int launch_solve(sdk_ctx* c, const uint8_t* d_in, const uint16_t* d_mask, uint8_t* d_out, int8_t* d_status,
                 uint64_t* d_work, size_t n, int count_mode, uint64_t limit, unsigned long long* d_count) {
    if (n == 0) return SDK_OK;
    if (n > 0x7FFFFFFFull) return fail(SDK_EINVAL, "at most 2^31-1 boards per call");
    const uint64_t want = (n + sdk::kChunk - 1) / sdk::kChunk;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)c->cus * c->waves_per_cu));
    int rc = ensure(c->stack, (size_t)grid * sdk::kStackWordsPerBlock * sizeof(uint32_t));
    if (rc) return rc;
    rc = ensure(c->counter, 256);
    if (rc) return rc;
    HIPCALL(hipMemsetAsync(c->counter.p, 0, 256, c->stream));
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
    a.count_mode = count_mode;
    hipEvent_t stop;
    rc = timer_begin(c, &stop);
    if (rc) return rc;
    sdk::solve_kernel<<<grid, 64, 0, c->stream>>>(a);
    HIPCALL(hipGetLastError());
    HIPCALL(hipEventRecord(stop, c->stream));
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
    for (DevBuf* b : {&c->stack, &c->counter, &c->in, &c->mask, &c->out, &c->status, &c->work, &c->verdict})
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
    int rc;
    if ((rc = ensure(c->in, 81)) || (rc = ensure(c->out, 81)) || (rc = ensure(c->status, 8)) ||
        (rc = ensure(c->work, 16)))
        return rc;
    HIPCALL(hipMemcpyAsync(c->in.p, board, 81, hipMemcpyHostToDevice, c->stream));
    unsigned long long* d_count = static_cast<unsigned long long*>(c->work.p) + 1;
    rc = launch_solve(c, static_cast<uint8_t*>(c->in.p), nullptr, static_cast<uint8_t*>(c->out.p),
                      static_cast<int8_t*>(c->status.p), static_cast<uint64_t*>(c->work.p), 1, 1, limit, d_count);
    if (rc) return rc;
    unsigned long long cnt = 0;
    int8_t st = 0;
    HIPCALL(hipMemcpyAsync(&cnt, d_count, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipMemcpyAsync(&st, c->status.p, 1, hipMemcpyDeviceToHost, c->stream));
    HIPCALL(hipStreamSynchronize(c->stream));
    *count = cnt;
    *status = st;
    return SDK_OK;
}

}  // extern "C"
