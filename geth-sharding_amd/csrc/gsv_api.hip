// C ABI of libgsv.so (include/gsv.h): context, device memory staging, launches, timing.
// Host-pointer entry points stage through a grow-only device arena on the context's stream;
// *_dev entry points take HBM-resident buffers and the caller's stream and never allocate or
// synchronize (graph-capturable).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "chunk_root.h"
#include "gsv_internal.h"
#include "tx_host.h"

struct gsv_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint4* gtab = nullptr;
    // grow-only staging arena for the host-pointer entry points
    uint8_t* arena = nullptr;
    size_t arena_cap = 0;
    std::mutex mu;
    // kernel timing
    int timing = 0;
    struct Pending { int kid; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> free_events;
    double total_ms[GSV_K_COUNT] = {0};
    long launches[GSV_K_COUNT] = {0};
    std::mutex tmu;
    // chunk-root trie plans (per body length) and the device workspace of the *_dev paths
    gsv::PlanCache plans;
    uint8_t* work = nullptr;
    size_t work_cap = 0;
    std::vector<hipEvent_t> open_ev;  // timer events opened by launch hooks
    hipStream_t cur_stream = nullptr;
    std::mutex wmu;                   // serializes users of `work`
    uint8_t* nwork = nullptr;         // notary workspace (blob tables, chain-id buffers)
    size_t nwork_cap = 0;
    uint8_t* pwork = nullptr;         // Proof-of-Custody salted bodies (outlive `work` regrowth)
    size_t pwork_cap = 0;
    // ordering of `work` users on different streams: the last user's stream + an event after its work
    hipStream_t work_st = nullptr;
    hipEvent_t work_ev = nullptr;
    // chunk-root body offsets cached on the device (re-uploaded only when they change)
    uint64_t* coff = nullptr;
    size_t coff_cap = 0;
    std::vector<uint64_t> coff_key;
};

namespace {

int hip_err(hipError_t e) { return e == hipSuccess ? GSV_SUCCESS : GSV_E_HIP; }

#define HIPCHK(x)                                  \
    do {                                           \
        hipError_t _e = (x);                       \
        if (_e != hipSuccess) return GSV_E_HIP;    \
    } while (0)

hipEvent_t take_event(gsv_ctx* c) {
    if (!c->free_events.empty()) {
        hipEvent_t e = c->free_events.back();
        c->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    hipEventCreate(&e);
    return e;
}

// Brackets one launch with events on the launching stream when timing is on.
struct KTimer {
    gsv_ctx* c;
    int kid;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    KTimer(gsv_ctx* c_, int kid_, hipStream_t st_) : c(c_), kid(kid_), st(st_) {
        if (c->timing) {
            std::lock_guard<std::mutex> g(c->tmu);
            a = take_event(c);
            b = take_event(c);
            hipEventRecord(a, st);
        }
    }
    ~KTimer() {
        if (a) {
            hipEventRecord(b, st);
            std::lock_guard<std::mutex> g(c->tmu);
            c->pending.push_back({kid, a, b});
        }
    }
};

void drain_timing(gsv_ctx* c) {
    std::lock_guard<std::mutex> g(c->tmu);
    for (auto& p : c->pending) {
        hipEventSynchronize(p.b);
        float ms = 0;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->total_ms[p.kid] += ms;
            c->launches[p.kid] += 1;
        }
        c->free_events.push_back(p.a);
        c->free_events.push_back(p.b);
    }
    c->pending.clear();
}

// timer hooks for multi-launch paths (chunk root levels)
void hook_begin(void* p, int kid) {
    gsv_ctx* c = (gsv_ctx*)p;
    if (!c->timing) return;
    std::lock_guard<std::mutex> g(c->tmu);
    hipEvent_t a = take_event(c);
    hipEventRecord(a, c->cur_stream);
    c->open_ev.push_back(a);
}
void hook_end(void* p, int kid) {
    gsv_ctx* c = (gsv_ctx*)p;
    if (!c->timing) return;
    std::lock_guard<std::mutex> g(c->tmu);
    hipEvent_t a = c->open_ev.back();
    c->open_ev.pop_back();
    hipEvent_t b = take_event(c);
    hipEventRecord(b, c->cur_stream);
    c->pending.push_back({kid, a, b});
}

int work_reserve(gsv_ctx* c, size_t bytes) {
    if (bytes <= c->work_cap) return GSV_SUCCESS;
    size_t cap = c->work_cap ? c->work_cap : (size_t)64 << 20;
    while (cap < bytes) cap *= 2;
    if (c->work) {
        hipDeviceSynchronize();
        hipFree(c->work);
        c->work = nullptr;
        c->work_cap = 0;
    }
    if (hipMalloc(&c->work, cap) != hipSuccess) return GSV_E_NOMEM;
    c->work_cap = cap;
    return GSV_SUCCESS;
}

// `work` is shared by the *_dev paths of one context: a call on a stream other than the previous
// user's waits (on the GPU) for that user's last enqueued work before touching it.
void work_begin(gsv_ctx* c, hipStream_t st) {
    if (c->work_st && c->work_st != st && c->work_ev) hipStreamWaitEvent(st, c->work_ev, 0);
}
void work_end(gsv_ctx* c, hipStream_t st) {
    if (!c->work_ev) hipEventCreateWithFlags(&c->work_ev, hipEventDisableTiming);
    if (c->work_ev) hipEventRecord(c->work_ev, st);
    c->work_st = st;
}

int arena_reserve(gsv_ctx* c, size_t bytes) {
    if (bytes <= c->arena_cap) return GSV_SUCCESS;
    size_t cap = c->arena_cap ? c->arena_cap : (size_t)64 << 20;
    while (cap < bytes) cap *= 2;
    if (c->arena) {
        hipStreamSynchronize(c->stream);
        hipFree(c->arena);
        c->arena = nullptr;
        c->arena_cap = 0;
    }
    if (hipMalloc(&c->arena, cap) != hipSuccess) return GSV_E_NOMEM;
    c->arena_cap = cap;
    return GSV_SUCCESS;
}

// bump allocator over the arena (256-B aligned slices)
struct Carve {
    uint8_t* base;
    size_t off = 0;
    explicit Carve(uint8_t* b) : base(b) {}
    template <typename T>
    T* take(size_t bytes) {
        T* p = (T*)(base + off);
        off += (bytes + 255) & ~(size_t)255;
        return p;
    }
};
size_t al(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

int gsv_abi_version(void) { return GSV_ABI_VERSION; }

int gsv_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* gsv_error_string(int err) {
    switch (err) {
        case GSV_SUCCESS: return "success";
        case GSV_E_INVALID_ARG: return "invalid argument";
        case GSV_E_HIP: return "HIP runtime error";
        case GSV_E_NOMEM: return "out of device memory";
        case GSV_E_NO_DEVICE: return "no HIP device";
        case GSV_E_TOO_LARGE: return "input exceeds the reference size limit";
        case GSV_E_RCCL: return "RCCL error";
        default: return "unknown error";
    }
}

int gsv_ctx_create(int device, gsv_ctx** out) {
    if (!out) return GSV_E_INVALID_ARG;
    *out = nullptr;
    int n = gsv_device_count();
    if (n <= 0) return GSV_E_NO_DEVICE;
    if (device < 0 || device >= n) return GSV_E_INVALID_ARG;
    HIPCHK(hipSetDevice(device));
    gsv_ctx* c = new gsv_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return GSV_E_HIP;
    }
    if (hipMalloc(&c->gtab, gsv::GTAB_BYTES) != hipSuccess) {
        hipStreamDestroy(c->stream);
        delete c;
        return GSV_E_NOMEM;
    }
    hipError_t e = gsv::launch_gtable_init(c->gtab, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        hipFree(c->gtab);
        hipStreamDestroy(c->stream);
        delete c;
        return GSV_E_HIP;
    }
    *out = c;
    return GSV_SUCCESS;
}

void gsv_ctx_destroy(gsv_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    drain_timing(c);
    for (auto e : c->free_events) hipEventDestroy(e);
    if (c->arena) hipFree(c->arena);
    if (c->work) hipFree(c->work);
    if (c->nwork) hipFree(c->nwork);
    if (c->pwork) hipFree(c->pwork);
    if (c->coff) hipFree(c->coff);
    if (c->work_ev) hipEventDestroy(c->work_ev);
    if (c->gtab) hipFree(c->gtab);
    hipStreamDestroy(c->stream);
    delete c;
}

int gsv_ctx_set_timing(gsv_ctx* c, int enable) {
    if (!c) return GSV_E_INVALID_ARG;
    c->timing = enable ? 1 : 0;
    return GSV_SUCCESS;
}

int gsv_ctx_kernel_time(gsv_ctx* c, int kid, double* total_ms, long* launches) {
    if (!c || kid < 0 || kid >= GSV_K_COUNT) return GSV_E_INVALID_ARG;
    drain_timing(c);
    if (total_ms) *total_ms = c->total_ms[kid];
    if (launches) *launches = c->launches[kid];
    return GSV_SUCCESS;
}

int gsv_ctx_reset_timing(gsv_ctx* c) {
    if (!c) return GSV_E_INVALID_ARG;
    drain_timing(c);
    for (int i = 0; i < GSV_K_COUNT; i++) {
        c->total_ms[i] = 0;
        c->launches[i] = 0;
    }
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ Keccak-256
int gsv_keccak256_batch_dev(gsv_ctx* c, const uint8_t* d_data, const uint64_t* d_off, size_t n,
                            uint8_t* d_out32, void* stream) {
    if (!c || (n && (!d_off || !d_out32)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    KTimer t(c, GSV_K_KECCAK, st);
    return hip_err(gsv::launch_keccak256(d_data, d_off, (uint32_t)n, d_out32, st));
}

int gsv_keccak256_batch(gsv_ctx* c, const uint8_t* data, const uint64_t* off, size_t n,
                        uint8_t* out32) {
    if (!c || (n && (!off || !out32)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    size_t bytes = off[n] - off[0];
    size_t need = al(bytes + 8) + al((n + 1) * 8) + al(n * 32);
    int rc = arena_reserve(c, need);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_data = cv.take<uint8_t>(bytes + 8);
    uint64_t* d_off = cv.take<uint64_t>((n + 1) * 8);
    uint8_t* d_out = cv.take<uint8_t>(n * 32);
    std::vector<uint64_t> rel(n + 1);
    for (size_t i = 0; i <= n; i++) rel[i] = off[i] - off[0];
    if (bytes) HIPCHK(hipMemcpyAsync(d_data, data + off[0], bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_off, rel.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    rc = gsv_keccak256_batch_dev(c, d_data, d_off, n, d_out, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out32, d_out, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ ecrecover
int gsv_ecrecover_batch_dev(gsv_ctx* c, const uint8_t* d_msg32, const uint8_t* d_sig65, size_t n,
                            uint8_t* d_pub65, uint8_t* d_addr20, uint8_t* d_status, void* stream) {
    if (!c || (n && (!d_msg32 || !d_sig65 || !d_status)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    KTimer t(c, GSV_K_ECRECOVER, st);
    return hip_err(gsv::launch_ecrecover(d_msg32, d_sig65, (uint32_t)n, c->gtab, d_pub65, d_addr20,
                                         d_status, st));
}

int gsv_ecrecover_batch(gsv_ctx* c, const uint8_t* msg32, const uint8_t* sig65, size_t n,
                        uint8_t* pub65_out, uint8_t* addr20_out, uint8_t* status) {
    if (!c || (n && (!msg32 || !sig65 || !status)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    size_t need = al(n * 32) + al(n * 65) + al(n * 65) + al(n * 20) + al(n);
    int rc = arena_reserve(c, need);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_msg = cv.take<uint8_t>(n * 32);
    uint8_t* d_sig = cv.take<uint8_t>(n * 65);
    uint8_t* d_pub = cv.take<uint8_t>(n * 65);
    uint8_t* d_addr = cv.take<uint8_t>(n * 20);
    uint8_t* d_st = cv.take<uint8_t>(n);
    HIPCHK(hipMemcpyAsync(d_msg, msg32, n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_sig, sig65, n * 65, hipMemcpyHostToDevice, c->stream));
    rc = gsv_ecrecover_batch_dev(c, d_msg, d_sig, n, pub65_out ? d_pub : nullptr,
                                 addr20_out ? d_addr : nullptr, d_st, c->stream);
    if (rc) return rc;
    if (pub65_out) HIPCHK(hipMemcpyAsync(pub65_out, d_pub, n * 65, hipMemcpyDeviceToHost, c->stream));
    if (addr20_out) HIPCHK(hipMemcpyAsync(addr20_out, d_addr, n * 20, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ recoverPlain
int gsv_sender_batch(gsv_ctx* c, const uint8_t* sighash32, const uint8_t* r32, const uint8_t* s32,
                     const uint64_t* v, const uint8_t* v_big, size_t n, int homestead,
                     uint8_t* addr20_out, uint8_t* status) {
    if (!c || (n && (!sighash32 || !r32 || !s32 || !v || !v_big || !addr20_out || !status)) ||
        n > 0xFFFFFFFFull)
        return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    size_t need = 3 * al(n * 32) + al(n * 8) + al(n) + al(n * 20) + al(n);
    int rc = arena_reserve(c, need);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_h = cv.take<uint8_t>(n * 32);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    uint8_t* d_s = cv.take<uint8_t>(n * 32);
    uint64_t* d_v = cv.take<uint64_t>(n * 8);
    uint8_t* d_vb = cv.take<uint8_t>(n);
    uint8_t* d_a = cv.take<uint8_t>(n * 20);
    uint8_t* d_st = cv.take<uint8_t>(n);
    HIPCHK(hipMemcpyAsync(d_h, sighash32, n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_r, r32, n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_s, s32, n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_v, v, n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_vb, v_big, n, hipMemcpyHostToDevice, c->stream));
    {
        KTimer t(c, GSV_K_ECRECOVER, c->stream);
        HIPCHK(gsv::launch_sender(d_h, d_r, d_s, d_v, d_vb, (uint32_t)n, homestead, c->gtab, d_a, d_st,
                                  c->stream));
    }
    HIPCHK(hipMemcpyAsync(addr20_out, d_a, n * 20, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ synthetic signer (bench data)
int gsv_synth_sign_dev(gsv_ctx* c, uint64_t seed, size_t n, uint8_t* d_msg32, uint8_t* d_sig65,
                       uint8_t* d_pub65, uint8_t* d_addr20, void* stream) {
    if (!c || (n && (!d_msg32 || !d_sig65)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return hip_err(gsv::launch_synth_sign(seed, (uint32_t)n, c->gtab, d_msg32, d_sig65, d_pub65,
                                          d_addr20, st));
}

int gsv_synth_sign(gsv_ctx* c, uint64_t seed, size_t n, uint8_t* msg32, uint8_t* sig65,
                   uint8_t* pub65, uint8_t* addr20) {
    if (!c || (n && (!msg32 || !sig65)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    size_t need = al(n * 32) + 2 * al(n * 65) + al(n * 20);
    int rc = arena_reserve(c, need);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_m = cv.take<uint8_t>(n * 32);
    uint8_t* d_s = cv.take<uint8_t>(n * 65);
    uint8_t* d_p = cv.take<uint8_t>(n * 65);
    uint8_t* d_a = cv.take<uint8_t>(n * 20);
    rc = gsv_synth_sign_dev(c, seed, n, d_m, d_s, pub65 ? d_p : nullptr, addr20 ? d_a : nullptr,
                            c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(msg32, d_m, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(sig65, d_s, n * 65, hipMemcpyDeviceToHost, c->stream));
    if (pub65) HIPCHK(hipMemcpyAsync(pub65, d_p, n * 65, hipMemcpyDeviceToHost, c->stream));
    if (addr20) HIPCHK(hipMemcpyAsync(addr20, d_a, n * 20, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ chunk root
static const uint8_t EMPTY_ROOT[32] = {0x56, 0xe8, 0x1f, 0x17, 0x1b, 0xcc, 0x55, 0xa6, 0xff, 0x83, 0x45,
                                       0xe6, 0x92, 0xc0, 0xf8, 0x6e, 0x5b, 0x48, 0xe0, 0x1b, 0x99, 0x6c,
                                       0xad, 0xc0, 0x01, 0x62, 0x2f, 0xb5, 0xe3, 0x63, 0xb4, 0x21};
static const uint64_t MAX_BODY = 1ull << 20;  // collationSizelimit (sharding/collation.go:45)

// Body i = d_bodies[start[i] .. end[i]); roots to d_roots (device) via workspace `work`.
static int chunk_root_dev_impl(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* start,
                               const uint64_t* end, size_t n, uint8_t* d_roots, hipStream_t st,
                               uint64_t max_len = MAX_BODY) {
    // group bodies by length (the trie shape depends only on N)
    std::map<uint64_t, std::vector<uint32_t>> groups;
    for (size_t i = 0; i < n; i++) {
        if (end[i] < start[i] || end[i] - start[i] > max_len) return GSV_E_TOO_LARGE;
        groups[end[i] - start[i]].push_back((uint32_t)i);
    }
    size_t need = 0;
    std::vector<uint64_t> key;  // all groups' body offsets, in group order
    key.reserve(n);
    for (auto& g : groups) {
        if (g.first == 0) continue;
        gsv::TriePlan* pl = c->plans.get((uint32_t)g.first);
        if (!pl) return GSV_E_NOMEM;
        need += al(g.second.size() * 32) + al(gsv::chunk_root_scratch_bytes(pl, (uint32_t)g.second.size()));
        for (uint32_t i : g.second) key.push_back(start[i]);
    }
    work_begin(c, st);
    int rc = work_reserve(c, need + 4096);
    if (rc) return rc;
    // device copy of the offsets: uploaded only when they differ from the previous call's
    if (key != c->coff_key) {
        if (key.size() * 8 > c->coff_cap) {
            if (c->coff) {
                hipDeviceSynchronize();
                hipFree(c->coff);
                c->coff = nullptr;
                c->coff_cap = 0;
            }
            size_t cap = (key.size() * 8 + 4095) & ~(size_t)4095;
            if (hipMalloc(&c->coff, cap) != hipSuccess) return GSV_E_NOMEM;
            c->coff_cap = cap;
        }
        if (!key.empty())  // pageable source: staged before return, so `key` may go out of scope
            HIPCHK(hipMemcpyAsync(c->coff, key.data(), key.size() * 8, hipMemcpyHostToDevice, st));
        c->coff_key = std::move(key);
    }
    Carve cv(c->work);
    c->cur_stream = st;
    size_t koff = 0;
    for (auto& g : groups) {
        const auto& idx = g.second;
        if (g.first == 0) {  // empty trie -> emptyRoot (trie/trie.go:472-474)
            for (uint32_t i : idx)
                HIPCHK(hipMemcpyAsync(d_roots + (size_t)i * 32, EMPTY_ROOT, 32, hipMemcpyHostToDevice, st));
            continue;
        }
        gsv::TriePlan* pl = c->plans.get((uint32_t)g.first);
        bool direct = idx.size() == n;  // one group holding bodies 0..n-1 in order: roots in place
        uint8_t* d_gr = direct ? d_roots : cv.take<uint8_t>(idx.size() * 32);
        uint8_t* d_scr = cv.take<uint8_t>(gsv::chunk_root_scratch_bytes(pl, (uint32_t)idx.size()));
        HIPCHK(gsv::launch_chunk_root_plan(pl, d_bodies, c->coff + koff, (uint32_t)idx.size(), d_scr, d_gr, st,
                                           hook_begin, hook_end, c));
        koff += idx.size();
        if (direct) continue;
        // scatter group roots to their positions (contiguous runs copied together)
        size_t k = 0;
        while (k < idx.size()) {
            size_t e2 = k + 1;
            while (e2 < idx.size() && idx[e2] == idx[e2 - 1] + 1) e2++;
            HIPCHK(hipMemcpyAsync(d_roots + (size_t)idx[k] * 32, d_gr + k * 32, (e2 - k) * 32,
                                  hipMemcpyDeviceToDevice, st));
            k = e2;
        }
    }
    work_end(c, st);
    return GSV_SUCCESS;
}

int gsv_chunk_root_batch_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n,
                             uint8_t* d_root32_out, void* stream) {
    if (!c || (n && (!h_off || !d_root32_out || !d_bodies))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->wmu);
    HIPCHK(hipSetDevice(c->device));
    return chunk_root_dev_impl(c, d_bodies, h_off, h_off + 1, n, d_root32_out,
                               stream ? (hipStream_t)stream : c->stream);
}

int gsv_chunk_root_batch(gsv_ctx* c, const uint8_t* bodies, const uint64_t* off, size_t n, uint8_t* root32_out) {
    if (!c || (n && (!off || !root32_out))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > MAX_BODY) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    // stage bodies in HBM with 16-byte aligned starts (vector loads in the bottom-level kernel)
    std::vector<uint64_t> st(n), en(n);
    uint64_t pos = 0;
    for (size_t i = 0; i < n; i++) {
        st[i] = pos;
        en[i] = pos + (off[i + 1] - off[i]);
        pos = (en[i] + 15) & ~15ull;
    }
    int rc = arena_reserve(c, al(pos + 16) + al(n * 32));
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_b = cv.take<uint8_t>(pos + 16);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    for (size_t i = 0; i < n; i++)
        if (en[i] > st[i])
            HIPCHK(hipMemcpyAsync(d_b + st[i], bodies + off[i], en[i] - st[i], hipMemcpyHostToDevice, c->stream));
    {
        std::lock_guard<std::mutex> g2(c->wmu);
        rc = chunk_root_dev_impl(c, d_b, st.data(), en.data(), n, d_r, c->stream);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(root32_out, d_r, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ types.Sender over tx RLP
// Host: decode + sighash preimages (threads). GPU: Keccak of the preimages, recoverPlain + address.
static int tx_sender_impl(gsv_ctx* c, const uint8_t* rlp, const uint64_t* off, size_t n, const uint8_t* cid,
                          size_t cidlen, int signer_kind, uint8_t* addr_out, uint8_t* status_out) {
    std::vector<uint8_t> hst(n), rr(n * 32), ss(n * 32), vb(n);
    std::vector<uint64_t> vv(n), plen(n);
    std::vector<std::vector<uint8_t>> pres;
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 4096) nt = 1;
    std::vector<std::vector<uint8_t>> tpre(nt);
    std::vector<std::thread> th;
    auto work = [&](unsigned t) {
        size_t lo = n * t / nt, hi = n * (t + 1) / nt;
        gsv::TxPrep p;
        for (size_t i = lo; i < hi; i++) {
            int st = gsv::tx_prepare(rlp + off[i], off[i + 1] - off[i], cid, cidlen, signer_kind, p);
            hst[i] = (uint8_t)st;
            if (st != GSV_ST_OK) {
                plen[i] = 0;
                vb[i] = 1;
                continue;
            }
            memcpy(&rr[i * 32], p.r32, 32);
            memcpy(&ss[i * 32], p.s32, 32);
            vv[i] = p.v;
            vb[i] = p.vbig;
            plen[i] = p.pre.size();
            tpre[t].insert(tpre[t].end(), p.pre.begin(), p.pre.end());
        }
    };
    for (unsigned t = 0; t < nt; t++) th.emplace_back(work, t);
    for (auto& x : th) x.join();
    std::vector<uint64_t> poff(n + 1);
    poff[0] = 0;
    for (size_t i = 0; i < n; i++) poff[i + 1] = poff[i] + plen[i];
    size_t pbytes = poff[n];
    int homestead = signer_kind == GSV_SIGNER_FRONTIER ? 0 : 1;
    size_t need = al(pbytes + 8) + al((n + 1) * 8) + 3 * al(n * 32) + al(n * 8) + al(n) + al(n * 20) + al(n);
    int rc = arena_reserve(c, need);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_pre = cv.take<uint8_t>(pbytes + 8);
    uint64_t* d_poff = cv.take<uint64_t>((n + 1) * 8);
    uint8_t* d_h = cv.take<uint8_t>(n * 32);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    uint8_t* d_s = cv.take<uint8_t>(n * 32);
    uint64_t* d_v = cv.take<uint64_t>(n * 8);
    uint8_t* d_vb = cv.take<uint8_t>(n);
    uint8_t* d_a = cv.take<uint8_t>(n * 20);
    uint8_t* d_st = cv.take<uint8_t>(n);
    size_t w = 0;
    for (unsigned t = 0; t < nt; t++) {
        if (!tpre[t].empty())
            HIPCHK(hipMemcpyAsync(d_pre + w, tpre[t].data(), tpre[t].size(), hipMemcpyHostToDevice, c->stream));
        w += tpre[t].size();
    }
    HIPCHK(hipMemcpyAsync(d_poff, poff.data(), (n + 1) * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_r, rr.data(), n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_s, ss.data(), n * 32, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_v, vv.data(), n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_vb, vb.data(), n, hipMemcpyHostToDevice, c->stream));
    {
        KTimer t(c, GSV_K_SENDER_PREP, c->stream);
        HIPCHK(gsv::launch_keccak256(d_pre, d_poff, (uint32_t)n, d_h, c->stream));
    }
    {
        KTimer t(c, GSV_K_ECRECOVER, c->stream);
        HIPCHK(gsv::launch_sender(d_h, d_r, d_s, d_v, d_vb, (uint32_t)n, homestead, c->gtab, d_a, d_st, c->stream));
    }
    HIPCHK(hipMemcpyAsync(addr_out, d_a, n * 20, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(status_out, d_st, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < n; i++)
        if (hst[i] != GSV_ST_OK) {
            status_out[i] = hst[i];
            memset(addr_out + i * 20, 0, 20);
        }
    return GSV_SUCCESS;
}

int gsv_tx_sender_batch(gsv_ctx* c, const uint8_t* rlp, const uint64_t* off, size_t n, const uint8_t* chain_id,
                        size_t chain_id_len, int signer_kind, uint8_t* addr20_out, uint8_t* status) {
    if (!c || (n && (!rlp || !off || !addr20_out || !status)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    if (signer_kind < GSV_SIGNER_EIP155 || signer_kind > GSV_SIGNER_FRONTIER) return GSV_E_INVALID_ARG;
    if (chain_id_len && !chain_id) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    return tx_sender_impl(c, rlp, off, n, chain_id, chain_id_len, signer_kind, addr20_out, status);
}

// ------------------------------------------------------------------ BN254 pairing check
// Host tables for a batch: check c = in[off[c] .. off[c+1]); a length that is not a multiple of
// 192 is errBadPairingInput (core/vm/contracts.go:336-338) and contributes no pairs.
struct BnTables {
    std::vector<uint64_t> pair_src;     // slot-major pair order
    std::vector<uint32_t> check_first;  // check c's pairs: pidx[check_first[c] .. check_first[c+1])
    std::vector<uint32_t> pidx;         // check-major position -> slot-major pair index
    std::vector<uint32_t> lane_first;   // Miller lane l's pairs: pidx[lane_first[l] .. lane_first[l+1])
    std::vector<uint32_t> check_lane;   // check c's Miller lanes: [check_lane[c], check_lane[c+1])
    std::vector<uint8_t> bad_len;
    bool final3 = false;                // final exponentiation on three cooperating lanes per check
};
// Final exponentiation layout: one lane per check is a ~10^4-product dependent chain; when the batch
// gives the SIMDs fewer than one such wave each, three lanes per check share its exponentiations by
// u (a third of the chain).  GSV_BN_FINAL3 = 0/1 forces the choice (A/B timing).
static bool bn_final3(size_t nchecks, int cus) {
    if (const char* e = getenv("GSV_BN_FINAL3")) return atoi(e) != 0;
    return nchecks < (size_t)std::max(cus, 1) * 4 * 64;
}
// Pairs per Miller lane.  Every lane of a check runs the 64-step loop (its F_p^12 squarings are per
// lane), so k = 4 pairs per lane spends the fewest products; but one lane is a long dependent chain,
// and a batch that gives the GPU's SIMDs fewer than `waves` waves each is latency-bound, so smaller
// batches split a check over more lanes (k = 2, 1).  GSV_BN_PAIRS_PER_LANE forces k (A/B timing).
static uint32_t bn_pairs_per_lane(size_t np, int cus) {
    if (const char* e = getenv("GSV_BN_PAIRS_PER_LANE")) {
        int k = atoi(e);
        if (k >= 1) return (uint32_t)k;
    }
    const size_t waves = 1;
    size_t target = (size_t)std::max(cus, 1) * 4 * 64 * waves;
    for (uint32_t k = 4; k > 1; k >>= 1)
        if ((np + k - 1) / k >= target) return k;
    return 1;
}
static int bn_tables(const uint64_t* off, size_t n, uint64_t base, int cus, BnTables& t) {
    t.check_first.resize(n + 1);
    t.bad_len.assign(n, 0);
    size_t np = 0, maxk = 0;
    for (size_t c = 0; c < n; c++) {
        if (off[c + 1] < off[c]) return GSV_E_INVALID_ARG;
        uint64_t len = off[c + 1] - off[c];
        if (len % 192) t.bad_len[c] = 1;
        else {
            np += len / 192;
            maxk = std::max<size_t>(maxk, len / 192);
        }
    }
    if (np > 0xFFFFFFFFull) return GSV_E_TOO_LARGE;
    // slot-major order: slot k holds the k-th pair of every check that has more than k pairs
    std::vector<uint32_t> per_slot(maxk + 1, 0);
    for (size_t c = 0; c < n; c++) {
        if (t.bad_len[c]) continue;
        per_slot[(off[c + 1] - off[c]) / 192]++;  // histogram of pair counts
    }
    std::vector<uint64_t> slot_base(maxk + 1, 0), fill(maxk + 1, 0);
    {
        uint64_t more = 0;  // checks with > k pairs, from the top
        std::vector<uint64_t> gt(maxk + 1, 0);
        for (size_t k = maxk + 1; k-- > 0;) {
            gt[k] = more;
            more += per_slot[k];
        }
        uint64_t acc = 0;
        for (size_t k = 0; k < maxk; k++) {
            slot_base[k] = acc;
            acc += gt[k];
        }
    }
    t.pair_src.resize(np);
    t.pidx.resize(np);
    size_t q = 0;
    for (size_t c = 0; c < n; c++) {
        t.check_first[c] = (uint32_t)q;
        if (t.bad_len[c]) continue;
        size_t k = 0;
        for (uint64_t o = off[c]; o < off[c + 1]; o += 192, k++) {
            uint64_t j = slot_base[k] + fill[k]++;
            t.pair_src[j] = o - base;
            t.pidx[q++] = (uint32_t)j;
        }
    }
    t.check_first[n] = (uint32_t)q;
    uint32_t k = bn_pairs_per_lane(np, cus);
    t.check_lane.resize(n + 1);
    t.lane_first.clear();
    t.lane_first.reserve(n + np / k + 2);
    for (size_t c = 0; c < n; c++) {
        t.check_lane[c] = (uint32_t)t.lane_first.size();
        uint32_t b = t.check_first[c], e = t.check_first[c + 1];
        t.lane_first.push_back(b);  // a check without pairs still gets one (empty) lane
        for (uint32_t p = b + k; p < e; p += k) t.lane_first.push_back(p);
    }
    t.check_lane[n] = (uint32_t)t.lane_first.size();
    t.lane_first.push_back((uint32_t)q);
    t.final3 = bn_final3(n, cus);
    return GSV_SUCCESS;
}
static int device_cus(int device) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
    return cus;
}

// enqueue the three pairing kernels; d_in already in HBM, tables from the host
static int bn_run(gsv_ctx* c, const uint8_t* d_in, const BnTables& t, size_t n, uint8_t* d_verdict,
                  hipStream_t st) {
    size_t np = t.pair_src.size();
    size_t nl = t.lane_first.size() - 1;
    size_t need = al(np * 8 + 8) + al((nl + 1) * 4) + al((n + 1) * 4) + al(np * 4 + 4) + al(np + 1) +
                  al(np * 48 * 4 + 4) + al(np * 64 * 4 + 4) + al(nl + 1) + al(nl * 96 * 4 + 4);
    work_begin(c, st);
    int rc = work_reserve(c, need + 4096);
    if (rc) return rc;
    Carve cv(c->work);
    uint64_t* d_src = cv.take<uint64_t>(np * 8 + 8);
    uint32_t* d_lfirst = cv.take<uint32_t>((nl + 1) * 4);
    uint32_t* d_clane = cv.take<uint32_t>((n + 1) * 4);
    uint32_t* d_pidx = cv.take<uint32_t>(np * 4 + 4);
    uint8_t* d_pstat = cv.take<uint8_t>(np + 1);
    uint32_t* d_pts = cv.take<uint32_t>(np * 48 * 4 + 4);
    uint32_t* d_rs = cv.take<uint32_t>(np * 64 * 4 + 4);
    uint8_t* d_lstat = cv.take<uint8_t>(nl + 1);
    uint32_t* d_fv = cv.take<uint32_t>(nl * 96 * 4 + 4);
    if (np) HIPCHK(hipMemcpyAsync(d_src, t.pair_src.data(), np * 8, hipMemcpyHostToDevice, st));
    if (np) HIPCHK(hipMemcpyAsync(d_pidx, t.pidx.data(), np * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_lfirst, t.lane_first.data(), (nl + 1) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_clane, t.check_lane.data(), (n + 1) * 4, hipMemcpyHostToDevice, st));
    c->cur_stream = st;
    HIPCHK(gsv::launch_bn256_pairing(d_in, d_src, (uint32_t)np, d_lfirst, d_pidx, (uint32_t)nl, d_clane, (uint32_t)n,
                                     d_pstat, d_pts, d_rs, d_lstat, d_fv, d_verdict, t.final3, st, hook_begin,
                                     hook_end, c));
    // errBadPairingInput for ragged lengths overrides the kernel's verdict (those checks had no pairs)
    static const uint8_t bad = GSV_PAIRING_BAD_INPUT;
    for (size_t i = 0; i < n; i++)
        if (t.bad_len[i]) HIPCHK(hipMemcpyAsync(d_verdict + i, &bad, 1, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // host tables must outlive the async copies
    return GSV_SUCCESS;
}

int gsv_bn256_pairing_check_batch_dev(gsv_ctx* c, const uint8_t* d_in, const uint64_t* h_off, size_t n,
                                      uint8_t* d_verdict, void* stream) {
    if (!c || (n && (!h_off || !d_verdict))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > 0xFFFFFFFFull) return GSV_E_TOO_LARGE;
    BnTables t;
    int rc = bn_tables(h_off, n, 0, device_cus(c->device), t);
    if (rc) return rc;
    if (!t.pair_src.empty() && !d_in) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->wmu);
    HIPCHK(hipSetDevice(c->device));
    return bn_run(c, d_in, t, n, d_verdict, stream ? (hipStream_t)stream : c->stream);
}

int gsv_bn256_pairing_check_batch(gsv_ctx* c, const uint8_t* in, const uint64_t* off, size_t n, uint8_t* verdict) {
    if (!c || (n && (!off || !verdict))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > 0xFFFFFFFFull) return GSV_E_TOO_LARGE;
    BnTables t;
    int rc = bn_tables(off, n, off[0], device_cus(c->device), t);
    if (rc) return rc;
    if (!t.pair_src.empty() && !in) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    size_t bytes = off[n] - off[0];
    rc = arena_reserve(c, al(bytes + 8) + al(n));
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_in = cv.take<uint8_t>(bytes + 8);
    uint8_t* d_v = cv.take<uint8_t>(n);
    if (bytes) HIPCHK(hipMemcpyAsync(d_in, in + off[0], bytes, hipMemcpyHostToDevice, c->stream));
    {
        std::lock_guard<std::mutex> g2(c->wmu);
        rc = bn_run(c, d_in, t, n, d_v, c->stream);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(verdict, d_v, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

int gsv_bn256_synth_checks_dev(gsv_ctx* c, uint64_t seed, size_t nchecks, uint8_t* d_out768, uint8_t* d_expect,
                               void* stream) {
    if (!c || (nchecks && !d_out768) || nchecks > 0x3FFFFFFFull) return GSV_E_INVALID_ARG;
    HIPCHK(hipSetDevice(c->device));
    return hip_err(gsv::launch_bn256_synth(seed, (uint32_t)nchecks, d_out768, d_expect,
                                           stream ? (hipStream_t)stream : c->stream));
}

// ------------------------------------------------------------------ notary validation (configs[3])
int gsv_notary_synth_dev(gsv_ctx* c, uint64_t seed, uint32_t shard0, size_t n_shards, uint32_t txs_per_shard,
                         uint8_t* d_bodies, uint8_t* d_exp_status, uint8_t* d_exp_sender, void* stream) {
    if (!c || (n_shards && !d_bodies) || (uint64_t)n_shards * txs_per_shard > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    HIPCHK(hipSetDevice(c->device));
    return hip_err(gsv::launch_notary_synth(seed, shard0, (uint32_t)n_shards, txs_per_shard, c->gtab, d_bodies,
                                            d_exp_status, d_exp_sender, stream ? (hipStream_t)stream : c->stream));
}

static int notary_dev_impl(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* start, const uint64_t* end,
                           size_t n, const uint8_t* cid, size_t cidlen, int signer_kind, uint32_t max_txs,
                           uint8_t* d_root, uint32_t* d_ntx, uint8_t* d_bitmap, uint8_t* d_senders, uint8_t* d_status,
                           hipStream_t st) {
    if (cidlen > 64) return GSV_E_INVALID_ARG;
    for (size_t i = 0; i < n; i++)
        if (end[i] < start[i] || end[i] - start[i] > MAX_BODY) return GSV_E_TOO_LARGE;
    work_begin(c, st);  // nwork / work of a previous call may still be in use on another stream
    // chain-id buffers: 64-byte big-endian value and the sighash suffix rlp(chainId) || 0x80 0x80
    uint8_t host[256] = {0};
    memcpy(host + 64 - cidlen, cid, cidlen);
    size_t z = 0;
    while (z < cidlen && cid[z] == 0) z++;
    size_t cn = cidlen - z, sl = 0;
    uint8_t* suf = host + 64;
    if (cn == 1 && cid[z] < 0x80) suf[sl++] = cid[z];
    else {
        suf[sl++] = (uint8_t)(0x80 + cn);
        memcpy(suf + sl, cid + z, cn);
        sl += cn;
    }
    suf[sl++] = 0x80;
    suf[sl++] = 0x80;
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    for (size_t i = 0; i < n; i++) {
        offs[i] = start[i];
        lens[i] = (uint32_t)(end[i] - start[i]);
    }
    size_t bm = (max_txs + 7) / 8;
    size_t need = al(256) + al(n * 8) + al(n * 4) + al(n * 4) + al((size_t)n * max_txs * gsv::blob_rec_bytes());
    if (need > c->nwork_cap) {
        size_t cap = std::max(need, (size_t)16 << 20);
        if (c->nwork) {
            hipDeviceSynchronize();
            hipFree(c->nwork);
            c->nwork = nullptr;
            c->nwork_cap = 0;
        }
        if (hipMalloc(&c->nwork, cap) != hipSuccess) return GSV_E_NOMEM;
        c->nwork_cap = cap;
    }
    Carve cv(c->nwork);
    uint8_t* d_cid = cv.take<uint8_t>(256);
    uint64_t* d_off = cv.take<uint64_t>(n * 8);
    uint32_t* d_len = cv.take<uint32_t>(n * 4);
    uint32_t* d_cnt = d_ntx ? d_ntx : cv.take<uint32_t>(n * 4);
    void* d_blobs = cv.take<uint8_t>((size_t)n * max_txs * gsv::blob_rec_bytes());
    HIPCHK(hipMemcpyAsync(d_cid, host, 256, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_off, offs.data(), n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_len, lens.data(), n * 4, hipMemcpyHostToDevice, st));
    if (d_senders) HIPCHK(hipMemsetAsync(d_senders, 0, (size_t)n * max_txs * 20, st));
    if (d_status) HIPCHK(hipMemsetAsync(d_status, GSV_ST_BAD_RLP, (size_t)n * max_txs, st));
    c->cur_stream = st;
    hook_begin(c, GSV_K_NOTARY);
    HIPCHK(gsv::launch_blob_index(d_bodies, d_off, d_len, (uint32_t)n, max_txs, d_blobs, d_cnt, st));
    HIPCHK(gsv::launch_notary_tx(d_bodies, d_off, d_blobs, d_cnt, (uint32_t)n, max_txs, d_cid, d_cid + 64,
                                 (uint32_t)sl, signer_kind, c->gtab, d_bitmap, (uint32_t)bm, d_senders, d_status,
                                 st));
    hook_end(c, GSV_K_NOTARY);
    // chunk roots of the same bodies (own workspace)
    return chunk_root_dev_impl(c, d_bodies, start, end, n, d_root, st);
}

int gsv_notary_validate_shards_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n_shards,
                                   const uint8_t* chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                                   uint8_t* d_root32, uint32_t* d_ntx, uint8_t* d_bitmap, uint8_t* d_senders,
                                   uint8_t* d_status, void* stream) {
    if (!c || (n_shards && (!d_bodies || !h_off || !d_root32 || !d_bitmap))) return GSV_E_INVALID_ARG;
    if ((chain_id_len && !chain_id) || signer_kind < GSV_SIGNER_EIP155 || signer_kind > GSV_SIGNER_FRONTIER)
        return GSV_E_INVALID_ARG;
    if (n_shards == 0) return GSV_SUCCESS;
    if (n_shards > 65535 || max_txs == 0) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->wmu);
    HIPCHK(hipSetDevice(c->device));
    return notary_dev_impl(c, d_bodies, h_off, h_off + 1, n_shards, chain_id, chain_id_len, signer_kind, max_txs,
                           d_root32, d_ntx, d_bitmap, d_senders, d_status, stream ? (hipStream_t)stream : c->stream);
}

int gsv_notary_validate_shards(gsv_ctx* c, const uint8_t* bodies, const uint64_t* off, size_t n_shards,
                               const uint8_t* chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                               uint8_t* root32_out, uint32_t* ntx_out, uint8_t* valid_bitmap_out,
                               uint8_t* senders_out, uint8_t* status_out) {
    if (!c || (n_shards && (!bodies || !off || !root32_out || !ntx_out || !valid_bitmap_out))) return GSV_E_INVALID_ARG;
    if ((chain_id_len && !chain_id) || signer_kind < GSV_SIGNER_EIP155 || signer_kind > GSV_SIGNER_FRONTIER)
        return GSV_E_INVALID_ARG;
    if (n_shards == 0) return GSV_SUCCESS;
    if (n_shards > 65535 || max_txs == 0 || chain_id_len > 64) return GSV_E_INVALID_ARG;
    for (size_t i = 0; i < n_shards; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > MAX_BODY) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    std::vector<uint64_t> st(n_shards), en(n_shards);
    uint64_t pos = 0;
    for (size_t i = 0; i < n_shards; i++) {
        st[i] = pos;
        en[i] = pos + (off[i + 1] - off[i]);
        pos = (en[i] + 15) & ~15ull;
    }
    size_t bm = (max_txs + 7) / 8, nt = n_shards * (size_t)max_txs;
    int rc = arena_reserve(c, al(pos + 16) + al(n_shards * 32) + al(n_shards * 4) + al(n_shards * bm) +
                                  al(nt * 20) + al(nt));
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_b = cv.take<uint8_t>(pos + 16);
    uint8_t* d_r = cv.take<uint8_t>(n_shards * 32);
    uint32_t* d_n = cv.take<uint32_t>(n_shards * 4);
    uint8_t* d_bm = cv.take<uint8_t>(n_shards * bm);
    uint8_t* d_snd = senders_out ? cv.take<uint8_t>(nt * 20) : nullptr;
    uint8_t* d_st = status_out ? cv.take<uint8_t>(nt) : nullptr;
    for (size_t i = 0; i < n_shards; i++)
        if (en[i] > st[i])
            HIPCHK(hipMemcpyAsync(d_b + st[i], bodies + off[i], en[i] - st[i], hipMemcpyHostToDevice, c->stream));
    {
        std::lock_guard<std::mutex> g2(c->wmu);
        rc = notary_dev_impl(c, d_b, st.data(), en.data(), n_shards, chain_id, chain_id_len, signer_kind, max_txs,
                             d_r, d_n, d_bm, d_snd, d_st, c->stream);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(root32_out, d_r, n_shards * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(ntx_out, d_n, n_shards * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(valid_bitmap_out, d_bm, n_shards * bm, hipMemcpyDeviceToHost, c->stream));
    if (senders_out) HIPCHK(hipMemcpyAsync(senders_out, d_snd, nt * 20, hipMemcpyDeviceToHost, c->stream));
    if (status_out) HIPCHK(hipMemcpyAsync(status_out, d_st, nt, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < n_shards; i++)
        if (ntx_out[i] > max_txs) return GSV_E_TOO_LARGE;
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ DeriveSha over any DerivableList
static const uint64_t MAX_LIST = 1ull << 24;

// item k = d_vals[voff[k] .. voff[k+1]); list i = items [list_off[i], list_off[i+1])
static int derive_sha_dev_impl(gsv_ctx* c, const uint8_t* d_vals, const uint64_t* voff, const uint64_t* list_off,
                               size_t n, uint8_t* d_roots, hipStream_t st) {
    std::map<uint64_t, std::vector<uint32_t>> groups;
    for (size_t i = 0; i < n; i++) {
        if (list_off[i + 1] < list_off[i]) return GSV_E_INVALID_ARG;
        uint64_t N = list_off[i + 1] - list_off[i];
        if (N > MAX_LIST) return GSV_E_TOO_LARGE;
        groups[N].push_back((uint32_t)i);
    }
    uint64_t total = list_off[n] - list_off[0];
    for (uint64_t k = list_off[0]; k < list_off[n]; k++)
        if (voff[k + 1] < voff[k] || voff[k + 1] - voff[k] >= (1ull << 32)) return GSV_E_INVALID_ARG;
    // per item: message buffer offset (8-aligned, value + 24 bytes of RLP headers) and ref slot
    // per-item leaf message buffers are placed by the kernel (k_derive_leaf): aligned bytes + 32 per item
    uint64_t pos = ((voff[list_off[n]] - voff[list_off[0]] + 7) & ~7ull) + 32ull * total;
    size_t need = al((total + 1) * 8) + al(pos + 256) + al(total * 48);
    for (auto& g : groups) {
        if (g.first == 0) continue;
        gsv::TriePlan* pl = c->plans.get((uint32_t)g.first, true);
        if (!pl) return GSV_E_NOMEM;
        need += al(g.second.size() * 8) + al(g.second.size() * 32) +
                al(gsv::derive_sha_scratch_bytes(pl, (uint32_t)g.second.size()));
    }
    work_begin(c, st);
    int rc = work_reserve(c, need + 4096);
    if (rc) return rc;
    Carve cv(c->work);
    c->cur_stream = st;
    // voff rebased to d_vals is what the caller gave; items indexed from list_off[0]
    uint64_t* d_voff = cv.take<uint64_t>((total + 1) * 8);
    uint8_t* d_lmsg = cv.take<uint8_t>(pos + 256);
    uint8_t* d_leafrefs = cv.take<uint8_t>(total * 48);
    HIPCHK(hipMemcpyAsync(d_voff, voff + list_off[0], (total + 1) * 8, hipMemcpyHostToDevice, st));
    std::vector<std::vector<uint64_t>> host_base;
    host_base.reserve(groups.size());
    for (auto& g : groups) {
        const auto& idx = g.second;
        if (g.first == 0) {  // empty list -> emptyRoot (trie/trie.go:472-474)
            for (uint32_t i : idx)
                HIPCHK(hipMemcpyAsync(d_roots + (size_t)i * 32, EMPTY_ROOT, 32, hipMemcpyHostToDevice, st));
            continue;
        }
        gsv::TriePlan* pl = c->plans.get((uint32_t)g.first, true);
        uint64_t* d_base = cv.take<uint64_t>(idx.size() * 8);
        uint8_t* d_gr = cv.take<uint8_t>(idx.size() * 32);
        uint8_t* d_scr = cv.take<uint8_t>(gsv::derive_sha_scratch_bytes(pl, (uint32_t)idx.size()));
        host_base.emplace_back(idx.size());
        auto& hb = host_base.back();
        for (size_t k = 0; k < idx.size(); k++) hb[k] = list_off[idx[k]] - list_off[0];
        HIPCHK(hipMemcpyAsync(d_base, hb.data(), hb.size() * 8, hipMemcpyHostToDevice, st));
        HIPCHK(gsv::launch_derive_sha_plan(pl, (uint32_t)idx.size(), d_vals, d_voff, d_base, d_lmsg,
                                           d_leafrefs, d_scr, d_gr, st, hook_begin, hook_end, c));
        size_t k = 0;
        while (k < idx.size()) {
            size_t e2 = k + 1;
            while (e2 < idx.size() && idx[e2] == idx[e2 - 1] + 1) e2++;
            HIPCHK(hipMemcpyAsync(d_roots + (size_t)idx[k] * 32, d_gr + k * 32, (e2 - k) * 32,
                                  hipMemcpyDeviceToDevice, st));
            k = e2;
        }
    }
    HIPCHK(hipStreamSynchronize(st));  // host staging must outlive the async copies
    return GSV_SUCCESS;
}

int gsv_derive_sha_batch_dev(gsv_ctx* c, const uint8_t* d_vals, const uint64_t* voff, const uint64_t* list_off,
                             size_t n, uint8_t* d_root32_out, void* stream) {
    if (!c || (n && (!voff || !list_off || !d_root32_out))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (list_off[n] > list_off[0] && !d_vals) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->wmu);
    HIPCHK(hipSetDevice(c->device));
    return derive_sha_dev_impl(c, d_vals, voff, list_off, n, d_root32_out, stream ? (hipStream_t)stream : c->stream);
}

int gsv_derive_sha_batch(gsv_ctx* c, const uint8_t* vals, const uint64_t* voff, const uint64_t* list_off, size_t n,
                         uint8_t* root32_out) {
    if (!c || (n && (!voff || !list_off || !root32_out))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (list_off[n] < list_off[0]) return GSV_E_INVALID_ARG;
    uint64_t v0 = voff[list_off[0]], v1 = voff[list_off[n]];
    if (v1 < v0 || (v1 > v0 && !vals)) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    // stage the values (rebased so item list_off[0] starts at 0)
    std::vector<uint64_t> rv(list_off[n] + 1, 0);
    for (uint64_t k = list_off[0]; k <= list_off[n]; k++) rv[k] = voff[k] - v0;
    int rc = arena_reserve(c, al(v1 - v0 + 16) + al(n * 32));
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_v = cv.take<uint8_t>(v1 - v0 + 16);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    if (v1 > v0) HIPCHK(hipMemcpyAsync(d_v, vals + v0, v1 - v0, hipMemcpyHostToDevice, c->stream));
    {
        std::lock_guard<std::mutex> g2(c->wmu);
        rc = derive_sha_dev_impl(c, d_v, rv.data(), list_off, n, d_r, c->stream);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(root32_out, d_r, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ Proof of Custody
static const uint64_t MAX_POC = 1ull << 26;

static int poc_dev_impl(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* start, const uint64_t* end, size_t n,
                        const uint8_t* salt, size_t slen, uint8_t* d_poc, hipStream_t st) {
    work_begin(c, st);  // pwork of a previous call may still be read on another stream
    std::vector<uint64_t> io(2 * n), oo(n), os(n), oe(n);
    uint64_t pos = 0, mx = 0;
    for (size_t i = 0; i < n; i++) {
        if (end[i] < start[i]) return GSV_E_INVALID_ARG;
        uint64_t L = end[i] - start[i];
        if (L > MAX_POC) return GSV_E_TOO_LARGE;
        uint64_t N = L ? L * (slen + 1) : slen;
        if (N > MAX_POC) return GSV_E_TOO_LARGE;
        io[2 * i] = start[i];
        io[2 * i + 1] = end[i];
        oo[i] = os[i] = pos;
        oe[i] = pos + N;
        mx = N > mx ? N : mx;
        pos = (oe[i] + 15) & ~15ull;
    }
    size_t need = al(pos + 16) + al(2 * n * 8) + al(n * 8) + al(slen + 1);
    if (need > c->pwork_cap) {
        size_t cap = c->pwork_cap ? c->pwork_cap : (size_t)64 << 20;
        while (cap < need) cap *= 2;
        if (c->pwork) {
            hipDeviceSynchronize();
            hipFree(c->pwork);
            c->pwork = nullptr;
            c->pwork_cap = 0;
        }
        if (hipMalloc(&c->pwork, cap) != hipSuccess) return GSV_E_NOMEM;
        c->pwork_cap = cap;
    }
    Carve cv(c->pwork);
    uint8_t* d_out = cv.take<uint8_t>(pos + 16);
    uint64_t* d_io = cv.take<uint64_t>(2 * n * 8);
    uint64_t* d_oo = cv.take<uint64_t>(n * 8);
    uint8_t* d_salt = cv.take<uint8_t>(slen + 1);
    HIPCHK(hipMemcpyAsync(d_io, io.data(), 2 * n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_oo, oo.data(), n * 8, hipMemcpyHostToDevice, st));
    if (slen) HIPCHK(hipMemcpyAsync(d_salt, salt, slen, hipMemcpyHostToDevice, st));
    HIPCHK(gsv::launch_poc_expand(d_bodies, d_io, d_oo, (uint32_t)n, mx, d_salt, (uint32_t)slen, d_out, st));
    return chunk_root_dev_impl(c, d_out, os.data(), oe.data(), n, d_poc, st, MAX_POC);
}

int gsv_collation_poc_batch_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n,
                                const uint8_t* salt, size_t salt_len, uint8_t* d_poc32_out, void* stream) {
    if (!c || (n && (!h_off || !d_poc32_out)) || (salt_len && !salt)) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->wmu);
    HIPCHK(hipSetDevice(c->device));
    return poc_dev_impl(c, d_bodies, h_off, h_off + 1, n, salt, salt_len, d_poc32_out,
                        stream ? (hipStream_t)stream : c->stream);
}

int gsv_collation_poc_batch(gsv_ctx* c, const uint8_t* bodies, const uint64_t* off, size_t n, const uint8_t* salt,
                            size_t salt_len, uint8_t* poc32_out) {
    if (!c || (n && (!off || !poc32_out)) || (salt_len && !salt)) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > MAX_POC) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    std::vector<uint64_t> st(n), en(n);
    uint64_t pos = 0;
    for (size_t i = 0; i < n; i++) {
        st[i] = pos;
        en[i] = pos + (off[i + 1] - off[i]);
        pos = (en[i] + 15) & ~15ull;
    }
    int rc = arena_reserve(c, al(pos + 16) + al(n * 32));
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_b = cv.take<uint8_t>(pos + 16);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    for (size_t i = 0; i < n; i++)
        if (en[i] > st[i])
            HIPCHK(hipMemcpyAsync(d_b + st[i], bodies + off[i], en[i] - st[i], hipMemcpyHostToDevice, c->stream));
    {
        std::lock_guard<std::mutex> g2(c->wmu);
        rc = poc_dev_impl(c, d_b, st.data(), en.data(), n, salt, salt_len, d_r, c->stream);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(poc32_out, d_r, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ collation header + proposer signature
int gsv_collation_header_verify_batch_dev(gsv_ctx* c, const uint8_t* d_sid, const uint8_t* d_root,
                                          const uint8_t* d_per, const uint8_t* d_prop, const uint8_t* d_sig,
                                          const uint8_t* d_nil, size_t n, uint8_t* d_hash, uint8_t* d_signer,
                                          uint8_t* d_st, void* stream) {
    if (!c || (n && (!d_sid || !d_root || !d_per || !d_prop || !d_sig || !d_st))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > (1u << 30)) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->wmu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    work_begin(c, st);
    int rc = work_reserve(c, al(gsv::header_scratch_bytes((uint32_t)n)));
    if (rc) return rc;
    {
        KTimer t(c, GSV_K_HEADER, st);
        HIPCHK(gsv::launch_header_verify(d_sid, d_root, d_per, d_prop, d_sig, d_nil, (uint32_t)n, c->gtab, c->work,
                                         d_hash, d_signer, d_st, st));
    }
    work_end(c, st);
    return GSV_SUCCESS;
}

int gsv_collation_header_verify_batch(gsv_ctx* c, const uint8_t* shard_id32, const uint8_t* chunk_root32,
                                      const uint8_t* period32, const uint8_t* proposer20, const uint8_t* sig65,
                                      const uint8_t* nil_flags, size_t n, uint8_t* hash32_out,
                                      uint8_t* signer20_out, uint8_t* status) {
    if (!c || (n && (!shard_id32 || !chunk_root32 || !period32 || !proposer20 || !sig65 || !status)))
        return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > (1u << 30)) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    int rc = arena_reserve(c, al(n * 32) * 4 + al(n * 20) * 2 + al(n * 65) + al(n) * 2 +
                                  al(gsv::header_scratch_bytes((uint32_t)n)));
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_sid = cv.take<uint8_t>(n * 32);
    uint8_t* d_root = cv.take<uint8_t>(n * 32);
    uint8_t* d_per = cv.take<uint8_t>(n * 32);
    uint8_t* d_prop = cv.take<uint8_t>(n * 20);
    uint8_t* d_sig = cv.take<uint8_t>(n * 65);
    uint8_t* d_nil = nil_flags ? cv.take<uint8_t>(n) : nullptr;
    uint8_t* d_hash = hash32_out ? cv.take<uint8_t>(n * 32) : nullptr;
    uint8_t* d_signer = signer20_out ? cv.take<uint8_t>(n * 20) : nullptr;
    uint8_t* d_st = cv.take<uint8_t>(n);
    uint8_t* d_scr = cv.take<uint8_t>(gsv::header_scratch_bytes((uint32_t)n));
    hipStream_t st = c->stream;
    HIPCHK(hipMemcpyAsync(d_sid, shard_id32, n * 32, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_root, chunk_root32, n * 32, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_per, period32, n * 32, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_prop, proposer20, n * 20, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_sig, sig65, n * 65, hipMemcpyHostToDevice, st));
    if (d_nil) HIPCHK(hipMemcpyAsync(d_nil, nil_flags, n, hipMemcpyHostToDevice, st));
    {
        KTimer t(c, GSV_K_HEADER, st);
        HIPCHK(gsv::launch_header_verify(d_sid, d_root, d_per, d_prop, d_sig, d_nil, (uint32_t)n, c->gtab, d_scr,
                                         d_hash, d_signer, d_st, st));
    }
    if (hash32_out) HIPCHK(hipMemcpyAsync(hash32_out, d_hash, n * 32, hipMemcpyDeviceToHost, st));
    if (signer20_out) HIPCHK(hipMemcpyAsync(signer20_out, d_signer, n * 20, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return GSV_SUCCESS;
}

}  // extern "C"
