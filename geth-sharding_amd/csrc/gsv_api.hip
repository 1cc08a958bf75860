// C ABI of libgsv.so (include/gsv.h): context, device memory staging, launches, timing.
//
// Host-pointer entry points stage through a grow-only device arena on the context's stream and are
// synchronous.  *_dev entry points take HBM-resident buffers and the caller's stream and only
// enqueue: they never allocate and never synchronize, so they can be captured into a HIP graph.
// Everything a *_dev call derives from its host-side arguments (trie plans per body length, device
// copies of offset tables, pairing lane tables, its workspace) lives in a PREPARED SHAPE built by the
// matching gsv_*_prepare call (which may allocate and synchronize) and cached per context, keyed by
// exactly those host-side arguments.  A *_dev call whose shape was not prepared returns
// GSV_E_NOT_PREPARED without touching the device.  With a pipeline depth D > 1
// (gsv_ctx_set_pipeline_depth) a shape holds D instances of its device memory, so calls of the same
// shape on up to D streams run concurrently (a notary validating consecutive collation batches keeps
// the latency-bound top of one batch's trie under the next batch's leaf level).
#include <rccl/rccl.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "chunk_root.h"
#include "gsv_internal.h"
#include "tx_host.h"

namespace {

size_t al(size_t b) { return (b + 255) & ~(size_t)255; }

// regions of one device allocation (256-B aligned offsets)
struct Layout {
    size_t n = 0;
    size_t add(size_t bytes) {
        size_t o = n;
        n += al(bytes ? bytes : 1);
        return o;
    }
};

enum ShapeKind : uint64_t {
    SK_CHUNK = 1, SK_PAIRING = 2, SK_NOTARY = 3, SK_DERIVE = 4, SK_POC = 5, SK_HEADER = 6, SK_PARTITION = 7
};

// scatter run: roots of group positions [from, from + count) go to output indices [dst, dst + count)
struct Run { uint32_t dst, from, count; };

// one launch of the trie-plan kernels over the bodies (or lists) of one length
struct TrieGroup {
    std::shared_ptr<gsv::TriePlan> plan;
    uint32_t count = 0;
    size_t koff = 0;      // chunk: first entry in the body-offset table
    bool direct = false;  // chunk: roots written in place (one group holding bodies 0..n-1 in order)
    size_t o_roots = 0, o_scr = 0, o_base = 0;
    std::vector<Run> runs;
};

// chunk roots of a set of bodies (d_bodies[start[i] .. end[i]))
struct ChunkLaunch {
    std::vector<TrieGroup> groups;
    std::vector<uint32_t> empty;  // zero-length bodies -> emptyRoot
    size_t o_off = 0, o_empty = 0;
};

struct Shape {
    uint64_t kind = 0;
    std::vector<uint64_t> key;
    uint8_t* mem = nullptr;
    size_t bytes = 0;   // one instance
    int ninst = 1;      // instances of the device memory (pipeline depth at prepare time)
    int cur = 0;        // instance of the run in progress (set by shape_run under the context's smu)
    int rr = 0;         // next instance to recycle when every instance was last used on another stream
    bool owned = true;  // false: carved from the host-path arena
    std::vector<hipEvent_t> ev;     // per instance: recorded after its last (non-captured) use
    std::vector<hipStream_t> last;  // per instance: stream of that use
    // pipelined instances: per instance, recorded where its last run's bulk kernels ended
    // (GSV_HOOK_TAIL); the next run on another instance starts its bulk kernels after that point
    std::vector<hipEvent_t> bulk_ev;
    std::vector<char> bulk_rec;
    int prev = -1;  // instance of the previous run
    std::vector<std::pair<size_t, std::vector<uint8_t>>> uploads;  // host tables, copied at prepare
    ChunkLaunch chunk;  // SK_CHUNK, SK_NOTARY, SK_POC
    // SK_PAIRING
    size_t np = 0, nl = 0, nchecks = 0;
    int layout = 0;  // GSV_BN_LAYOUT_* flags
    size_t o_src = 0, o_pidx = 0, o_lfirst = 0, o_clane = 0, o_cbad = 0, o_pstat = 0, o_lines = 0,
           o_lstat = 0, o_fv = 0, o_fws = 0;
    uint32_t maxl = 1;  // the most Miller lanes of any check
    int deep = 0;  // pairing layout class of the depth it was prepared at (bn_depth_class)
    // per instance, the side stream and fork/join events of a shape that runs two launch chains at
    // once (the notary's chunk roots beside its transactions), created at prepare
    std::vector<hipStream_t> side;
    std::vector<hipEvent_t> efork, ejoin;
    bool side_borrowed = false;  // host-path shape: the context's side stream and events, not its own
    int* side_queues = nullptr;  // prepared shape: the context's count of live side queues (own streams)
    // SK_NOTARY
    uint32_t max_txs = 0, sfx_len = 0;
    int signer_kind = 0;
    size_t o_cid = 0, o_noff = 0, o_nlen = 0, o_cnt = 0, o_blobs = 0;
    // SK_DERIVE
    std::vector<TrieGroup> dgroups;
    std::vector<uint32_t> dempty;
    size_t o_voff = 0, o_lmsg = 0, o_leafrefs = 0, o_dempty = 0;
    uint64_t vend = 0;  // end of the batch's value bytes (absolute offset into the caller's vals)
    // SK_POC
    size_t o_io = 0, o_oo = 0, o_salt = 0, o_out = 0;
    uint64_t poc_max = 0;
    uint32_t salt_len = 0;
    // SK_HEADER
    size_t o_hscr = 0;
    // SK_PARTITION (+ the SK_NOTARY fields of the rank's own block)
    size_t p_n = 0, p_total = 0;
    int p_ranks = 1, p_rank = 0;
    size_t o_lroot = 0, o_lntx = 0, o_lbm = 0, o_block = 0, o_all = 0;

    Shape() = default;
    Shape(const Shape&) = delete;
    Shape& operator=(const Shape&) = delete;
    // the shape's own side streams (hardware queues) and events; a borrowed set stays the context's
    void release_side() {
        if (!side_borrowed) {
            for (hipStream_t q : side)
                if (q) {
                    hipStreamSynchronize(q);
                    hipStreamDestroy(q);
                    if (side_queues) --*side_queues;
                }
            for (hipEvent_t e : efork)
                if (e) hipEventDestroy(e);
            for (hipEvent_t e : ejoin)
                if (e) hipEventDestroy(e);
        }
        side.clear();
        efork.clear();
        ejoin.clear();
    }
    ~Shape() {
        release_side();
        for (hipEvent_t e : ev)
            if (e) hipEventDestroy(e);
        for (hipEvent_t e : bulk_ev)
            if (e) hipEventDestroy(e);
        if (owned && mem) hipFree(mem);
    }
    template <typename T>
    void stage(size_t off, const T* p, size_t count) {
        if (!count) return;
        const uint8_t* b = (const uint8_t*)p;
        uploads.emplace_back(off, std::vector<uint8_t>(b, b + count * sizeof(T)));
    }
    template <typename T>
    T* at(size_t off) const { return (T*)(mem + (size_t)cur * bytes + off); }
};

constexpr size_t kMaxShapes = 32;
// side streams on hardware queues of their own, over all of a context's prepared shapes: the hardware
// scheduler time-slices queues beyond what it maps at once (r05: ~40 leaked queues ran an 8,192-check
// pairing pipeline at 8.6 instead of 3.8 ms, profiles/r05/ab/pairing_depth_dedicated_leaked_queues.txt);
// a shape prepared past the bound runs its chains one after the other on the caller's stream.
// GSV_MAX_SIDE_STREAMS (0..8) lowers the bound: 0 = no side streams, every notary step runs its chunk
// roots after its transactions on one stream (the leg-only profile pass: tools/profile_round.sh, so no
// dispatch of a traced step overlaps another)
constexpr int kMaxSideQueues = 8;
int max_side_queues() {
    static const int v = [] {
        const char* e = getenv("GSV_MAX_SIDE_STREAMS");
        return e ? std::min(std::max(atoi(e), 0), kMaxSideQueues) : kMaxSideQueues;
    }();
    return v;
}
constexpr size_t kMaxShapeBytes = (size_t)32 << 30;  // of the 288 GB of HBM

}  // namespace

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
    std::vector<hipEvent_t> open_ev;  // timer events opened by launch hooks
    hipStream_t cur_stream = nullptr;  // stream of the shape run in progress (launch hooks)
    bool cur_capture = false;          // that run is being captured into a graph: no timer events
    Shape* cur_shape = nullptr;        // the shape of that run (GSV_HOOK_TAIL marks)
    // trie plans per body length, prepared shapes (most recently used first)
    gsv::PlanCache plans;
    std::list<std::unique_ptr<Shape>> shapes;
    size_t shape_bytes = 0;
    std::mutex smu;  // shapes, cur_stream / cur_capture
    // RCCL communicator of the shard partition (gsv_comm_init), nullptr = single rank
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // completion of the last all-gather issued on `comm`: the next one, possibly on another stream (a
    // pipelined partition call), waits for it, so collectives on the communicator never overlap
    hipEvent_t coll_ev = nullptr;
    bool coll_rec = false;
    std::mutex cmu;  // the collective: coll_ev / coll_rec and the ncclAllGather issue order
    // the host paths' side stream and fork/join events (lent to their per-call shapes)
    hipStream_t hside = nullptr;
    hipEvent_t hfork = nullptr, hjoin = nullptr;
    // live side streams of the prepared shapes (each shape owns its own, on hardware queues of their
    // own, own_queue_stream: HIP's four shared in-order queues would order a side chain after unrelated
    // work; the notary pipeline two deep measured 11,734 vs 11,419 shards/s, profiles/r05/ab/notary_sweep_*)
    int side_queues = 0;
    // streams made by gsv_stream_create, destroyed by gsv_stream_destroy or with the context
    std::vector<hipStream_t> user_streams;
    std::mutex qmu;
    int pipeline_depth = 1;  // instances per prepared shape (gsv_ctx_set_pipeline_depth)
};

namespace {

int hip_err(hipError_t e) { return e == hipSuccess ? GSV_SUCCESS : GSV_E_HIP; }

#define HIPCHK(x)                                  \
    do {                                           \
        hipError_t _e = (x);                       \
        if (_e != hipSuccess) return GSV_E_HIP;    \
    } while (0)

bool capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) return false;
    return cs != hipStreamCaptureStatusNone;
}

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

// Brackets one launch with events on the launching stream when timing is on (never inside a capture).
struct KTimer {
    gsv_ctx* c;
    int kid;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    KTimer(gsv_ctx* c_, int kid_, hipStream_t st_) : c(c_), kid(kid_), st(st_) {
        if (c->timing && !capturing(st)) {
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

// timer hooks for multi-launch paths (chunk-root levels, pairing stages)
void hook_begin(void* p, int kid) {
    gsv_ctx* c = (gsv_ctx*)p;
    if (kid == gsv::GSV_HOOK_TAIL) {  // the run's bulk kernels are enqueued: mark the point for the next run
        Shape* s = c->cur_shape;
        if (s && !c->cur_capture && !s->bulk_ev.empty()) {
            hipEventRecord(s->bulk_ev[s->cur], c->cur_stream);
            s->bulk_rec[s->cur] = 1;
        }
        return;
    }
    if (!c->timing || c->cur_capture) return;
    std::lock_guard<std::mutex> g(c->tmu);
    hipEvent_t a = take_event(c);
    hipEventRecord(a, c->cur_stream);
    c->open_ev.push_back(a);
}
void hook_end(void* p, int kid) {
    gsv_ctx* c = (gsv_ctx*)p;
    if (!c->timing || c->cur_capture) return;
    std::lock_guard<std::mutex> g(c->tmu);
    hipEvent_t a = c->open_ev.back();
    c->open_ev.pop_back();
    hipEvent_t b = take_event(c);
    hipEventRecord(b, c->cur_stream);
    c->pending.push_back({kid, a, b});
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

// ------------------------------------------------------------------ prepared shapes
// allocates `ninst` instances (or, for a host-path shape, carves one) of the shape's memory and
// uploads its host tables into each
int shape_materialize(Shape& s, size_t bytes, uint8_t* carve = nullptr, int ninst = 1) {
    bytes = al(bytes ? bytes : 1);
    s.bytes = bytes;
    s.ninst = carve ? 1 : std::max(ninst, 1);
    if (carve) {
        s.mem = carve;
        s.owned = false;
    } else if (hipMalloc(&s.mem, bytes * s.ninst) != hipSuccess) {
        s.mem = nullptr;
        return GSV_E_NOMEM;
    }
    for (int k = 0; k < s.ninst; k++)
        for (auto& u : s.uploads)
            HIPCHK(hipMemcpy(s.mem + (size_t)k * bytes + u.first, u.second.data(), u.second.size(), hipMemcpyHostToDevice));
    s.uploads.clear();
    s.uploads.shrink_to_fit();
    s.ev.assign(s.ninst, nullptr);
    s.last.assign(s.ninst, nullptr);
    if (s.owned)
        for (auto& e : s.ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    s.bulk_ev.assign(s.ninst > 1 ? s.ninst : 0, nullptr);
    s.bulk_rec.assign(s.bulk_ev.size(), 0);
    for (auto& e : s.bulk_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return GSV_SUCCESS;
}

size_t shape_total_bytes(const Shape& s) { return s.bytes * (size_t)s.ninst; }

void shape_drain(Shape& s) {
    for (hipEvent_t e : s.ev)
        if (e) hipEventSynchronize(e);
}

Shape* shape_find(gsv_ctx* c, uint64_t kind, const std::vector<uint64_t>& key) {
    for (auto it = c->shapes.begin(); it != c->shapes.end(); ++it) {
        Shape* s = it->get();
        if (s->kind == kind && s->key == key) {
            if (it != c->shapes.begin()) c->shapes.splice(c->shapes.begin(), c->shapes, it);
            return s;
        }
    }
    return nullptr;
}

// inserts a materialized shape; drops least-recently-used shapes beyond the bounds (after their
// queued work has drained — a graph captured from a dropped shape must not be replayed)
void shape_insert(gsv_ctx* c, std::unique_ptr<Shape> s) {
    c->shape_bytes += shape_total_bytes(*s);
    c->shapes.push_front(std::move(s));
    while (c->shapes.size() > 1 && (c->shapes.size() > kMaxShapes || c->shape_bytes > kMaxShapeBytes)) {
        Shape* v = c->shapes.back().get();
        shape_drain(*v);
        c->shape_bytes -= shape_total_bytes(*v);
        c->shapes.pop_back();
    }
}

// The instance a run on `st` uses: the one last used on `st` (the stream orders it), else one never
// used, else the next in turn, ordered after its previous use.  Inside a capture: the instance last
// used on `st`, else instance 0 (the caller orders graph replays against other uses of the shape).
int shape_pick(Shape& s, hipStream_t st, bool cap) {
    for (int k = 0; k < s.ninst; k++)
        if (s.last[k] == st) return k;
    if (cap) return 0;
    for (int k = 0; k < s.ninst; k++)
        if (!s.last[k]) return k;
    int k = s.rr;
    s.rr = (s.rr + 1) % s.ninst;
    return k;
}

// Runs a shape's launches on `st`.  Users of one shape on different streams are ordered on the GPU
// (the workspace is the shape's); inside a stream capture no event is touched, and the caller orders
// graph replays against other uses of the same shape.
template <typename F>
int shape_run(gsv_ctx* c, Shape& s, hipStream_t st, F&& body) {
    bool cap = capturing(st);
    int k = shape_pick(s, st, cap);
    s.cur = k;
    if (!cap && s.ev[k] && s.last[k] && s.last[k] != st) HIPCHK(hipStreamWaitEvent(st, s.ev[k], 0));
    if (!cap && !s.bulk_ev.empty()) {
        // staggered pipeline: this run's bulk kernels follow the previous run's (on the other
        // instance), so they overlap that run's latency-bound tail rather than its bulk kernels
        if (s.prev >= 0 && s.prev != k && s.bulk_rec[s.prev]) HIPCHK(hipStreamWaitEvent(st, s.bulk_ev[s.prev], 0));
        s.bulk_rec[k] = 0;
        s.prev = k;
    }
    c->cur_stream = st;
    c->cur_capture = cap;
    c->cur_shape = &s;
    int rc = body();
    c->cur_shape = nullptr;
    s.cur = 0;
    if (rc) return rc;
    if (!cap && s.ev[k]) {
        HIPCHK(hipEventRecord(s.ev[k], st));
        s.last[k] = st;
    }
    return GSV_SUCCESS;
}

void key_push_bytes(std::vector<uint64_t>& key, const uint8_t* p, size_t n) {
    key.push_back(n);
    for (size_t i = 0; i < n; i += 8) {
        uint64_t w = 0;
        memcpy(&w, p + i, std::min<size_t>(8, n - i));
        key.push_back(w);
    }
}

// ------------------------------------------------------------------ chunk root launch description
static const uint8_t EMPTY_ROOT[32] = {0x56, 0xe8, 0x1f, 0x17, 0x1b, 0xcc, 0x55, 0xa6, 0xff, 0x83, 0x45,
                                       0xe6, 0x92, 0xc0, 0xf8, 0x6e, 0x5b, 0x48, 0xe0, 0x1b, 0x99, 0x6c,
                                       0xad, 0xc0, 0x01, 0x62, 0x2f, 0xb5, 0xe3, 0x63, 0xb4, 0x21};
constexpr uint64_t MAX_BODY = 1ull << 20;  // collationSizelimit (sharding/collation.go:45)
constexpr uint64_t MAX_POC = 1ull << 26;   // salted bodies (Proof of Custody)
constexpr uint64_t MAX_LIST = 1ull << 24;  // generic DeriveSha items per list

std::vector<Run> runs_of(const std::vector<uint32_t>& idx) {
    std::vector<Run> r;
    size_t k = 0;
    while (k < idx.size()) {
        size_t e = k + 1;
        while (e < idx.size() && idx[e] == idx[e - 1] + 1) e++;
        r.push_back({idx[k], (uint32_t)k, (uint32_t)(e - k)});
        k = e;
    }
    return r;
}

// bodies grouped by length (the trie shape depends only on N, chunk_root.h)
int chunk_prepare(gsv_ctx* c, Shape& s, ChunkLaunch& cl, Layout& L, const uint64_t* start, const uint64_t* end,
                  size_t n, uint64_t max_len) {
    std::map<uint64_t, std::vector<uint32_t>> groups;
    for (size_t i = 0; i < n; i++) {
        if (end[i] < start[i] || end[i] - start[i] > max_len) return GSV_E_TOO_LARGE;
        groups[end[i] - start[i]].push_back((uint32_t)i);
    }
    std::vector<uint64_t> offs;
    offs.reserve(n);
    for (auto& g : groups) {
        if (g.first == 0) {  // empty trie -> emptyRoot (trie/trie.go:472-474)
            cl.empty = g.second;
            continue;
        }
        TrieGroup tg;
        tg.plan = c->plans.get((uint32_t)g.first);
        if (!tg.plan) return GSV_E_NOMEM;
        tg.count = (uint32_t)g.second.size();
        tg.koff = offs.size();
        tg.direct = g.second.size() == n;
        for (uint32_t i : g.second) offs.push_back(start[i]);
        if (!tg.direct) {
            tg.o_roots = L.add((size_t)tg.count * 32);
            tg.runs = runs_of(g.second);
        }
        tg.o_scr = L.add(gsv::chunk_root_scratch_bytes(tg.plan.get(), tg.count));
        cl.groups.push_back(std::move(tg));
    }
    cl.o_off = L.add(offs.size() * 8);
    cl.o_empty = L.add(32);
    s.stage(cl.o_off, offs.data(), offs.size());
    s.stage(cl.o_empty, EMPTY_ROOT, 32);
    return GSV_SUCCESS;
}

int chunk_run(gsv_ctx* c, const Shape& s, const ChunkLaunch& cl, const uint8_t* d_bodies, uint8_t* d_roots,
              hipStream_t st) {
    for (const TrieGroup& g : cl.groups) {
        uint8_t* d_gr = g.direct ? d_roots : s.at<uint8_t>(g.o_roots);
        HIPCHK(gsv::launch_chunk_root_plan(g.plan.get(), d_bodies, s.at<uint64_t>(cl.o_off) + g.koff, g.count,
                                           s.at<uint8_t>(g.o_scr), d_gr, st, hook_begin, hook_end, c));
        for (const Run& r : g.runs)
            HIPCHK(hipMemcpyAsync(d_roots + (size_t)r.dst * 32, d_gr + (size_t)r.from * 32, (size_t)r.count * 32,
                                  hipMemcpyDeviceToDevice, st));
    }
    for (uint32_t i : cl.empty)
        HIPCHK(hipMemcpyAsync(d_roots + (size_t)i * 32, s.at<uint8_t>(cl.o_empty), 32, hipMemcpyDeviceToDevice, st));
    return GSV_SUCCESS;
}

int device_cus(int device);

// A stream on an HSA queue of its own: HIP multiplexes ordinary streams over GPU_MAX_HW_QUEUES (4) shared
// in-order queues, but backs a CU-masked stream (here: every CU) by a dedicated queue.  It is ordered with
// the legacy NULL stream like a hipStreamDefault stream.
int own_queue_stream(int device, hipStream_t* q) {
    const int cus = device_cus(device);
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
    for (int i = 0; i < cus; i++) mask[i / 32] |= 1u << (i % 32);
    HIPCHK(hipExtStreamCreateWithCUMask(q, (uint32_t)mask.size(), mask.data()));
    return GSV_SUCCESS;
}

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
        case GSV_E_NOT_PREPARED: return "batch shape not prepared (call the matching gsv_*_prepare first)";
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
    // a BLOCKING stream: a *_dev call made with stream = NULL is ordered with the legacy default
    // (NULL) stream of the process both ways — a caller's prior fills and copies there (e.g. PyTorch's
    // default stream) complete before it, and later default-stream work sees its results
    if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess) {
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
    hipDeviceSynchronize();  // every stream's work on the context's shapes has drained
    drain_timing(c);
    for (auto e : c->free_events) hipEventDestroy(e);
    c->shapes.clear();
    {
        std::lock_guard<std::mutex> g(c->qmu);
        for (hipStream_t q : c->user_streams) hipStreamDestroy(q);
        c->user_streams.clear();
    }
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->coll_ev) hipEventDestroy(c->coll_ev);
    if (c->hfork) hipEventDestroy(c->hfork);
    if (c->hjoin) hipEventDestroy(c->hjoin);
    if (c->hside) hipStreamDestroy(c->hside);
    if (c->arena) hipFree(c->arena);
    if (c->gtab) hipFree(c->gtab);
    hipStreamDestroy(c->stream);
    delete c;
}

int gsv_ctx_set_timing(gsv_ctx* c, int enable) {
    if (!c) return GSV_E_INVALID_ARG;
    c->timing = enable ? 1 : 0;
    return GSV_SUCCESS;
}

// A pipeline's streams on queues of their own (gsv.h): r05 measured 8,192-check pairing batches three
// deep at 6.0 or 3.75 ms per batch by which of torch's pool streams the caller took (two of the three on
// one HSA queue in the kernel trace), 3.75 on every set of CU-masked streams
// (profiles/r05/ab/stream_sets_*).
// The context owns them: at most GSV_MAX_STREAMS live at once (more queues oversubscribe the hardware
// scheduler), and gsv_ctx_destroy destroys the ones the caller did not, before the runtime's own teardown.
int gsv_stream_create(gsv_ctx* c, void** stream_out) {
    if (!c || !stream_out) return GSV_E_INVALID_ARG;
    *stream_out = nullptr;
    std::lock_guard<std::mutex> g(c->qmu);
    if (c->user_streams.size() >= GSV_MAX_STREAMS) return GSV_E_INVALID_ARG;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t q = nullptr;
    int rc = own_queue_stream(c->device, &q);
    if (rc) return rc;
    c->user_streams.push_back(q);
    *stream_out = (void*)q;
    return GSV_SUCCESS;
}

int gsv_stream_destroy(gsv_ctx* c, void* stream) {
    if (!c || !stream) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->qmu);
    auto it = std::find(c->user_streams.begin(), c->user_streams.end(), (hipStream_t)stream);
    if (it == c->user_streams.end()) return GSV_E_INVALID_ARG;  // not this context's (or already destroyed)
    c->user_streams.erase(it);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamDestroy((hipStream_t)stream));
    return GSV_SUCCESS;
}

int gsv_ctx_stream_count(gsv_ctx* c, int* user_streams, int* side_streams) {
    if (!c) return GSV_E_INVALID_ARG;
    {
        std::lock_guard<std::mutex> g(c->qmu);
        if (user_streams) *user_streams = (int)c->user_streams.size();
    }
    std::lock_guard<std::mutex> g(c->smu);
    if (side_streams) *side_streams = c->side_queues;
    return GSV_SUCCESS;
}

int gsv_ctx_set_pipeline_depth(gsv_ctx* c, int depth) {
    if (!c || depth < 1 || depth > GSV_MAX_PIPELINE_DEPTH) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->smu);
    c->pipeline_depth = depth;
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

int gsv_ctx_prepared_shapes(gsv_ctx* c, size_t* count, size_t* device_bytes) {
    if (!c) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->smu);
    if (count) *count = c->shapes.size();
    if (device_bytes) *device_bytes = c->shape_bytes;
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
    for (size_t i = 0; i < n; i++)  // the kernel trusts off[i] <= off[i+1]
        if (off[i + 1] < off[i]) return GSV_E_INVALID_ARG;
    if (off[n] > off[0] && !data) return GSV_E_INVALID_ARG;
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

// ------------------------------------------------------------------ ecrecover precompile (contracts.go:78-101)
int gsv_ecrecover_precompile_batch_dev(gsv_ctx* c, const uint8_t* d_in128, size_t n, uint8_t* d_out32, uint8_t* d_ok,
                                       void* stream) {
    if (!c || (n && (!d_in128 || !d_out32 || !d_ok)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    KTimer t(c, GSV_K_ECRECOVER, st);
    return hip_err(gsv::launch_ecrecover_precompile(d_in128, (uint32_t)n, c->gtab, d_out32, d_ok, st));
}

int gsv_ecrecover_precompile_batch(gsv_ctx* c, const uint8_t* in, const uint64_t* off, size_t n, uint8_t* out32,
                                   uint8_t* ok) {
    if (!c || (n && (!off || !out32 || !ok)) || n > 0xFFFFFFFFull) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) return GSV_E_INVALID_ARG;
    if (off[n] > off[0] && !in) return GSV_E_INVALID_ARG;
    // common.RightPadBytes(input, 128); only input[0:128] is read (contracts.go:81-90)
    std::vector<uint8_t> pad(n * 128, 0);
    for (size_t i = 0; i < n; i++) {
        size_t len = std::min<uint64_t>(off[i + 1] - off[i], 128);
        if (len) memcpy(&pad[i * 128], in + off[i], len);
    }
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    int rc = arena_reserve(c, al(n * 128) + al(n * 32) + al(n));
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_in = cv.take<uint8_t>(n * 128);
    uint8_t* d_out = cv.take<uint8_t>(n * 32);
    uint8_t* d_ok = cv.take<uint8_t>(n);
    HIPCHK(hipMemcpyAsync(d_in, pad.data(), n * 128, hipMemcpyHostToDevice, c->stream));
    rc = gsv_ecrecover_precompile_batch_dev(c, d_in, n, d_out, d_ok, c->stream);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(out32, d_out, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(ok, d_ok, n, hipMemcpyDeviceToHost, c->stream));
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

}  // extern "C"

// ================================================================== shape builders per entry point
namespace {

// ---- chunk root: key = body offsets
std::vector<uint64_t> chunk_key(const uint64_t* h_off, size_t n) {
    std::vector<uint64_t> k(h_off, h_off + n + 1);
    return k;
}
int chunk_shape(gsv_ctx* c, Shape& s, const uint64_t* start, const uint64_t* end, size_t n, Layout& L) {
    s.kind = SK_CHUNK;
    return chunk_prepare(c, s, s.chunk, L, start, end, n, MAX_BODY);
}

// ---- BN254 pairing: check c = in[off[c] .. off[c+1]); a length that is not a multiple of 192 is
// errBadPairingInput (core/vm/contracts.go:336-338) and contributes no pairs.
// Final exponentiation layout: one lane per check is a ~10^4-product dependent chain; when the batch
// gives the SIMDs fewer than one such wave each, three lanes per check share its exponentiations by
// u (a third of the chain).  GSV_BN_FINAL3 = 0/1 forces the choice (A/B timing).
// From BN_DEEP batches in flight the other batches fill what one small batch leaves idle even at k = 4
// pairs per Miller lane and one lane per check in the final exponentiation (the layout with the fewest
// products): 8,192 checks 3.13 ms per batch at depth 6 against 3.30 for the depth-3 rule's k = 2 /
// three-lane final at depth 4 (r06, profiles/r06/ab/pairing_rank_depth.txt; k = 4 at depth 4: 3.86).
constexpr int BN_DEEP = 6;
// the depth classes whose pairing layouts differ: 1-2, 3-5 (bn_pairs_per_lane's sixth-of-a-wave
// target, no two-lane Miller), 6 and up
int bn_depth_class(int depth) { return depth >= BN_DEEP ? 2 : depth >= 3 ? 1 : 0; }
bool bn_final3(size_t nchecks, int cus, int depth) {
    if (const char* e = getenv("GSV_BN_FINAL3")) return atoi(e) != 0;
    return depth < BN_DEEP && nchecks < (size_t)std::max(cus, 1) * 4 * 64;
}
// Two lanes per Miller lane while twice the Miller lanes still fit one wave per SIMD (the Miller
// kernel's register budget admits one wave per SIMD).  GSV_BN_MILLER2 = 0/1 forces the choice.
// With three or more batches in flight (pipeline depth) the other batches' kernels fill the SIMDs a
// small batch leaves idle, so the work-efficient layout wins: no second Miller lane.
bool bn_miller2(size_t nlanes, int cus, int depth) {
    if (const char* e = getenv("GSV_BN_MILLER2")) return atoi(e) != 0;
    return depth < 3 && 2 * nlanes <= (size_t)std::max(cus, 1) * 4 * 64;
}
// The Miller loop at two waves per SIMD (k_bn_miller_w2: one F_p^6 value per lane in LDS, products one
// output coordinate at a time) or at one (k_bn_miller, the default).  The two-wave kernel measured
// slower at every batch size (r05: 65,536 checks at k = 2 11.2 vs 9.8 ms of Miller, k = 4 17.0 vs
// 8.3 ms; 8,192 checks three deep 4.7 vs 3.75 ms per batch, profiles/r05/ab/miller_w2_sweep_*.txt):
// 19 % more VALU per line product and exposed LDS / line-load latency outweigh the second wave.
// GSV_BN_MILLER_W2 = 1 selects it (A/B and its GPU test).
bool bn_miller_w2() {
    if (const char* e = getenv("GSV_BN_MILLER_W2")) return atoi(e) != 0;
    return false;
}
// The Miller loop at two waves per SIMD with each line in LDS (k_bn_miller_l, r05; GSV_BN_MILLER_L = 1).
bool bn_miller_l() {
    if (const char* e = getenv("GSV_BN_MILLER_L")) return atoi(e) != 0;
    return false;
}
// The lines at two waves per SIMD (k_bn_lines_w2: P and Q in LDS, coefficients stored as computed; 256
// registers, no scratch) or at one (k_bn_lines, 256 + 125).  Measured (r05, profiles/r05/ab/lines_w2_*,
// pipe_l*): alone at 65,536 checks 5.95 vs 6.67 ms; in the two-deep pipeline equal (19.98 vs 19.96 ms per
// batch), three deep 19.9-20.0 vs 20.2 ms; at 8,192 checks three deep 4.12 vs 3.75 ms per batch (slower:
// its 512 waves then share SIMDs with the other batches' one-wave Miller / final waves, which a two-wave
// budget cannot join).  So the two-wave kernel is taken from four waves' worth of pairs per SIMD up.
// GSV_BN_LINES_W2 = 0/1 forces the choice.
bool bn_lines_w2(size_t npairs, int cus) {
    if (const char* e = getenv("GSV_BN_LINES_W2")) return atoi(e) != 0;
    return npairs >= (size_t)std::max(cus, 1) * 4 * 64 * 4;
}
// Pairs per Miller lane.  Every lane of a check runs the 64-step loop (its F_p^12 squarings are per
// lane), so k = 4 pairs per lane spends the fewest products; but one lane is a long dependent chain,
// and a batch that gives the GPU's SIMDs fewer than `waves` waves each is latency-bound, so smaller
// batches split a check over more lanes (k = 2, 1).  GSV_BN_PAIRS_PER_LANE forces k (A/B timing).
// At pipeline depth >= 3 a batch only needs a sixth of that (batches overlap): 8,192 checks 4.69 ->
// 3.66 ms per batch at depth 4 with k = 2 and no second Miller lane, 16,384 6.96 -> 6.04 ms at depth 3
// with k = 4 (profiles/r03/ab_pairing_layout_pipe.txt).
uint32_t bn_pairs_per_lane(size_t np, int cus, int depth) {
    if (const char* e = getenv("GSV_BN_PAIRS_PER_LANE")) {
        int k = atoi(e);
        if (k >= 1) return (uint32_t)k;
    }
    if (depth >= BN_DEEP) return 4;  // six or more batches in flight: the most work-efficient layout
    const size_t waves = bn_miller_w2() ? 2 : 1;  // Miller waves per SIMD the kernel's registers admit
    size_t target = (size_t)std::max(cus, 1) * 4 * 64 * waves / (depth >= 3 ? 6 : 1);
    for (uint32_t k = 4; k > 1; k >>= 1)
        if ((np + k - 1) / k >= target) return k;
    return 1;
}
int device_cus(int device) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
    return cus;
}
// key: the offsets plus the A/B overrides of the layout choice (tools/pairing_sweep.py)
std::vector<uint64_t> pairing_key(const uint64_t* h_off, size_t n) {
    const char* k = getenv("GSV_BN_PAIRS_PER_LANE");
    const char* f = getenv("GSV_BN_FINAL3");
    const char* m = getenv("GSV_BN_MILLER2");
    const char* cc = getenv("GSV_BN_CONC");
    const char* w2 = getenv("GSV_BN_MILLER_W2");
    const char* lw = getenv("GSV_BN_LINES_W2");
    const char* ml = getenv("GSV_BN_MILLER_L");
    std::vector<uint64_t> key{k ? (uint64_t)atoi(k) + 1 : 0, f ? (uint64_t)atoi(f) + 1 : 0, m ? (uint64_t)atoi(m) + 1 : 0,
                              cc ? (uint64_t)atoi(cc) + 1 : 0, w2 ? (uint64_t)atoi(w2) + 1 : 0, lw ? (uint64_t)atoi(lw) + 1 : 0,
                              ml ? (uint64_t)atoi(ml) + 1 : 0};
    key.insert(key.end(), h_off, h_off + n + 1);
    return key;
}
// depth: batches the caller keeps in flight on this shape (1 for the synchronous host path)
int pairing_shape(gsv_ctx* c, Shape& s, const uint64_t* off, size_t n, Layout& L, int depth) {
    s.kind = SK_PAIRING;
    int cus = device_cus(c->device);
    std::vector<uint8_t> bad_len(n, 0);
    size_t np = 0, maxk = 0;
    for (size_t k = 0; k < n; k++) {
        if (off[k + 1] < off[k]) return GSV_E_INVALID_ARG;
        uint64_t len = off[k + 1] - off[k];
        if (len % 192) bad_len[k] = 1;
        else {
            np += len / 192;
            maxk = std::max<size_t>(maxk, len / 192);
        }
    }
    if (np > 0xFFFFFFFFull) return GSV_E_TOO_LARGE;
    // slot-major order: slot k holds the k-th pair of every check that has more than k pairs
    std::vector<uint64_t> per_slot(maxk + 1, 0), slot_base(maxk + 1, 0), fill(maxk + 1, 0);
    for (size_t k = 0; k < n; k++)
        if (!bad_len[k]) per_slot[(off[k + 1] - off[k]) / 192]++;  // histogram of pair counts
    {
        uint64_t more = 0, acc = 0;  // checks with > k pairs, from the top
        std::vector<uint64_t> gt(maxk + 1, 0);
        for (size_t k = maxk + 1; k-- > 0;) {
            gt[k] = more;
            more += per_slot[k];
        }
        for (size_t k = 0; k < maxk; k++) {
            slot_base[k] = acc;
            acc += gt[k];
        }
    }
    std::vector<uint64_t> pair_src(np);
    std::vector<uint32_t> pidx(np), check_first(n + 1);
    size_t q = 0;
    for (size_t k = 0; k < n; k++) {
        check_first[k] = (uint32_t)q;
        if (bad_len[k]) continue;
        size_t slot = 0;
        for (uint64_t o = off[k]; o < off[k + 1]; o += 192, slot++) {
            uint64_t j = slot_base[slot] + fill[slot]++;
            pair_src[j] = o;
            pidx[q++] = (uint32_t)j;
        }
    }
    check_first[n] = (uint32_t)q;
    uint32_t kpl = bn_pairs_per_lane(np, cus, depth);
    std::vector<uint32_t> check_lane(n + 1), lane_first;
    lane_first.reserve(n + np / kpl + 2);
    s.maxl = 1;
    for (size_t k = 0; k < n; k++) {
        check_lane[k] = (uint32_t)lane_first.size();
        uint32_t b = check_first[k], e = check_first[k + 1];
        lane_first.push_back(b);  // a check without pairs still gets one (empty) lane
        for (uint32_t p = b + kpl; p < e; p += kpl) lane_first.push_back(p);
        s.maxl = std::max<uint32_t>(s.maxl, (uint32_t)(lane_first.size() - check_lane[k]));
    }
    check_lane[n] = (uint32_t)lane_first.size();
    lane_first.push_back((uint32_t)q);
    s.np = np;
    s.nl = lane_first.size() - 1;
    s.nchecks = n;
    s.deep = bn_depth_class(depth);
    s.layout = (bn_final3(n, cus, depth) ? gsv::GSV_BN_LAYOUT_FINAL3 : 0) |
               (bn_miller2(s.nl, cus, depth) ? gsv::GSV_BN_LAYOUT_MILLER2 : 0) |
               (bn_miller_w2() ? gsv::GSV_BN_LAYOUT_MILLERW2 : 0) |
               (bn_lines_w2(np, cus) ? gsv::GSV_BN_LAYOUT_LINESW2 : 0) | (bn_miller_l() ? gsv::GSV_BN_LAYOUT_MILLERL : 0);
    s.o_src = L.add(np * 8 + 8);
    s.o_pidx = L.add(np * 4 + 4);
    s.o_lfirst = L.add((s.nl + 1) * 4);
    s.o_clane = L.add((n + 1) * 4);
    s.o_cbad = L.add(n);
    s.o_pstat = L.add(np + 1);
    // the pairs' Miller-loop lines (bn256.hip BN_NLINES).
    // The final exponentiation's workspace (BN_FINAL_SLOTS F_p^12 values per check) reuses the region:
    // the lines are dead once the Miller kernel, which precedes k_bn_final on the run's stream, is done.
    // (a separate region measured the same, r04)
    const size_t lines_bytes = np * 91 * 54 * 4;
    const size_t fws_bytes = n * 108 * 4 * gsv::BN_FINAL_SLOTS;
    s.o_lines = L.add(std::max(lines_bytes, fws_bytes) + 4);
    s.o_lstat = L.add(s.nl + 1);
    s.o_fv = L.add(s.nl * 108 * 4 + 4);
    s.o_fws = s.o_lines;
    s.stage(s.o_src, pair_src.data(), np);
    s.stage(s.o_pidx, pidx.data(), np);
    s.stage(s.o_lfirst, lane_first.data(), lane_first.size());
    s.stage(s.o_clane, check_lane.data(), n + 1);
    s.stage(s.o_cbad, bad_len.data(), n);
    return GSV_SUCCESS;
}
// a side stream and fork/join events per instance (at prepare), for shapes that run two independent
// launch chains at once: the notary's chunk roots beside its transactions.  The streams are
// the SHAPE's own, on hardware queues of their own (a context-wide pool let an uncaptured call
// of one shape enqueue onto a side stream another shape's capture had joined); they live until the shape
// is evicted or retired.  Past kMaxSideQueues live side queues the shape being prepared takes them from
// the least recently used shapes that hold some (those then run their chains one after the other until
// they are prepared again: r06, a sweep over shard counts had left a 13-shard shape holding six queues
// and the next 25-shard shape ran serially, 2.74 instead of 2.15 ms per step).  When that is not enough
// (a capture still open on every candidate's side stream), or HIP refuses a stream or event, the shape
// gets no side streams and runs its chains one after the other on the caller's stream: the results are
// the same and the prepare succeeds (gsv.h).
int shape_side_init(gsv_ctx* c, Shape& s) {
    if (!s.side.empty()) return GSV_SUCCESS;
    const int cap = max_side_queues();
    if (s.ninst > cap) return GSV_SUCCESS;  // serial chains
    for (auto it = c->shapes.rbegin(); it != c->shapes.rend() && c->side_queues + s.ninst > cap; ++it) {
        Shape* v = it->get();
        if (v == &s || v->side.empty() || v->side_borrowed) continue;
        bool open = false;  // a graph being captured through v's side streams keeps them
        for (hipStream_t q : v->side) open = open || (q && capturing(q));
        if (!open) v->release_side();
    }
    if (c->side_queues + s.ninst > cap) return GSV_SUCCESS;  // serial chains
    s.side.assign(s.ninst, nullptr);
    s.efork.assign(s.ninst, nullptr);
    s.ejoin.assign(s.ninst, nullptr);
    s.side_queues = &c->side_queues;
    bool ok = true;
    for (int k = 0; k < s.ninst && ok; k++) {
        ok = own_queue_stream(c->device, &s.side[k]) == GSV_SUCCESS;
        if (ok) c->side_queues++;
        else s.side[k] = nullptr;
        ok = ok && hipEventCreateWithFlags(&s.efork[k], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&s.ejoin[k], hipEventDisableTiming) == hipSuccess;
    }
    if (!ok) s.release_side();  // no partial set
    return GSV_SUCCESS;
}
// a host-path (per-call) shape borrows the context's side stream and events instead of creating its own
int shape_side_borrow(gsv_ctx* c, Shape& s) {
    if (!s.side.empty()) return GSV_SUCCESS;
    if (!c->hside) {
        HIPCHK(hipStreamCreateWithFlags(&c->hside, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&c->hfork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&c->hjoin, hipEventDisableTiming));
    }
    s.side.assign(1, c->hside);
    s.efork.assign(1, c->hfork);
    s.ejoin.assign(1, c->hjoin);
    s.side_borrowed = true;
    return GSV_SUCCESS;
}
int pairing_run(gsv_ctx* c, const Shape& s, const uint8_t* d_in, uint8_t* d_verdict, hipStream_t st) {
    return hip_err(gsv::launch_bn256_pairing(
        d_in, s.at<uint64_t>(s.o_src), (uint32_t)s.np, s.at<uint32_t>(s.o_lfirst), s.at<uint32_t>(s.o_pidx),
        (uint32_t)s.nl, s.at<uint32_t>(s.o_clane), s.at<uint8_t>(s.o_cbad), (uint32_t)s.nchecks,
        s.at<uint8_t>(s.o_pstat), s.at<uint32_t>(s.o_lines), s.at<uint8_t>(s.o_lstat),
        s.at<uint32_t>(s.o_fv), s.at<uint32_t>(s.o_fws), s.maxl, d_verdict, s.layout, st, hook_begin, hook_end, c));
}

// ---- notary: key = chain id, signer, max_txs, body offsets
std::vector<uint64_t> notary_key(const uint64_t* h_off, size_t n, const uint8_t* cid, size_t cidlen, int signer,
                                 uint32_t max_txs) {
    std::vector<uint64_t> k{(uint64_t)signer, max_txs};
    key_push_bytes(k, cid, cidlen);
    k.insert(k.end(), h_off, h_off + n + 1);
    return k;
}
int notary_shape(gsv_ctx* c, Shape& s, const uint64_t* start, const uint64_t* end, size_t n, const uint8_t* cid,
                 size_t cidlen, int signer_kind, uint32_t max_txs, Layout& L) {
    s.kind = SK_NOTARY;
    if (cidlen > 64) return GSV_E_INVALID_ARG;
    for (size_t i = 0; i < n; i++)
        if (end[i] < start[i] || end[i] - start[i] > MAX_BODY) return GSV_E_TOO_LARGE;
    // chain-id buffers: 64-byte big-endian value at 0 and the sighash suffix rlp(chainId) || 0x80 0x80
    // (<= 67 bytes) at 128, zero bytes around it (k_notary_tx reads it as aligned dwords)
    uint8_t host[256] = {0};
    if (cidlen) memcpy(host + 64 - cidlen, cid, cidlen);
    size_t z = 0;
    while (z < cidlen && cid[z] == 0) z++;
    size_t cn = cidlen - z, sl = 0;
    uint8_t* suf = host + 128;
    if (cn == 1 && cid[z] < 0x80) suf[sl++] = cid[z];
    else {
        suf[sl++] = (uint8_t)(0x80 + cn);
        if (cn) memcpy(suf + sl, cid + z, cn);
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
    s.max_txs = max_txs;
    s.signer_kind = signer_kind;
    s.sfx_len = (uint32_t)sl;
    s.o_cid = L.add(256);
    s.o_noff = L.add(n * 8);
    s.o_nlen = L.add(n * 4);
    s.o_cnt = L.add(n * 4);
    s.o_blobs = L.add((size_t)n * max_txs * gsv::blob_rec_bytes());
    s.stage(s.o_cid, host, 256);
    s.stage(s.o_noff, offs.data(), n);
    s.stage(s.o_nlen, lens.data(), n);
    return chunk_prepare(c, s, s.chunk, L, start, end, n, MAX_BODY);
}
int notary_run(gsv_ctx* c, const Shape& s, size_t n, const uint8_t* d_bodies, uint8_t* d_root, uint32_t* d_ntx,
               uint8_t* d_bitmap, uint8_t* d_senders, uint8_t* d_status, hipStream_t st) {
    size_t bm = (s.max_txs + 7) / 8;
    uint32_t* d_cnt = d_ntx ? d_ntx : s.at<uint32_t>(s.o_cnt);
    if (d_senders) HIPCHK(hipMemsetAsync(d_senders, 0, n * s.max_txs * 20, st));
    if (d_status) HIPCHK(hipMemsetAsync(d_status, GSV_ST_BAD_RLP, n * s.max_txs, st));
    // The chunk roots of the same bodies are independent of the transactions: with a side stream they
    // run beside the blob decode + recovery (fork / join by events, so a capture still works) and
    // fill the SIMDs the recovery kernel's tail and the trie top leave idle.
    // The chunk roots fork onto the shape's side stream when it has one (r03: +3.3 % against the serial
    // form, profiles/r03/ab_notary_fork.txt; r05: 11,491 vs 11,233 shards/s, profiles/r05/ab/notary_fork*.json)
    const bool fork = (size_t)s.cur < s.side.size();
    // The pipelined step's mark for the next step (GSV_HOOK_TAIL, shape_run) is the chunk root's, after
    // its bottom level.  r06 A/B at 13 / 25 / 100 shards, depth 2-4: no mark, or a mark after the blob
    // index, measured the same (profiles/r06/ab/notary_stagger_steps.txt).
    if (fork) {
        HIPCHK(hipEventRecord(s.efork[s.cur], st));
        HIPCHK(hipStreamWaitEvent(s.side[s.cur], s.efork[s.cur], 0));
        hipStream_t keep = c->cur_stream;
        c->cur_stream = s.side[s.cur];  // the chunk-root launch hooks time on the stream they run on
        int rc = chunk_run(c, s, s.chunk, d_bodies, d_root, s.side[s.cur]);
        c->cur_stream = keep;
        if (rc) return rc;
        HIPCHK(hipEventRecord(s.ejoin[s.cur], s.side[s.cur]));
    }
    hook_begin(c, GSV_K_NOTARY);
    HIPCHK(gsv::launch_blob_index(d_bodies, s.at<uint64_t>(s.o_noff), s.at<uint32_t>(s.o_nlen), (uint32_t)n,
                                  s.max_txs, s.at<void>(s.o_blobs), d_cnt, st));
    HIPCHK(gsv::launch_notary_tx(d_bodies, s.at<uint64_t>(s.o_noff), s.at<void>(s.o_blobs), d_cnt, (uint32_t)n,
                                 s.max_txs, s.at<uint8_t>(s.o_cid), s.at<uint8_t>(s.o_cid) + 128, s.sfx_len,
                                 s.signer_kind, c->gtab, d_bitmap, (uint32_t)bm, d_senders, d_status, st));
    hook_end(c, GSV_K_NOTARY);
    if (fork) {
        HIPCHK(hipStreamWaitEvent(st, s.ejoin[s.cur], 0));
        return GSV_SUCCESS;
    }
    return chunk_run(c, s, s.chunk, d_bodies, d_root, st);  // chunk roots of the same bodies
}

// ---- generic DeriveSha: key = list offsets and the items' value offsets
std::vector<uint64_t> derive_key(const uint64_t* voff, const uint64_t* list_off, size_t n) {
    std::vector<uint64_t> k(list_off, list_off + n + 1);
    k.insert(k.end(), voff + list_off[0], voff + list_off[n] + 1);
    return k;
}
// item k = d_vals[voff[k] .. voff[k+1]); list i = items [list_off[i], list_off[i+1])
int derive_shape(gsv_ctx* c, Shape& s, const uint64_t* voff, const uint64_t* list_off, size_t n, Layout& L) {
    s.kind = SK_DERIVE;
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
    // per-item leaf message buffers are placed by the kernel (k_derive_leaf): aligned bytes + 32 per item
    uint64_t pos = ((voff[list_off[n]] - voff[list_off[0]] + 7) & ~7ull) + 32ull * total;
    s.o_voff = L.add((total + 1) * 8);
    s.o_lmsg = L.add(pos + 256);
    s.o_leafrefs = L.add(total * 48);
    s.o_dempty = L.add(32);
    s.stage(s.o_voff, voff + list_off[0], total + 1);
    s.vend = voff[list_off[n]];
    s.stage(s.o_dempty, EMPTY_ROOT, 32);
    for (auto& g : groups) {
        if (g.first == 0) {  // empty list -> emptyRoot (trie/trie.go:472-474)
            s.dempty = g.second;
            continue;
        }
        TrieGroup tg;
        tg.plan = c->plans.get((uint32_t)g.first, true);
        if (!tg.plan) return GSV_E_NOMEM;
        tg.count = (uint32_t)g.second.size();
        std::vector<uint64_t> base(tg.count);
        for (size_t k = 0; k < tg.count; k++) base[k] = list_off[g.second[k]] - list_off[0];
        tg.o_base = L.add(tg.count * 8);
        tg.o_roots = L.add((size_t)tg.count * 32);
        tg.o_scr = L.add(gsv::derive_sha_scratch_bytes(tg.plan.get(), tg.count));
        tg.runs = runs_of(g.second);
        s.stage(tg.o_base, base.data(), base.size());
        s.dgroups.push_back(std::move(tg));
    }
    return GSV_SUCCESS;
}
int derive_run(gsv_ctx* c, const Shape& s, const uint8_t* d_vals, uint8_t* d_roots, hipStream_t st) {
    for (const TrieGroup& g : s.dgroups) {
        uint8_t* d_gr = s.at<uint8_t>(g.o_roots);
        HIPCHK(gsv::launch_derive_sha_plan(g.plan.get(), g.count, d_vals, s.at<uint64_t>(s.o_voff), s.vend,
                                           s.at<uint64_t>(g.o_base), s.at<uint8_t>(s.o_lmsg),
                                           s.at<uint8_t>(s.o_leafrefs), s.at<uint8_t>(g.o_scr), d_gr, st, hook_begin,
                                           hook_end, c));
        for (const Run& r : g.runs)
            HIPCHK(hipMemcpyAsync(d_roots + (size_t)r.dst * 32, d_gr + (size_t)r.from * 32, (size_t)r.count * 32,
                                  hipMemcpyDeviceToDevice, st));
    }
    for (uint32_t i : s.dempty)
        HIPCHK(hipMemcpyAsync(d_roots + (size_t)i * 32, s.at<uint8_t>(s.o_dempty), 32, hipMemcpyDeviceToDevice, st));
    return GSV_SUCCESS;
}

// ---- Proof of Custody: key = salt, body offsets
std::vector<uint64_t> poc_key(const uint64_t* h_off, size_t n, const uint8_t* salt, size_t slen) {
    std::vector<uint64_t> k;
    key_push_bytes(k, salt, slen);
    k.insert(k.end(), h_off, h_off + n + 1);
    return k;
}
int poc_shape(gsv_ctx* c, Shape& s, const uint64_t* start, const uint64_t* end, size_t n, const uint8_t* salt,
              size_t slen, Layout& L) {
    s.kind = SK_POC;
    std::vector<uint64_t> io(2 * n), oo(n), os(n), oe(n);
    uint64_t pos = 0, mx = 0;
    for (size_t i = 0; i < n; i++) {
        if (end[i] < start[i]) return GSV_E_INVALID_ARG;
        uint64_t len = end[i] - start[i];
        if (len > MAX_POC) return GSV_E_TOO_LARGE;
        uint64_t N = len ? len * (slen + 1) : slen;
        if (N > MAX_POC) return GSV_E_TOO_LARGE;
        io[2 * i] = start[i];
        io[2 * i + 1] = end[i];
        oo[i] = os[i] = pos;
        oe[i] = pos + N;
        mx = N > mx ? N : mx;
        pos = (oe[i] + 15) & ~15ull;
    }
    s.poc_max = mx;
    s.salt_len = (uint32_t)slen;
    s.o_io = L.add(2 * n * 8);
    s.o_oo = L.add(n * 8);
    s.o_salt = L.add(slen + 1);
    s.o_out = L.add(pos + 16);
    s.stage(s.o_io, io.data(), io.size());
    s.stage(s.o_oo, oo.data(), oo.size());
    s.stage(s.o_salt, salt, slen);
    return chunk_prepare(c, s, s.chunk, L, os.data(), oe.data(), n, MAX_POC);
}
int poc_run(gsv_ctx* c, const Shape& s, size_t n, const uint8_t* d_bodies, uint8_t* d_poc, hipStream_t st) {
    HIPCHK(gsv::launch_poc_expand(d_bodies, s.at<uint64_t>(s.o_io), s.at<uint64_t>(s.o_oo), (uint32_t)n, s.poc_max,
                                  s.at<uint8_t>(s.o_salt), s.salt_len, s.at<uint8_t>(s.o_out), st));
    return chunk_run(c, s, s.chunk, s.at<uint8_t>(s.o_out), d_poc, st);
}

// ---- collation headers: key = batch size
int header_shape(gsv_ctx*, Shape& s, size_t n, Layout& L) {
    s.kind = SK_HEADER;
    s.o_hscr = L.add(gsv::header_scratch_bytes((uint32_t)n));
    return GSV_SUCCESS;
}

// ---- shard partition: the notary shape of this rank's block + its record block and the gathered
// blocks; key = notary key of the block + (n_total, nranks, rank)
struct PartDims {
    size_t first, n, per, R, bm, B;
};
PartDims part_dims(size_t n_total, int N, int r, uint32_t max_txs) {
    PartDims d;
    d.first = n_total * (size_t)r / (size_t)N;
    d.n = n_total * (size_t)(r + 1) / (size_t)N - d.first;
    d.per = (n_total + N - 1) / N;
    d.bm = (max_txs + 7) / 8;
    d.R = (36 + d.bm + 7) / 8 * 8;  // root 32 | ntx 4 | bitmap, padded to 8 (gsv/shards.py)
    d.B = 8 + d.per * d.R;          // header {int32 status, uint32 shards} + records
    return d;
}
std::vector<uint64_t> partition_key(const uint64_t* h_off, size_t n, size_t n_total, int N, int r, const uint8_t* cid,
                                    size_t cidlen, int signer, uint32_t max_txs) {
    std::vector<uint64_t> k = notary_key(h_off, n, cid, cidlen, signer, max_txs);
    k.push_back(n_total);
    k.push_back((uint64_t)N);
    k.push_back((uint64_t)r);
    return k;
}
int partition_shape(gsv_ctx* c, Shape& s, const uint64_t* h_off, size_t n_total, int N, int r, const uint8_t* cid,
                    size_t cidlen, int signer_kind, uint32_t max_txs, Layout& L) {
    PartDims d = part_dims(n_total, N, r, max_txs);
    if (d.n) {
        int rc = notary_shape(c, s, h_off, h_off + 1, d.n, cid, cidlen, signer_kind, max_txs, L);
        if (rc) return rc;
    }
    s.kind = SK_PARTITION;
    s.max_txs = max_txs;
    s.p_n = d.n;
    s.p_total = n_total;
    s.p_ranks = N;
    s.p_rank = r;
    s.o_lroot = L.add(d.n * 32);
    s.o_lntx = L.add(d.n * 4);
    s.o_lbm = L.add(d.n * d.bm);
    s.o_block = L.add(d.B);
    s.o_all = L.add((size_t)N * d.B);
    return GSV_SUCCESS;
}
// validate the rank's block and pack its records into `blk`
int partition_pack(gsv_ctx* c, const Shape& s, const PartDims& d, const uint8_t* d_bodies, uint8_t* d_senders,
                   uint8_t* d_status, uint8_t* blk, hipStream_t st) {
    uint8_t* lroot = s.at<uint8_t>(s.o_lroot);
    uint32_t* lntx = s.at<uint32_t>(s.o_lntx);
    uint8_t* lbm = s.at<uint8_t>(s.o_lbm);
    if (d.n) {
        int rc = notary_run(c, s, d.n, d_bodies, lroot, lntx, lbm, d_senders, d_status, st);
        if (rc) return rc;
    }
    return hip_err(gsv::launch_partition_pack(lroot, lntx, lbm, (uint32_t)d.n, (uint32_t)d.per, (uint32_t)d.R,
                                              (uint32_t)d.bm, 0, blk, st));
}
// the path's one collective: every rank's block to every rank (one ncclAllGather over xGMI)
int partition_gather(gsv_ctx* c, const uint8_t* blk, uint8_t* all, const PartDims& d, hipStream_t st) {
    if (c->comm) {  // any communicator, one rank included: the same chain on every rank count
        std::lock_guard<std::mutex> g(c->cmu);  // callers hold mu (error path) or smu (success path)
        // calls kept in flight on several streams (pipeline depth) overlap their validation, not their
        // collectives: each all-gather follows the previous one on the communicator (every rank issues
        // them in the same order).  Inside a graph capture the caller's graph orders them.
        const bool cap = capturing(st);
        if (!cap) {
            if (!c->coll_ev && hipEventCreateWithFlags(&c->coll_ev, hipEventDisableTiming) != hipSuccess)
                return GSV_E_HIP;
            if (c->coll_rec && hipStreamWaitEvent(st, c->coll_ev, 0) != hipSuccess) return GSV_E_HIP;
        }
        if (ncclAllGather(blk, all, d.B, ncclUint8, c->comm, st) != ncclSuccess) return GSV_E_RCCL;
        if (!cap) {
            if (hipEventRecord(c->coll_ev, st) != hipSuccess) return GSV_E_HIP;
            c->coll_rec = true;
        }
        return GSV_SUCCESS;
    }
    if (c->nranks > 1) return GSV_E_INVALID_ARG;
    return hip_err(hipMemcpyAsync(all, blk, d.B, hipMemcpyDeviceToDevice, st));
}

// Prepare-or-find: returns the cached shape for (kind, key), building it with `build` on a miss.
template <typename B>
int shape_get(gsv_ctx* c, uint64_t kind, std::vector<uint64_t>&& key, B&& build, Shape** out) {
    Shape* s = shape_find(c, kind, key);
    // a pairing shape's layout depends on the depth class it was prepared at (three or more batches in
    // flight pick the work-efficient layout, pairing_shape): a prepare at the other class rebuilds it
    const bool reclass = s && kind == SK_PAIRING && s->deep != bn_depth_class(c->pipeline_depth);
    if (s && (s->ninst < c->pipeline_depth || reclass)) {
        // prepared before the depth was raised (or at the other depth class): build a new one, and
        // RETIRE the old one instead of freeing it (it is never found again but keeps its memory until
        // LRU eviction, which drains its queued work first), so a graph captured from it stays valid.
        // Its side streams go now (a captured graph holds no streams): the new shape needs the queues.
        s->kind |= 1ull << 63;
        bool cap = false;  // a capture still open on a side stream keeps it until eviction
        for (hipStream_t q : s->side) cap = cap || (q && capturing(q));
        if (!cap) s->release_side();
        s = nullptr;
    }
    if (!s) {
        auto ns = std::make_unique<Shape>();
        Layout L;
        int rc = build(*ns, L);
        if (rc) return rc;
        rc = shape_materialize(*ns, L.n, nullptr, c->pipeline_depth);
        if (rc) return rc;
        ns->kind = kind;
        ns->key = std::move(key);
        s = ns.get();
        shape_insert(c, std::move(ns));
    }
    *out = s;
    return GSV_SUCCESS;
}

// Host-path shape: built per call in the arena after `staged` bytes of inputs, run, synchronized.
template <typename B>
int shape_temp(gsv_ctx* c, size_t staged, B&& build, Shape& s) {
    Layout L;
    int rc = build(s, L);
    if (rc) return rc;
    rc = arena_reserve(c, staged + L.n);
    if (rc) return rc;
    return shape_materialize(s, L.n, c->arena + staged);
}

// bodies staged in HBM with 16-byte aligned starts (vector loads in the bottom-level kernel)
uint64_t stage_offsets(const uint64_t* off, size_t n, std::vector<uint64_t>& st, std::vector<uint64_t>& en) {
    st.resize(n);
    en.resize(n);
    uint64_t pos = 0;
    for (size_t i = 0; i < n; i++) {
        st[i] = pos;
        en[i] = pos + (off[i + 1] - off[i]);
        pos = (en[i] + 15) & ~15ull;
    }
    return pos;
}
int stage_bodies(gsv_ctx* c, uint8_t* d_b, const uint8_t* bodies, const uint64_t* off, size_t n,
                 const std::vector<uint64_t>& st, const std::vector<uint64_t>& en) {
    for (size_t i = 0; i < n; i++)
        if (en[i] > st[i])
            HIPCHK(hipMemcpyAsync(d_b + st[i], bodies + off[i], en[i] - st[i], hipMemcpyHostToDevice, c->stream));
    return GSV_SUCCESS;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------ chunk root
int gsv_chunk_root_prepare(gsv_ctx* c, const uint64_t* h_off, size_t n) {
    if (!c || (n && !h_off)) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->smu);
    HIPCHK(hipSetDevice(c->device));
    Shape* s;
    return shape_get(c, SK_CHUNK, chunk_key(h_off, n),
                     [&](Shape& ns, Layout& L) { return chunk_shape(c, ns, h_off, h_off + 1, n, L); }, &s);
}

int gsv_chunk_root_batch_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n,
                             uint8_t* d_root32_out, void* stream) {
    if (!c || (n && (!h_off || !d_root32_out || !d_bodies))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->smu);
    Shape* s = shape_find(c, SK_CHUNK, chunk_key(h_off, n));
    if (!s) return GSV_E_NOT_PREPARED;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return shape_run(c, *s, st, [&] { return chunk_run(c, *s, s->chunk, d_bodies, d_root32_out, st); });
}

int gsv_chunk_root_batch(gsv_ctx* c, const uint8_t* bodies, const uint64_t* off, size_t n, uint8_t* root32_out) {
    if (!c || (n && (!off || !root32_out))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > MAX_BODY) return GSV_E_TOO_LARGE;
    if (off[n] > off[0] && !bodies) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    std::lock_guard<std::mutex> g2(c->smu);
    HIPCHK(hipSetDevice(c->device));
    std::vector<uint64_t> st, en;
    uint64_t pos = stage_offsets(off, n, st, en);
    size_t staged = al(pos + 16) + al(n * 32);
    Shape s;
    int rc = shape_temp(c, staged, [&](Shape& ns, Layout& L) { return chunk_shape(c, ns, st.data(), en.data(), n, L); },
                        s);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_b = cv.take<uint8_t>(pos + 16);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    rc = stage_bodies(c, d_b, bodies, off, n, st, en);
    if (rc) return rc;
    rc = shape_run(c, s, c->stream, [&] { return chunk_run(c, s, s.chunk, d_b, d_r, c->stream); });
    if (rc) return rc;
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
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    return tx_sender_impl(c, rlp, off, n, chain_id, chain_id_len, signer_kind, addr20_out, status);
}

// ------------------------------------------------------------------ BN254 pairing check
int gsv_bn256_pairing_prepare(gsv_ctx* c, const uint64_t* h_off, size_t n) {
    if (!c || (n && !h_off)) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > 0xFFFFFFFFull) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->smu);
    HIPCHK(hipSetDevice(c->device));
    Shape* s;
    const int depth = std::max(1, c->pipeline_depth);
    int rc = shape_get(c, SK_PAIRING, pairing_key(h_off, n),
                       [&](Shape& ns, Layout& L) { return pairing_shape(c, ns, h_off, n, L, depth); }, &s);
    return rc;
}

int gsv_bn256_pairing_check_batch_dev(gsv_ctx* c, const uint8_t* d_in, const uint64_t* h_off, size_t n,
                                      uint8_t* d_verdict, void* stream) {
    if (!c || (n && (!h_off || !d_verdict))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > 0xFFFFFFFFull) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->smu);
    Shape* s = shape_find(c, SK_PAIRING, pairing_key(h_off, n));
    if (!s) return GSV_E_NOT_PREPARED;
    if (s->np && !d_in) return GSV_E_INVALID_ARG;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return shape_run(c, *s, st, [&] { return pairing_run(c, *s, d_in, d_verdict, st); });
}

int gsv_bn256_pairing_check_batch(gsv_ctx* c, const uint8_t* in, const uint64_t* off, size_t n, uint8_t* verdict) {
    if (!c || (n && (!off || !verdict))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > 0xFFFFFFFFull) return GSV_E_TOO_LARGE;
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i]) return GSV_E_INVALID_ARG;
    if (off[n] > off[0] && !in) return GSV_E_INVALID_ARG;
    std::vector<uint64_t> rel(n + 1);
    for (size_t i = 0; i <= n; i++) rel[i] = off[i] - off[0];
    std::lock_guard<std::mutex> g(c->mu);
    std::lock_guard<std::mutex> g2(c->smu);
    HIPCHK(hipSetDevice(c->device));
    size_t bytes = off[n] - off[0];
    size_t staged = al(bytes + 8) + al(n);
    Shape s;
    int rc = shape_temp(c, staged, [&](Shape& ns, Layout& L) { return pairing_shape(c, ns, rel.data(), n, L, 1); }, s);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_in = cv.take<uint8_t>(bytes + 8);
    uint8_t* d_v = cv.take<uint8_t>(n);
    if (bytes) HIPCHK(hipMemcpyAsync(d_in, in + off[0], bytes, hipMemcpyHostToDevice, c->stream));
    rc = shape_run(c, s, c->stream, [&] { return pairing_run(c, s, d_in, d_v, c->stream); });
    if (rc) return rc;
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

static int notary_args(const uint8_t* chain_id, size_t chain_id_len, int signer_kind, size_t n_shards,
                       uint32_t max_txs) {
    if ((chain_id_len && !chain_id) || chain_id_len > 64 || signer_kind < GSV_SIGNER_EIP155 ||
        signer_kind > GSV_SIGNER_FRONTIER)
        return GSV_E_INVALID_ARG;
    // every blob takes at least one 32-byte chunk, so a body of at most 2^20 bytes holds at most
    // GSV_MAX_TXS_PER_SHARD = 32,768 of them (also keeps the partition's record offsets in 32 bits)
    if (n_shards > 65535 || max_txs == 0 || max_txs > GSV_MAX_TXS_PER_SHARD) return GSV_E_INVALID_ARG;
    return GSV_SUCCESS;
}

int gsv_notary_prepare(gsv_ctx* c, const uint64_t* h_off, size_t n_shards, const uint8_t* chain_id,
                       size_t chain_id_len, int signer_kind, uint32_t max_txs) {
    if (!c || (n_shards && !h_off)) return GSV_E_INVALID_ARG;
    int rc = notary_args(chain_id, chain_id_len, signer_kind, n_shards, max_txs);
    if (rc || n_shards == 0) return rc;
    std::lock_guard<std::mutex> g(c->smu);
    HIPCHK(hipSetDevice(c->device));
    Shape* s;
    rc = shape_get(c, SK_NOTARY, notary_key(h_off, n_shards, chain_id, chain_id_len, signer_kind, max_txs),
                   [&](Shape& ns, Layout& L) {
                       return notary_shape(c, ns, h_off, h_off + 1, n_shards, chain_id, chain_id_len, signer_kind,
                                           max_txs, L);
                   },
                   &s);
    if (rc) return rc;
    return shape_side_init(c, *s);
}

int gsv_notary_validate_shards_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n_shards,
                                   const uint8_t* chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                                   uint8_t* d_root32, uint32_t* d_ntx, uint8_t* d_bitmap, uint8_t* d_senders,
                                   uint8_t* d_status, void* stream) {
    if (!c || (n_shards && (!d_bodies || !h_off || !d_root32 || !d_bitmap))) return GSV_E_INVALID_ARG;
    int rc = notary_args(chain_id, chain_id_len, signer_kind, n_shards, max_txs);
    if (rc || n_shards == 0) return rc;
    std::lock_guard<std::mutex> g(c->smu);
    Shape* s = shape_find(c, SK_NOTARY, notary_key(h_off, n_shards, chain_id, chain_id_len, signer_kind, max_txs));
    if (!s) return GSV_E_NOT_PREPARED;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return shape_run(c, *s, st, [&] {
        return notary_run(c, *s, n_shards, d_bodies, d_root32, d_ntx, d_bitmap, d_senders, d_status, st);
    });
}

int gsv_notary_validate_shards(gsv_ctx* c, const uint8_t* bodies, const uint64_t* off, size_t n_shards,
                               const uint8_t* chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                               uint8_t* root32_out, uint32_t* ntx_out, uint8_t* valid_bitmap_out,
                               uint8_t* senders_out, uint8_t* status_out) {
    if (!c || (n_shards && (!bodies || !off || !root32_out || !ntx_out || !valid_bitmap_out))) return GSV_E_INVALID_ARG;
    int rc = notary_args(chain_id, chain_id_len, signer_kind, n_shards, max_txs);
    if (rc || n_shards == 0) return rc;
    for (size_t i = 0; i < n_shards; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > MAX_BODY) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->mu);
    std::lock_guard<std::mutex> g2(c->smu);
    HIPCHK(hipSetDevice(c->device));
    std::vector<uint64_t> st, en;
    uint64_t pos = stage_offsets(off, n_shards, st, en);
    size_t bm = (max_txs + 7) / 8, nt = n_shards * (size_t)max_txs;
    size_t staged = al(pos + 16) + al(n_shards * 32) + al(n_shards * 4) + al(n_shards * bm) + al(nt * 20) + al(nt);
    Shape s;
    rc = shape_temp(c, staged,
                    [&](Shape& ns, Layout& L) {
                        return notary_shape(c, ns, st.data(), en.data(), n_shards, chain_id, chain_id_len,
                                            signer_kind, max_txs, L);
                    },
                    s);
    if (rc) return rc;
    rc = shape_side_borrow(c, s);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_b = cv.take<uint8_t>(pos + 16);
    uint8_t* d_r = cv.take<uint8_t>(n_shards * 32);
    uint32_t* d_n = cv.take<uint32_t>(n_shards * 4);
    uint8_t* d_bm = cv.take<uint8_t>(n_shards * bm);
    uint8_t* d_snd = cv.take<uint8_t>(nt * 20);
    uint8_t* d_st = cv.take<uint8_t>(nt);
    rc = stage_bodies(c, d_b, bodies, off, n_shards, st, en);
    if (rc) return rc;
    rc = shape_run(c, s, c->stream, [&] {
        return notary_run(c, s, n_shards, d_b, d_r, d_n, d_bm, senders_out ? d_snd : nullptr,
                          status_out ? d_st : nullptr, c->stream);
    });
    if (rc) return rc;
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

// ------------------------------------------------------------------ shard partition + RCCL all-gather
// Record per shard (the layout of gsv/shards.py): root 32 | ntx 4 | bitmap ceil(max_txs/8), padded to
// 8 bytes.  Each rank packs its block's records with three strided copies, one ncclAllGather moves
// every rank's block (ceil(S/N) records, the tail of a short block unused), and three strided copies
// per rank unpack the gathered records into shard order.
int gsv_comm_unique_id(uint8_t id[GSV_COMM_ID_BYTES]) {
    if (!id) return GSV_E_INVALID_ARG;
    static_assert(sizeof(ncclUniqueId) == GSV_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return GSV_E_RCCL;
    memcpy(id, &u, sizeof(u));
    return GSV_SUCCESS;
}

int gsv_comm_init(gsv_ctx* c, const uint8_t id[GSV_COMM_ID_BYTES], int nranks, int rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    HIPCHK(hipSetDevice(c->device));
    if (c->comm) {
        ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (ncclCommInitRank(&c->comm, nranks, u, rank) != ncclSuccess) {
        c->comm = nullptr;
        return GSV_E_RCCL;
    }
    c->nranks = nranks;
    c->rank = rank;
    return GSV_SUCCESS;
}

int gsv_comm_info(gsv_ctx* c, int* nranks, int* rank) {
    if (!c) return GSV_E_INVALID_ARG;
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    return GSV_SUCCESS;
}

int gsv_shard_range(size_t n_shards, int nranks, int rank, size_t* first, size_t* count) {
    if (nranks < 1 || rank < 0 || rank >= nranks || !first || !count) return GSV_E_INVALID_ARG;
    size_t a = n_shards * (size_t)rank / (size_t)nranks, b = n_shards * (size_t)(rank + 1) / (size_t)nranks;
    *first = a;
    *count = b - a;
    return GSV_SUCCESS;
}

size_t gsv_partition_block_bytes(size_t n_total, int nranks, uint32_t max_txs) {
    if (nranks < 1) return 0;
    return part_dims(n_total, nranks, 0, max_txs).B;
}

int gsv_notary_partition_prepare(gsv_ctx* c, const uint64_t* h_off, size_t n_total, int nranks, int rank,
                                 const uint8_t* chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs) {
    if (!c || !h_off || nranks < 1 || rank < 0 || rank >= nranks) return GSV_E_INVALID_ARG;
    int rc = notary_args(chain_id, chain_id_len, signer_kind, n_total, max_txs);
    if (rc) return rc;
    if (n_total > 0xFFFFFFFFull / 4096) return GSV_E_TOO_LARGE;
    PartDims d = part_dims(n_total, nranks, rank, max_txs);
    std::lock_guard<std::mutex> g(c->smu);
    HIPCHK(hipSetDevice(c->device));
    Shape* s;
    rc = shape_get(c, SK_PARTITION,
                   partition_key(h_off, d.n, n_total, nranks, rank, chain_id, chain_id_len, signer_kind, max_txs),
                   [&](Shape& ns, Layout& L) {
                       return partition_shape(c, ns, h_off, n_total, nranks, rank, chain_id, chain_id_len,
                                              signer_kind, max_txs, L);
                   },
                   &s);
    if (rc) return rc;
    return d.n ? shape_side_init(c, *s) : GSV_SUCCESS;
}

int gsv_notary_partition_pack_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n_total,
                                  int nranks, int rank, const uint8_t* chain_id, size_t chain_id_len, int signer_kind,
                                  uint32_t max_txs, uint8_t* d_block, uint8_t* d_senders, uint8_t* d_status,
                                  void* stream) {
    if (!c || !h_off || !d_block || nranks < 1 || rank < 0 || rank >= nranks) return GSV_E_INVALID_ARG;
    int rc = notary_args(chain_id, chain_id_len, signer_kind, n_total, max_txs);
    if (rc) return rc;
    PartDims d = part_dims(n_total, nranks, rank, max_txs);
    if (d.n && !d_bodies) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->smu);
    Shape* s = shape_find(c, SK_PARTITION,
                          partition_key(h_off, d.n, n_total, nranks, rank, chain_id, chain_id_len, signer_kind, max_txs));
    if (!s) return GSV_E_NOT_PREPARED;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return shape_run(c, *s, st, [&] { return partition_pack(c, *s, d, d_bodies, d_senders, d_status, d_block, st); });
}

int gsv_notary_partition_unpack_dev(gsv_ctx* c, const uint8_t* d_blocks, size_t n_total, int nranks, uint32_t max_txs,
                                    uint8_t* d_root32_all, uint32_t* d_ntx_all, uint8_t* d_bitmap_all,
                                    int32_t* d_rank_status, void* stream) {
    if (!c || !d_blocks || nranks < 1 || max_txs == 0 || (n_total && (!d_root32_all || !d_ntx_all || !d_bitmap_all)))
        return GSV_E_INVALID_ARG;
    if (n_total > 0xFFFFFFFFull / 4096) return GSV_E_TOO_LARGE;
    PartDims d = part_dims(n_total, nranks, 0, max_txs);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return hip_err(gsv::launch_partition_unpack(d_blocks, (uint32_t)nranks, (uint32_t)n_total, (uint32_t)d.R,
                                                (uint32_t)d.bm, d.B, d_root32_all, d_ntx_all, d_bitmap_all,
                                                d_rank_status, st));
}

int gsv_notary_validate_partition_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n_total,
                                      const uint8_t* chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                                      uint8_t* d_root32_all, uint32_t* d_ntx_all, uint8_t* d_bitmap_all,
                                      uint8_t* d_senders, uint8_t* d_status, int32_t* d_rank_status, void* stream) {
    // arguments every rank passes alike: an error here is the same error on every rank, and no rank
    // enters the collective
    if (!c || (n_total && (!d_root32_all || !d_ntx_all || !d_bitmap_all))) return GSV_E_INVALID_ARG;
    int rc = notary_args(chain_id, chain_id_len, signer_kind, n_total, max_txs);
    if (rc || n_total == 0) return rc;
    if (n_total > 0xFFFFFFFFull / 4096) return GSV_E_TOO_LARGE;
    const int N = c->nranks, r = c->rank;
    PartDims d = part_dims(n_total, N, r, max_txs);
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    // rank-local failures still reach the all-gather with the rank's status in its block header
    int lrc = (!h_off || (d.n && !d_bodies)) ? GSV_E_INVALID_ARG : GSV_SUCCESS;
    bool joined = false;  // this rank has entered the all-gather
    if (!lrc) {
        std::lock_guard<std::mutex> g(c->smu);
        Shape* s = shape_find(c, SK_PARTITION, partition_key(h_off, d.n, n_total, N, r, chain_id, chain_id_len,
                                                             signer_kind, max_txs));
        if (!s) lrc = GSV_E_NOT_PREPARED;
        else if (hipSetDevice(c->device) != hipSuccess) lrc = GSV_E_HIP;
        else {
            lrc = shape_run(c, *s, st, [&] {
                uint8_t* blk = s->at<uint8_t>(s->o_block);
                uint8_t* all = s->at<uint8_t>(s->o_all);
                int e = partition_pack(c, *s, d, d_bodies, d_senders, d_status, blk, st);
                if (e) return e;
                joined = true;
                e = partition_gather(c, blk, all, d, st);
                if (e) return e;
                return hip_err(gsv::launch_partition_unpack(all, (uint32_t)N, (uint32_t)n_total, (uint32_t)d.R,
                                                            (uint32_t)d.bm, d.B, d_root32_all, d_ntx_all,
                                                            d_bitmap_all, d_rank_status, st));
            });
            if (!lrc || joined) return lrc;  // done, or failed at/after the collective: nothing more to join
        }
    }
    // error path: join the collective from the staging arena with this rank's status and no records
    std::lock_guard<std::mutex> g(c->mu);
    if (hipSetDevice(c->device) != hipSuccess) return lrc;
    if (arena_reserve(c, al(d.B) + al((size_t)N * d.B))) return lrc;
    uint8_t* blk = c->arena;
    uint8_t* all = c->arena + al(d.B);
    if (gsv::launch_partition_pack(nullptr, nullptr, nullptr, 0, (uint32_t)d.per, (uint32_t)d.R, (uint32_t)d.bm, lrc,
                                   blk, st) != hipSuccess)
        return lrc;
    if (partition_gather(c, blk, all, d, st)) return lrc;
    gsv::launch_partition_unpack(all, (uint32_t)N, (uint32_t)n_total, (uint32_t)d.R, (uint32_t)d.bm, d.B,
                                 d_root32_all, d_ntx_all, d_bitmap_all, d_rank_status, st);
    hipStreamSynchronize(st);  // the arena is reused by the next host-path call
    return lrc;
}

int gsv_notary_validate_partition(gsv_ctx* c, const uint8_t* bodies, const uint64_t* off, size_t n_total,
                                  const uint8_t* chain_id, size_t chain_id_len, int signer_kind, uint32_t max_txs,
                                  uint8_t* root32_all, uint32_t* ntx_all, uint8_t* bitmap_all,
                                  uint8_t* senders_out, uint8_t* status_out) {
    // arguments every rank passes alike (see the _dev form)
    if (!c || !off || (n_total && (!root32_all || !ntx_all || !bitmap_all))) return GSV_E_INVALID_ARG;
    int rc = notary_args(chain_id, chain_id_len, signer_kind, n_total, max_txs);
    if (rc || n_total == 0) return rc;
    if (n_total > 0xFFFFFFFFull / 4096) return GSV_E_TOO_LARGE;
    const int N = c->nranks, r = c->rank;
    PartDims d = part_dims(n_total, N, r, max_txs);
    const size_t n = d.n, nt = n * (size_t)max_txs;
    std::lock_guard<std::mutex> g(c->mu);
    std::lock_guard<std::mutex> g2(c->smu);
    HIPCHK(hipSetDevice(c->device));
    hipStream_t sm = c->stream;
    // gathered outputs + statuses first in the arena, so the error path finds them at the same place
    const size_t out_bytes = al(d.B) + al((size_t)N * d.B) + al(n_total * 32) + al(n_total * 4) +
                             al(n_total * d.bm) + al((size_t)N * 4);
    int lrc = (n && !bodies) ? GSV_E_INVALID_ARG : GSV_SUCCESS;
    for (size_t i = 0; i < n && !lrc; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > MAX_BODY) lrc = GSV_E_TOO_LARGE;
    std::vector<uint64_t> st, en;
    uint64_t pos = n ? stage_offsets(off, n, st, en) : 0;
    size_t staged = out_bytes + al(pos + 16) + al(n * 32 + 1) + al(n * 4 + 1) + al(n * d.bm + 1) + al(nt * 20 + 1) +
                    al(nt + 1);
    Shape s;
    if (!lrc) {
        lrc = shape_temp(c, staged,
                         [&](Shape& ns, Layout& L) {
                             if (!n) return GSV_SUCCESS;
                             return notary_shape(c, ns, st.data(), en.data(), n, chain_id, chain_id_len, signer_kind,
                                                 max_txs, L);
                         },
                         s);
        if (!lrc && n) lrc = shape_side_borrow(c, s);
    }
    if (lrc && arena_reserve(c, out_bytes)) return lrc;  // cannot even join the collective
    Carve cv(c->arena);
    uint8_t* d_blk = cv.take<uint8_t>(d.B);
    uint8_t* d_all = cv.take<uint8_t>((size_t)N * d.B);
    uint8_t* d_oroot = cv.take<uint8_t>(n_total * 32);
    uint32_t* d_ontx = cv.take<uint32_t>(n_total * 4);
    uint8_t* d_obm = cv.take<uint8_t>(n_total * d.bm);
    int32_t* d_rst = cv.take<int32_t>((size_t)N * 4);
    uint8_t* d_snd = nullptr;
    uint8_t* d_st = nullptr;
    if (!lrc) {
        uint8_t* d_b = cv.take<uint8_t>(pos + 16);
        uint8_t* d_r = cv.take<uint8_t>(n * 32 + 1);
        uint32_t* d_n = cv.take<uint32_t>(n * 4 + 1);
        uint8_t* d_bm = cv.take<uint8_t>(n * d.bm + 1);
        d_snd = cv.take<uint8_t>(nt * 20 + 1);
        d_st = cv.take<uint8_t>(nt + 1);
        if (n) lrc = stage_bodies(c, d_b, bodies, off, n, st, en);
        if (!lrc && n)
            lrc = shape_run(c, s, sm, [&] {
                return notary_run(c, s, n, d_b, d_r, d_n, d_bm, senders_out ? d_snd : nullptr,
                                  status_out ? d_st : nullptr, sm);
            });
        if (!lrc)
            lrc = hip_err(gsv::launch_partition_pack(d_r, d_n, d_bm, (uint32_t)n, (uint32_t)d.per, (uint32_t)d.R,
                                                     (uint32_t)d.bm, 0, d_blk, sm));
    }
    if (lrc && gsv::launch_partition_pack(nullptr, nullptr, nullptr, 0, (uint32_t)d.per, (uint32_t)d.R,
                                          (uint32_t)d.bm, lrc, d_blk, sm) != hipSuccess)
        return lrc;
    int grc = partition_gather(c, d_blk, d_all, d, sm);
    if (grc) return grc;
    HIPCHK(gsv::launch_partition_unpack(d_all, (uint32_t)N, (uint32_t)n_total, (uint32_t)d.R, (uint32_t)d.bm, d.B,
                                        d_oroot, d_ontx, d_obm, d_rst, sm));
    std::vector<int32_t> rst(N);
    HIPCHK(hipMemcpyAsync(root32_all, d_oroot, n_total * 32, hipMemcpyDeviceToHost, sm));
    HIPCHK(hipMemcpyAsync(ntx_all, d_ontx, n_total * 4, hipMemcpyDeviceToHost, sm));
    HIPCHK(hipMemcpyAsync(bitmap_all, d_obm, n_total * d.bm, hipMemcpyDeviceToHost, sm));
    HIPCHK(hipMemcpyAsync(rst.data(), d_rst, (size_t)N * 4, hipMemcpyDeviceToHost, sm));
    if (!lrc && n && senders_out) HIPCHK(hipMemcpyAsync(senders_out, d_snd, nt * 20, hipMemcpyDeviceToHost, sm));
    if (!lrc && n && status_out) HIPCHK(hipMemcpyAsync(status_out, d_st, nt, hipMemcpyDeviceToHost, sm));
    HIPCHK(hipStreamSynchronize(sm));
    // every rank returns the same verdict: the status of the lowest failing rank
    for (int q = 0; q < N; q++)
        if (rst[q]) return rst[q];
    for (size_t i = 0; i < n_total; i++)
        if (ntx_all[i] > max_txs) return GSV_E_TOO_LARGE;
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ DeriveSha over any DerivableList
static int derive_args(const uint64_t* voff, const uint64_t* list_off, size_t n) {
    if (list_off[n] < list_off[0]) return GSV_E_INVALID_ARG;
    for (size_t i = 0; i < n; i++)
        if (list_off[i + 1] < list_off[i]) return GSV_E_INVALID_ARG;
    return GSV_SUCCESS;
}

int gsv_derive_sha_prepare(gsv_ctx* c, const uint64_t* voff, const uint64_t* list_off, size_t n) {
    if (!c || (n && (!voff || !list_off))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    int rc = derive_args(voff, list_off, n);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(c->smu);
    HIPCHK(hipSetDevice(c->device));
    Shape* s;
    return shape_get(c, SK_DERIVE, derive_key(voff, list_off, n),
                     [&](Shape& ns, Layout& L) { return derive_shape(c, ns, voff, list_off, n, L); }, &s);
}

int gsv_derive_sha_batch_dev(gsv_ctx* c, const uint8_t* d_vals, const uint64_t* voff, const uint64_t* list_off,
                             size_t n, uint8_t* d_root32_out, void* stream) {
    if (!c || (n && (!voff || !list_off || !d_root32_out))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    int rc = derive_args(voff, list_off, n);
    if (rc) return rc;
    if (list_off[n] > list_off[0] && !d_vals) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->smu);
    Shape* s = shape_find(c, SK_DERIVE, derive_key(voff, list_off, n));
    if (!s) return GSV_E_NOT_PREPARED;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return shape_run(c, *s, st, [&] { return derive_run(c, *s, d_vals, d_root32_out, st); });
}

int gsv_derive_sha_batch(gsv_ctx* c, const uint8_t* vals, const uint64_t* voff, const uint64_t* list_off, size_t n,
                         uint8_t* root32_out) {
    if (!c || (n && (!voff || !list_off || !root32_out))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    int rc = derive_args(voff, list_off, n);
    if (rc) return rc;
    uint64_t v0 = voff[list_off[0]], v1 = voff[list_off[n]];
    if (v1 < v0 || (v1 > v0 && !vals)) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    std::lock_guard<std::mutex> g2(c->smu);
    HIPCHK(hipSetDevice(c->device));
    // stage the values (rebased so item list_off[0] starts at 0)
    std::vector<uint64_t> rv(list_off[n] + 1, 0);
    for (uint64_t k = list_off[0]; k <= list_off[n]; k++) rv[k] = voff[k] - v0;
    size_t staged = al(v1 - v0 + 16) + al(n * 32);
    Shape s;
    rc = shape_temp(c, staged, [&](Shape& ns, Layout& L) { return derive_shape(c, ns, rv.data(), list_off, n, L); },
                    s);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_v = cv.take<uint8_t>(v1 - v0 + 16);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    if (v1 > v0) HIPCHK(hipMemcpyAsync(d_v, vals + v0, v1 - v0, hipMemcpyHostToDevice, c->stream));
    rc = shape_run(c, s, c->stream, [&] { return derive_run(c, s, d_v, d_r, c->stream); });
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(root32_out, d_r, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ Proof of Custody
int gsv_collation_poc_prepare(gsv_ctx* c, const uint64_t* h_off, size_t n, const uint8_t* salt, size_t salt_len) {
    if (!c || (n && !h_off) || (salt_len && !salt)) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->smu);
    HIPCHK(hipSetDevice(c->device));
    Shape* s;
    return shape_get(c, SK_POC, poc_key(h_off, n, salt, salt_len),
                     [&](Shape& ns, Layout& L) { return poc_shape(c, ns, h_off, h_off + 1, n, salt, salt_len, L); },
                     &s);
}

int gsv_collation_poc_batch_dev(gsv_ctx* c, const uint8_t* d_bodies, const uint64_t* h_off, size_t n,
                                const uint8_t* salt, size_t salt_len, uint8_t* d_poc32_out, void* stream) {
    if (!c || (n && (!h_off || !d_poc32_out)) || (salt_len && !salt)) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    std::lock_guard<std::mutex> g(c->smu);
    Shape* s = shape_find(c, SK_POC, poc_key(h_off, n, salt, salt_len));
    if (!s) return GSV_E_NOT_PREPARED;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return shape_run(c, *s, st, [&] { return poc_run(c, *s, n, d_bodies, d_poc32_out, st); });
}

int gsv_collation_poc_batch(gsv_ctx* c, const uint8_t* bodies, const uint64_t* off, size_t n, const uint8_t* salt,
                            size_t salt_len, uint8_t* poc32_out) {
    if (!c || (n && (!off || !poc32_out)) || (salt_len && !salt)) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > MAX_POC) return GSV_E_TOO_LARGE;
    if (off[n] > off[0] && !bodies) return GSV_E_INVALID_ARG;
    std::lock_guard<std::mutex> g(c->mu);
    std::lock_guard<std::mutex> g2(c->smu);
    HIPCHK(hipSetDevice(c->device));
    std::vector<uint64_t> st, en;
    uint64_t pos = stage_offsets(off, n, st, en);
    size_t staged = al(pos + 16) + al(n * 32);
    Shape s;
    int rc = shape_temp(c, staged,
                        [&](Shape& ns, Layout& L) {
                            return poc_shape(c, ns, st.data(), en.data(), n, salt, salt_len, L);
                        },
                        s);
    if (rc) return rc;
    Carve cv(c->arena);
    uint8_t* d_b = cv.take<uint8_t>(pos + 16);
    uint8_t* d_r = cv.take<uint8_t>(n * 32);
    rc = stage_bodies(c, d_b, bodies, off, n, st, en);
    if (rc) return rc;
    rc = shape_run(c, s, c->stream, [&] { return poc_run(c, s, n, d_b, d_r, c->stream); });
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(poc32_out, d_r, n * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GSV_SUCCESS;
}

// ------------------------------------------------------------------ collation header + proposer signature
int gsv_collation_header_prepare(gsv_ctx* c, size_t n) {
    if (!c) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > (1u << 30)) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->smu);
    HIPCHK(hipSetDevice(c->device));
    Shape* s;
    return shape_get(c, SK_HEADER, std::vector<uint64_t>{n},
                     [&](Shape& ns, Layout& L) { return header_shape(c, ns, n, L); }, &s);
}

int gsv_collation_header_verify_batch_dev(gsv_ctx* c, const uint8_t* d_sid, const uint8_t* d_root,
                                          const uint8_t* d_per, const uint8_t* d_prop, const uint8_t* d_sig,
                                          const uint8_t* d_nil, size_t n, uint8_t* d_hash, uint8_t* d_signer,
                                          uint8_t* d_st, void* stream) {
    if (!c || (n && (!d_sid || !d_root || !d_per || !d_prop || !d_sig || !d_st))) return GSV_E_INVALID_ARG;
    if (n == 0) return GSV_SUCCESS;
    if (n > (1u << 30)) return GSV_E_TOO_LARGE;
    std::lock_guard<std::mutex> g(c->smu);
    Shape* s = shape_find(c, SK_HEADER, std::vector<uint64_t>{n});
    if (!s) return GSV_E_NOT_PREPARED;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return shape_run(c, *s, st, [&] {
        KTimer t(c, GSV_K_HEADER, st);
        return hip_err(gsv::launch_header_verify(d_sid, d_root, d_per, d_prop, d_sig, d_nil, (uint32_t)n, c->gtab,
                                                 s->at<uint8_t>(s->o_hscr), d_hash, d_signer, d_st, st));
    });
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
