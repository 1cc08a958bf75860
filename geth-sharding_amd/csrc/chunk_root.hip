// Chunk root (DeriveSha over body bytes) on gfx950 — see chunk_root.h for the design.
//
// Restated semantics:
//   core/types/derive_sha.go:32-41   key_i = rlp(uint(i)), value_i = Chunks.GetRlp(i) = rlp(body[i])
//   trie/trie.go:218-286             insert: short (leaf/extension) and full (branch) nodes
//   trie/hasher.go:56-212            post-order hashing, RLP < 32 bytes inlined, root forced
//   trie/encoding.go:37-75           hexToCompact (flag 2 = leaf, +1 odd) and keybytesToHex
//   trie/trie.go:471-478             empty trie -> emptyRoot (handled by the host)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <utility>

#include "chunk_root.h"
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {

// ================================================================ key helpers (host + device)
// nibbles of keybytesToHex(rlp(uint(i))) including the terminator 16
__host__ __device__ inline int key_nbytes(uint32_t i) {
    return i < 128 ? 1 : i < 256 ? 2 : i < 65536 ? 3 : i < (1u << 24) ? 4 : 5;  // i == 0 -> [0x80] (1 byte)
}
__host__ __device__ inline uint8_t key_byte(uint32_t i, int b) {
    int nb = key_nbytes(i);
    if (nb == 1) return i == 0 ? 0x80 : (uint8_t)i;
    if (b == 0) return (uint8_t)(0x80 + nb - 1);
    return (uint8_t)(i >> (8 * (nb - 1 - b)));
}
__host__ __device__ inline int key_len(uint32_t i) { return 2 * key_nbytes(i) + 1; }
__host__ __device__ inline uint8_t key_nib(uint32_t i, int d) {
    int nb = key_nbytes(i);
    if (d >= 2 * nb) return 16;
    uint8_t by = key_byte(i, d >> 1);
    return (d & 1) ? (by & 15) : (by >> 4);
}

// ================================================================ host plan builder
namespace {

struct Builder {
    uint32_t N;
    uint32_t nB;  // keys 1..127 present (they sort first)
    bool generic = false;
    std::vector<uint16_t>* leaf_depth = nullptr;  // generic: depth per body index
    std::vector<PNode> nodes;
    std::vector<std::vector<PChild>> kids;

    uint32_t ipos(uint32_t p) const {
        if (p < nB) return 1 + p;
        p -= nB;
        return p == 0 ? 0u : 127u + p;
    }

    struct Res {
        bool leaf;
        uint32_t i;      // leaf body index
        uint16_t depth;  // leaf remainder start
        int node;        // node id
        int height;
    };

    int new_node(uint8_t kind) {
        PNode n{};
        n.kind = kind;
        n.msg_off = -1;
        n.parent_msg = -1;
        n.ref_slot = -1;
        n.child_begin = -1;
        nodes.push_back(n);
        kids.emplace_back();
        return (int)nodes.size() - 1;
    }

    Res build(uint32_t lo, uint32_t hi, int depth) {
        if (hi - lo == 1) {
            if (generic) (*leaf_depth)[ipos(lo)] = (uint16_t)depth;
            return Res{true, ipos(lo), (uint16_t)depth, -1, 0};
        }
        uint32_t fi = ipos(lo), la = ipos(hi - 1);
        int cp = depth;
        while (key_nib(fi, cp) == key_nib(la, cp)) cp++;
        if (cp > depth) {
            Res c = build(lo, hi, cp);
            int id = new_node(PK_EXT);
            nodes[id].first_i = fi;
            nodes[id].depth = (uint16_t)depth;
            nodes[id].ext_end = (uint16_t)cp;
            nodes[id].height = (uint8_t)(c.height + 1);
            kids[id].push_back(PChild{0, PC_NODE, 0, (uint32_t)c.node});
            return Res{false, 0, 0, id, c.height + 1};
        }
        // branch at `depth`: partition [lo, hi) by nibble (monotone in sorted order)
        uint32_t starts[17];
        uint8_t vals[16];
        int nch = 0;
        uint32_t s = lo;
        while (s < hi) {
            uint8_t v = key_nib(ipos(s), depth);
            uint32_t a = s + 1, b = hi;  // first position with nibble > v
            while (a < b) {
                uint32_t m = a + (b - a) / 2;
                if (key_nib(ipos(m), depth) > v) b = m;
                else a = m + 1;
            }
            starts[nch] = s;
            vals[nch] = v;
            nch++;
            s = a;
        }
        starts[nch] = hi;
        // full bottom branch: 16 single keys whose remainder after this nibble is the terminator
        if (!generic && nch == 16 && hi - lo == 16) {
            bool bottom = true;
            for (uint32_t p = lo; p < hi && bottom; p++) bottom = key_len(ipos(p)) - 1 == depth + 1;
            if (bottom) {
                int id = new_node(PK_BOTTOM);
                nodes[id].first_i = fi;
                nodes[id].depth = (uint16_t)depth;
                nodes[id].height = 1;
                return Res{false, 0, 0, id, 1};
            }
        }
        std::vector<PChild> ch;
        int h = 0;
        bool all_hashed_full = !generic && (nch == 16);
        for (int c = 0; c < nch; c++) {
            Res r = build(starts[c], starts[c + 1], depth + 1);
            if (r.leaf) {
                ch.push_back(PChild{vals[c], PC_LEAF, r.depth, r.i});
                all_hashed_full = false;
            } else {
                ch.push_back(PChild{vals[c], PC_NODE, 0, (uint32_t)r.node});
                uint8_t k = nodes[r.node].kind;
                if (k != PK_BOTTOM && k != PK_HFULL) all_hashed_full = false;
            }
            h = std::max(h, r.height);
        }
        int id = new_node(all_hashed_full ? PK_HFULL : PK_BRANCH);
        nodes[id].first_i = fi;
        nodes[id].depth = (uint16_t)depth;
        nodes[id].height = (uint8_t)(h + 1);
        kids[id] = std::move(ch);
        return Res{false, 0, 0, id, h + 1};
    }
};

}  // namespace

void build_trie_plan(TriePlanHost& p, uint32_t N, bool generic) {
    p = TriePlanHost();
    p.N = N;
    p.generic = generic;
    if (N == 0) return;
    Builder b;
    b.N = N;
    b.nB = N > 128 ? 127 : N - 1;
    b.generic = generic;
    if (generic) {
        p.leaf_depth.assign(N, 0);
        b.leaf_depth = &p.leaf_depth;
    }
    Builder::Res r = b.build(0, N, 0);
    if (generic && r.leaf) return;  // N == 1: k_derive_leaf hashes the lone leaf as the root
    int root;
    if (r.leaf) {  // N == 1: a single leaf is the root
        root = b.new_node(PK_LEAF);
        b.nodes[root].first_i = r.i;
        b.nodes[root].depth = r.depth;
        b.nodes[root].height = 1;
    } else {
        root = r.node;
    }
    b.nodes[root].is_root = 1;
    // an HFULL root still has to produce the root hash (no parent message): fine, handled in-kernel
    // order: by height; inside a height BOTTOM, then HFULL, then generic nodes
    int M = (int)b.nodes.size();
    std::vector<int> order(M);
    for (int i = 0; i < M; i++) order[i] = i;
    auto rank = [](uint8_t k) { return k == PK_BOTTOM ? 0 : k == PK_HFULL ? 1 : 2; };
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
        const PNode &a = b.nodes[x], &c = b.nodes[y];
        if (a.height != c.height) return a.height < c.height;
        return rank(a.kind) < rank(c.kind);
    });
    std::vector<int> newid(M);
    for (int i = 0; i < M; i++) newid[order[i]] = i;
    p.nodes.resize(M);
    int nmsg = 0;
    for (int i = 0; i < M; i++) {
        int o = order[i];
        PNode n = b.nodes[o];
        n.ref_slot = i;
        if (n.kind != PK_BOTTOM) n.msg_off = (nmsg++) * MSG_STRIDE;
        const auto& kv = b.kids[o];
        if (!kv.empty() && n.kind != PK_HFULL) {
            n.child_begin = (int)p.children.size();
            n.nchild = (uint8_t)kv.size();
            for (auto c : kv) {
                if (c.type == PC_NODE) c.idx = (uint32_t)newid[c.idx];
                p.children.push_back(c);
            }
        }
        p.nodes[i] = n;
    }
    // HFULL parents: children store their raw 32-byte hash at 32 * slot of the parent's buffer
    for (int i = 0; i < M; i++) {
        int o = order[i];
        if (b.nodes[o].kind != PK_HFULL) continue;
        for (auto& c : b.kids[o]) p.nodes[newid[c.idx]].parent_msg = p.nodes[i].msg_off + 32 * c.slot;
    }
    p.root = newid[root];
    p.n_msg = nmsg;
    p.n_slots = M;
    p.height = p.nodes.back().height;
    p.lvl_bottom_begin.assign(p.height, 0);
    p.lvl_bottom_end.assign(p.height, 0);
    p.lvl_hfull_begin.assign(p.height, 0);
    p.lvl_hfull_end.assign(p.height, 0);
    p.lvl_gen_begin.assign(p.height, 0);
    p.lvl_gen_end.assign(p.height, 0);
    for (int i = M - 1; i >= 0; i--) {  // nodes are sorted: the first index seen last wins
        int h = p.nodes[i].height - 1;
        uint8_t k = p.nodes[i].kind;
        std::vector<int>& bg = k == PK_BOTTOM ? p.lvl_bottom_begin : k == PK_HFULL ? p.lvl_hfull_begin : p.lvl_gen_begin;
        std::vector<int>& en = k == PK_BOTTOM ? p.lvl_bottom_end : k == PK_HFULL ? p.lvl_hfull_end : p.lvl_gen_end;
        if (en[h] == 0) en[h] = i + 1;
        bg[h] = i;
    }
    // the top of the trie (few nodes per height, no BOTTOM) runs as one fused launch: one
    // workgroup per body walks those heights with barriers instead of one launch per height
    p.top_h = p.height + 1;
    for (int h = p.height; h >= 1; h--) {
        int nb = p.lvl_bottom_end[h - 1] - p.lvl_bottom_begin[h - 1];
        int nf = p.lvl_hfull_end[h - 1] - p.lvl_hfull_begin[h - 1];
        int ng = p.lvl_gen_end[h - 1] - p.lvl_gen_begin[h - 1];
        if (nb || nf > TOP_MAX_HFULL || ng > TOP_MAX_GEN) break;
        p.top_h = h;
    }
}

TriePlan::~TriePlan() {
    if (d_nodes) (void)hipFree(d_nodes);
    if (d_children) (void)hipFree(d_children);
    if (d_leaf_depth) (void)hipFree(d_leaf_depth);
}

template <typename T>
static bool upload(T** dst, const std::vector<T>& src) {
    if (src.empty()) return true;
    size_t nb = src.size() * sizeof(T);
    if (hipMalloc(dst, nb) != hipSuccess) {
        *dst = nullptr;
        return false;
    }
    return hipMemcpy(*dst, src.data(), nb, hipMemcpyHostToDevice) == hipSuccess;
}

std::shared_ptr<TriePlan> PlanCache::get(uint32_t N, bool generic) {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t key = (uint64_t)N | (generic ? (1ull << 32) : 0ull);
    auto it = plans_.find(key);
    if (it != plans_.end()) {
        it->second.last_use = ++tick_;
        return it->second.plan;
    }
    auto pl = std::make_shared<TriePlan>();
    build_trie_plan(pl->h, N, generic);
    // a failed upload returns nullptr; the destructor frees whatever was allocated
    if (!upload(&pl->d_leaf_depth, pl->h.leaf_depth) || !upload(&pl->d_nodes, pl->h.nodes) ||
        !upload(&pl->d_children, pl->h.children))
        return nullptr;
    pl->bytes = 2 * (pl->h.leaf_depth.size() * sizeof(uint16_t) + pl->h.nodes.size() * sizeof(PNode) +
                     pl->h.children.size() * sizeof(PChild));
    bytes_ += pl->bytes;
    plans_[key] = Entry{pl, ++tick_};
    // evict least-recently-used plans nobody else holds
    while (bytes_ > kMaxBytes) {
        auto victim = plans_.end();
        for (auto e = plans_.begin(); e != plans_.end(); ++e)
            if (e->first != key && e->second.plan.use_count() == 1 &&
                (victim == plans_.end() || e->second.last_use < victim->second.last_use))
                victim = e;
        if (victim == plans_.end()) break;
        bytes_ -= victim->second.plan->bytes;
        plans_.erase(victim);
    }
    return pl;
}

// ================================================================ device side
struct BodyBatch {
    const uint8_t* bodies;     // base of all bodies
    const uint64_t* body_off;  // per body start offset (device)
    uint8_t* msg;              // msg arena base; body b at msg + b * msg_stride
    uint8_t* refs;             // ref arena base; body b at refs + b * ref_stride
    uint8_t* roots;            // 32 B per body
    uint64_t msg_stride, ref_stride;
    uint32_t nbodies;
    // generic DeriveSha: leaf j of list b has its reference at leafrefs + (leaf_base[b] + j) * REF_STRIDE
    const uint8_t* leafrefs;
    const uint64_t* leaf_base;
    int generic;
};

// Keccak-256 of len bytes at p (8-byte aligned, global or LDS; bytes past len may be garbage)
GSV_DI void keccak_buf(uint32_t h[8], const uint8_t* p, uint32_t len) {
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    const uint64_t* q = (const uint64_t*)p;
    while (len >= 136) {
#pragma unroll
        for (int k = 0; k < 17; k++) a[k] ^= q[k];
        keccakf(a);
        q += 17;
        len -= 136;
    }
#pragma unroll
    for (int k = 0; k < 17; k++) {
        int32_t avail = (int32_t)len - 8 * k;
        uint64_t w = 0;
        if (avail >= 8) w = q[k];
        else if (avail > 0) w = q[k] & ((1ull << (8 * avail)) - 1ull);
        if ((uint32_t)(len >> 3) == (uint32_t)k) w ^= 0x01ull << (8 * (len & 7u));
        if (k == 16) w ^= 0x8000000000000000ULL;
        a[k] ^= w;
    }
    keccakf_digest(a);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        h[2 * k] = (uint32_t)a[k];
        h[2 * k + 1] = (uint32_t)(a[k] >> 32);
    }
}

// raw 32-byte hash to a 16-byte aligned destination (two dwordx4 stores)
GSV_DI void store_hash32(uint8_t* dst, const uint32_t h[8]) {
    uint4* d = (uint4*)dst;
    d[0] = make_uint4(h[0], h[1], h[2], h[3]);
    d[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

// canonical ref slot (16-byte aligned): s[0] = 33, s[8 .. 41) = a0 || hash
GSV_DI void store_hashref_slot(uint8_t* s, const uint32_t h[8]) {
    uint32_t w[12];
    w[0] = 33;
    w[1] = 0;
    w[2] = 0xa0u | (h[0] << 8);
#pragma unroll
    for (int k = 1; k < 8; k++) w[2 + k] = (h[k - 1] >> 24) | (h[k] << 8);
    w[10] = h[7] >> 24;
    w[11] = 0;
    uint4* d = (uint4*)s;
    d[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d[1] = make_uint4(w[4], w[5], w[6], w[7]);
    d[2] = make_uint4(w[8], w[9], w[10], w[11]);
}

// deliver a hashed node's reference (root output / HFULL parent's hash slot / canonical slot)
GSV_DI void emit_hash(const PNode& nd, const BodyBatch& bb, uint32_t body, const uint32_t h[8]) {
    if (nd.is_root) {
        store_hash32(bb.roots + (size_t)body * 32, h);
    } else if (nd.parent_msg >= 0) {
        store_hash32(bb.msg + (size_t)body * bb.msg_stride + nd.parent_msg, h);
    } else {
        store_hashref_slot(bb.refs + (size_t)body * bb.ref_stride + (size_t)nd.ref_slot * REF_STRIDE, h);
    }
}

// ---------------------------------------------------------------- BOTTOM: 16 leaf children
// leaf j = [0x20, rlp(b)]: b == 0 -> c3 20 81 80; b < 128 -> c2 20 b; else c4 20 82 81 b
constexpr int BOT_BLOCK = 256;
// a lane's message buffer stride in LDS (bytes, a multiple of 8, >= 88): 96 = 24 words put the 64
// lanes of a wave on 4 of the 32 banks (8-way conflicts for the 64-bit accesses); 88 (22 words) spreads
// them over 16.  r05: bottom level 0.80 vs 0.82 ms, configs[2] equal within noise
// (profiles/r05/ab/bottom_lds_stride.txt).
constexpr int BOT_BUF = 88;
static_assert(BOT_BUF % 8 == 0 && BOT_BUF >= 88, "the 88-byte window, 8-byte aligned");

// m: this lane's BOT_BUF-byte LDS buffer (8-byte aligned)
GSV_DI void do_bottom(const PNode& nd, const BodyBatch& bb, uint32_t body, uint8_t* m) {
    const uint8_t* src = bb.bodies + bb.body_off[body] + nd.first_i;
    uint8_t v[16];
    if ((((uintptr_t)src) & 15u) == 0) {
        uint4 w = *(const uint4*)src;
        uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = (uint8_t)(ws[j >> 2] >> (8 * (j & 3)));
    } else {
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = src[j];
    }
    uint32_t payload = 1;  // trailing empty value slot 0x80
#pragma unroll
    for (int j = 0; j < 16; j++) payload += v[j] == 0 ? 4u : v[j] < 128 ? 3u : 5u;
    // the 88-byte window zeroed by eleven 64-bit stores up front (no per-byte tail loop), the sponge's
    // 0x01 pad byte stored after the message instead of XOR-ed into the loaded word by lane compares
    {
        uint64_t* mz = (uint64_t*)m;
#pragma unroll
        for (int k = 0; k < 11; k++) mz[k] = 0;
    }
    uint32_t o = 0;
    if (payload < 56) {
        m[o++] = (uint8_t)(0xc0 + payload);
    } else {
        m[o++] = 0xf8;
        m[o++] = (uint8_t)payload;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint8_t b = v[j];
        if (b == 0) {
            m[o] = 0xc3; m[o + 1] = 0x20; m[o + 2] = 0x81; m[o + 3] = 0x80;
            o += 4;
        } else if (b < 128) {
            m[o] = 0xc2; m[o + 1] = 0x20; m[o + 2] = b;
            o += 3;
        } else {
            m[o] = 0xc4; m[o + 1] = 0x20; m[o + 2] = 0x82; m[o + 3] = 0x81; m[o + 4] = b;
            o += 5;
        }
    }
    m[o++] = 0x80;
    m[o] = 0x01;  // single block: len <= 83 < 136
    uint64_t a[25];
    const uint64_t* q = (const uint64_t*)m;
#pragma unroll
    for (int k = 0; k < 11; k++) a[k] = q[k];
#pragma unroll
    for (int k = 11; k < 25; k++) a[k] = 0;
    a[16] ^= 0x8000000000000000ULL;
    keccakf_digest(a);
    uint32_t h[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        h[2 * k] = (uint32_t)a[k];
        h[2 * k + 1] = (uint32_t)(a[k] >> 32);
    }
    emit_hash(nd, bb, body, h);
}

// ---------------------------------------------------------------- HFULL: 16 hashed children
constexpr int HF_LEN = 532;
constexpr bool hf_is_const(int p) { return p < 3 || p >= HF_LEN - 1 || (p - 3) % 33 == 0; }
constexpr uint32_t hf_const(int p) {
    return p == 0 ? 0xf9u : p == 1 ? 0x02u : p == 2 ? 0x11u : p == HF_LEN - 1 ? 0x80u : p >= HF_LEN ? 0u : 0xa0u;
}
constexpr int hf_slot(int p) { return (p - 3) / 33; }
constexpr int hf_idx(int p) { return (p - 3) % 33 - 1; }
// child-hash slots touched by block B (136 bytes at 136 * B)
constexpr int hf_s0(int B) { return B == 0 ? 0 : hf_slot(136 * B); }
constexpr int hf_s1(int B) { return hf_slot(136 * B + 135 < HF_LEN - 2 ? 136 * B + 135 : HF_LEN - 2); }

template <int B, int P>
GSV_DI uint32_t hf_byte(const uint32_t* win) {
    constexpr int p = 136 * B + P;
    if constexpr (hf_is_const(p)) {
        return hf_const(p);
    } else {
        constexpr int s = hf_slot(p) - hf_s0(B), j = hf_idx(p);
        return (win[s * 8 + (j >> 2)] >> (8 * (j & 3))) & 0xffu;
    }
}
template <int B, int W>
GSV_DI uint32_t hf_word(const uint32_t* win) {
    return hf_byte<B, 4 * W>(win) | (hf_byte<B, 4 * W + 1>(win) << 8) | (hf_byte<B, 4 * W + 2>(win) << 16) |
           (hf_byte<B, 4 * W + 3>(win) << 24);
}
template <int B, int... K>
GSV_DI void hf_absorb(uint32_t al[25], uint32_t ah[25], const uint32_t* win, std::integer_sequence<int, K...>) {
    ((al[K] ^= hf_word<B, 2 * K>(win), ah[K] ^= hf_word<B, 2 * K + 1>(win)), ...);
}
template <int B>
struct HfWin {  // the child-hash slots block B reads, as 32-bit words
    static constexpr int s0 = hf_s0(B), ns = hf_s1(B) - s0 + 1;
    uint32_t w[ns * 8];
};
template <int B>
GSV_DI void hf_load(HfWin<B>& W, const uint4* __restrict__ Hq) {
#pragma unroll
    for (int s = 0; s < HfWin<B>::ns; s++) {
        uint4 a = Hq[2 * (HfWin<B>::s0 + s)], b = Hq[2 * (HfWin<B>::s0 + s) + 1];
        W.w[8 * s + 0] = a.x; W.w[8 * s + 1] = a.y; W.w[8 * s + 2] = a.z; W.w[8 * s + 3] = a.w;
        W.w[8 * s + 4] = b.x; W.w[8 * s + 5] = b.y; W.w[8 * s + 6] = b.z; W.w[8 * s + 7] = b.w;
    }
}
template <int B>
GSV_DI void hf_absorb_block(uint32_t al[25], uint32_t ah[25], const HfWin<B>& W) {
    hf_absorb<B>(al, ah, W.w, std::make_integer_sequence<int, 17>{});
    if constexpr (B == 3) {  // pad: 0x01 at byte 532 - 408 = 124 (lane 15, high half), 0x80 at byte 135
        ah[15] ^= 0x01u;
        ah[16] ^= 0x80000000u;
    }
}
// Keccak-256 of the full branch f9 02 11 | (a0 || H_0) ... (a0 || H_15) | 80 (532 bytes, 4 blocks).
// Every byte's source is a compile-time function of its offset (templates above), so each 32-bit
// message word is a v_perm / shift of at most two child-hash words held in registers — no message
// buffer.  Block B + 1's child-hash words are loaded after block B's permutation: loading them before
// measured slower (r05: configs[2] 100.0 vs 101.3 GB/s, the held words raise the level kernel to 129
// VGPRs, three waves per SIMD; profiles/r05/ab/hfull_prefetch.txt).
GSV_DI void hash_hfull(uint32_t h[8], const uint32_t* __restrict__ H) {
    uint32_t al[25], ah[25];
#pragma unroll
    for (int k = 0; k < 25; k++) al[k] = ah[k] = 0;
    const uint4* Hq = (const uint4*)H;
    HfWin<0> w0;
    HfWin<1> w1;
    HfWin<2> w2;
    HfWin<3> w3;
    hf_load(w0, Hq);
    hf_absorb_block(al, ah, w0);
    keccakf_split(al, ah);
    hf_load(w1, Hq);
    hf_absorb_block(al, ah, w1);
    keccakf_split(al, ah);
    hf_load(w2, Hq);
    hf_absorb_block(al, ah, w2);
    keccakf_split(al, ah);
    hf_load(w3, Hq);
    hf_absorb_block(al, ah, w3);
    keccakf_split_digest(al, ah);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        h[2 * k] = al[k];
        h[2 * k + 1] = ah[k];
    }
}

GSV_DI void do_hfull(const PNode& nd, const BodyBatch& bb, uint32_t body) {
    const uint32_t* H = (const uint32_t*)(bb.msg + (size_t)body * bb.msg_stride + nd.msg_off);
    uint32_t h[8];
    hash_hfull(h, H);
    emit_hash(nd, bb, body, h);
}

// ---------------------------------------------------------------- generic nodes
// compact encoding (trie/encoding.go:37-52) of nibbles key(i)[d0:d1] (terminator included iff
// present); returns byte length, writes into c[0..]
GSV_DI int compact_key(uint8_t c[8], uint32_t i, int d0, int d1) {
    int term = (d1 > d0 && key_nib(i, d1 - 1) == 16) ? 1 : 0;
    int hl = d1 - d0 - term;
    int n = 1;
    c[0] = (uint8_t)(term << 5);
    int d = d0;
    if (hl & 1) {
        c[0] |= (uint8_t)(0x10 | key_nib(i, d));
        d++;
        hl--;
    }
    for (int k = 0; k < hl; k += 2) c[n++] = (uint8_t)((key_nib(i, d + k) << 4) | key_nib(i, d + k + 1));
    return n;
}

struct Writer {
    uint8_t* p;
    uint32_t n;
    GSV_DI void put(uint8_t b) { p[n++] = b; }
    GSV_DI void str(const uint8_t* s, int len) {  // RLP string, len < 56
        if (len == 1 && s[0] < 0x80) {
            put(s[0]);
            return;
        }
        put((uint8_t)(0x80 + len));
        for (int k = 0; k < len; k++) put(s[k]);
    }
    GSV_DI void list_header(uint32_t len) {
        if (len < 56) put((uint8_t)(0xc0 + len));
        else if (len < 256) {
            put(0xf8);
            put((uint8_t)len);
        } else {
            put(0xf9);
            put((uint8_t)(len >> 8));
            put((uint8_t)len);
        }
    }
};

GSV_DI uint32_t str_len(const uint8_t* s, int len) { return (len == 1 && s[0] < 0x80) ? 1u : 1u + len; }
GSV_DI uint32_t byte_val_len(uint8_t b) { return b == 0 ? 2u : b < 128 ? 1u : 3u; }  // rlp(rlp(uint(b)))
GSV_DI void put_byte_val(Writer& w, uint8_t b) {
    if (b == 0) {
        w.put(0x81);
        w.put(0x80);
    } else if (b < 128) {
        w.put(b);
    } else {
        w.put(0x82);
        w.put(0x81);
        w.put(b);
    }
}

// byte-mode leaf [compact(rem), rlp(value)] where value = rlp(uint(body byte)): RLP length
GSV_DI uint32_t leaf_len(uint32_t i, int d, uint8_t b) {
    uint8_t ck[8];
    int cl = compact_key(ck, i, d, key_len(i));
    uint32_t pl = str_len(ck, cl) + byte_val_len(b);
    return pl + 1;  // pl < 56
}
GSV_DI void write_leaf(Writer& w, uint32_t i, int d, uint8_t b) {
    uint8_t ck[8];
    int cl = compact_key(ck, i, d, key_len(i));
    w.list_header(str_len(ck, cl) + byte_val_len(b));
    w.str(ck, cl);
    put_byte_val(w, b);
}

// ref slot (16-byte aligned, global) -> its bytes appended to w; returns its length
GSV_DI void copy_ref(Writer& w, const uint8_t* s) {
    const uint4* q = (const uint4*)s;
    uint4 a = q[0], b = q[1], c = q[2];
    uint32_t x[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    uint32_t len = x[0] & 0xffu;
#pragma unroll
    for (int k = 0; k < 33; k++)
        if ((uint32_t)k < len) w.put((uint8_t)(x[(k + 8) >> 2] >> (8 * ((k + 8) & 3))));
}
GSV_DI uint32_t ref_len(const uint8_t* s) { return s[0]; }

GSV_DI const uint8_t* child_slot(const BodyBatch& bb, uint32_t body, const PChild& c, const PNode* nodes) {
    if (c.type == PC_LEAF) return bb.leafrefs + (bb.leaf_base[body] + c.idx) * REF_STRIDE;
    return bb.refs + (size_t)body * bb.ref_stride + (size_t)nodes[c.idx].ref_slot * REF_STRIDE;
}
GSV_DI uint32_t child_len(const BodyBatch& bb, uint32_t body, const PChild& c, const PNode* nodes) {
    if (c.type == PC_LEAF && !bb.generic) return leaf_len(c.idx, c.depth, bb.bodies[bb.body_off[body] + c.idx]);
    return ref_len(child_slot(bb, body, c, nodes));
}
GSV_DI void write_child(Writer& w, const BodyBatch& bb, uint32_t body, const PChild& c, const PNode* nodes) {
    if (c.type == PC_LEAF && !bb.generic) write_leaf(w, c.idx, c.depth, bb.bodies[bb.body_off[body] + c.idx]);
    else copy_ref(w, child_slot(bb, body, c, nodes));
}

// One generic node assembled and hashed by one lane in the node's own HBM message buffer (msg_off):
// the throughput form, for heights with many generic nodes (every height of a generic DeriveSha
// plan over a large batch), where a wave per node would idle 63 lanes through the permutations.
GSV_DI void do_generic_lane(const PNode& nd, const PChild* __restrict__ children, const PNode* __restrict__ nodes,
                            const BodyBatch& bb, uint32_t body) {
    const PChild* ch = nd.child_begin >= 0 ? children + nd.child_begin : nullptr;
    uint8_t* m = bb.msg + (size_t)body * bb.msg_stride + nd.msg_off;
    uint8_t ck[8];
    int cl = 0;
    uint32_t plen;
    if (nd.kind == PK_BRANCH) {
        plen = 1 + (16 - nd.nchild);
        for (int k = 0; k < nd.nchild; k++) plen += child_len(bb, body, ch[k], nodes);
    } else if (nd.kind == PK_EXT) {
        cl = compact_key(ck, nd.first_i, nd.depth, nd.ext_end);
        plen = str_len(ck, cl) + child_len(bb, body, ch[0], nodes);
    } else {
        cl = compact_key(ck, nd.first_i, nd.depth, key_len(nd.first_i));
        plen = str_len(ck, cl) + byte_val_len(bb.bodies[bb.body_off[body] + nd.first_i]);
    }
    Writer w{m, 0};
    w.list_header(plen);
    if (nd.kind == PK_BRANCH) {
        int k = 0;
        for (int slot = 0; slot < 16; slot++) {
            if (k < nd.nchild && ch[k].slot == slot) {
                write_child(w, bb, body, ch[k], nodes);
                k++;
            } else {
                w.put(0x80);
            }
        }
        w.put(0x80);
    } else if (nd.kind == PK_EXT) {
        w.str(ck, cl);
        write_child(w, bb, body, ch[0], nodes);
    } else {
        w.str(ck, cl);
        put_byte_val(w, bb.bodies[bb.body_off[body] + nd.first_i]);
    }
    uint32_t len = w.n;
    if (len >= 32 || nd.is_root) {
        uint32_t h[8];
        keccak_buf(h, m, len);
        emit_hash(nd, bb, body, h);
    } else {
        uint8_t* s = bb.refs + (size_t)body * bb.ref_stride + (size_t)nd.ref_slot * REF_STRIDE;
        s[0] = (uint8_t)len;
        for (uint32_t k = 0; k < len; k++) s[8 + k] = m[k];
    }
}

// generic nodes of one height, over all bodies, above which one lane per node beats one wave per node
// (r06: thresholds of 65,536 / 262,144 / never made the tx-root leg's 26 k-node first height 25 % slower,
// profiles/r06/ab/gen_lane_mode.txt)
constexpr uint64_t GEN_LANE_MODE_MIN = 4096;

// Generic node (BRANCH / EXT / byte-mode root LEAF) handled by a 32-lane group: lane k writes
// payload piece k of the RLP (BRANCH: slots 0..15 + the value slot; EXT / LEAF: key, child/value)
// at an offset from a group prefix sum into the group's LDS buffer m (8-byte aligned, MSG_STRIDE
// bytes), so the <= 16 child-ref loads run in parallel; the group then hashes it with the
// cooperative Keccak (>= 32 bytes or root, trie/hasher.go:163) or lane 0 inlines the RLP into the
// node's ref slot.  All 32 lanes of the group must call, with the same node.
GSV_DI void group_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

GSV_DI void do_generic_group(const PNode& nd, const PChild* __restrict__ children, const PNode* __restrict__ nodes,
                             const BodyBatch& bb, uint32_t body, uint8_t* m) {
    const int lane = threadIdx.x & 31;
    const PChild* ch = nd.child_begin >= 0 ? children + nd.child_begin : nullptr;
    // this lane's piece: 0 none, 1 empty slot / value slot (0x80), 2 child, 3 key, 4 byte value
    int piece = 0;
    const PChild* mine = nullptr;
    uint8_t ck[8];
    int cl = 0;
    if (nd.kind == PK_BRANCH) {
        if (lane < 16) {
            piece = 1;
            for (int k = 0; k < nd.nchild; k++)
                if (ch[k].slot == lane) {
                    piece = 2;
                    mine = ch + k;
                }
        } else if (lane == 16) {
            piece = 1;  // value slot (never set: keys are prefix-free)
        }
    } else if (lane == 0) {
        piece = 3;
        cl = nd.kind == PK_EXT ? compact_key(ck, nd.first_i, nd.depth, nd.ext_end)
                               : compact_key(ck, nd.first_i, nd.depth, key_len(nd.first_i));
    } else if (lane == 1) {
        piece = nd.kind == PK_EXT ? 2 : 4;
        mine = ch;
    }
    uint8_t bval = piece == 4 ? bb.bodies[bb.body_off[body] + nd.first_i] : 0;
    uint32_t plen = piece == 1 ? 1u : piece == 2 ? child_len(bb, body, *mine, nodes)
                  : piece == 3 ? str_len(ck, cl) : piece == 4 ? byte_val_len(bval) : 0u;
    uint32_t incl = plen;
#pragma unroll
    for (int d = 1; d < 32; d <<= 1) {
        uint32_t v = __shfl_up(incl, d, 32);
        if (lane >= d) incl += v;
    }
    uint32_t total = __shfl(incl, 31, 32);
    uint32_t hl = total < 56 ? 1u : total < 256 ? 2u : 3u;
    Writer w{m, hl + incl - plen};
    if (piece == 1) w.put(0x80);
    else if (piece == 2) write_child(w, bb, body, *mine, nodes);
    else if (piece == 3) w.str(ck, cl);
    else if (piece == 4) put_byte_val(w, bval);
    if (lane == 0) {
        Writer hw{m, 0};
        hw.list_header(total);
    }
    group_sync();
    uint32_t len = hl + total;
    if (len >= 32 || nd.is_root) {
        uint32_t h[8];
        keccak256_coop(h, m, len, lane);
        if (lane == 0) emit_hash(nd, bb, body, h);
    } else if (lane == 0) {
        uint8_t* s = bb.refs + (size_t)body * bb.ref_stride + (size_t)nd.ref_slot * REF_STRIDE;
        s[0] = (uint8_t)len;
        for (uint32_t k = 0; k < len; k++) s[8 + k] = m[k];
    }
    group_sync();  // m is reused by the group's next node
}

// HFULL node by a 32-lane group: the 532-byte message is laid out in LDS (lanes 0..15 copy child
// hash s after its a0 byte, lane 16 the list header and value slot), then hashed cooperatively
GSV_DI void do_hfull_group(const PNode& nd, const BodyBatch& bb, uint32_t body, uint8_t* m) {
    const int lane = threadIdx.x & 31;
    const uint4* H = (const uint4*)(bb.msg + (size_t)body * bb.msg_stride + nd.msg_off);
    if (lane < 16) {
        uint4 a = H[2 * lane], b = H[2 * lane + 1];
        uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint8_t* d = m + 3 + 33 * lane;
        d[0] = 0xa0;
#pragma unroll
        for (int k = 0; k < 32; k++) d[1 + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    } else if (lane == 16) {
        m[0] = 0xf9;
        m[1] = 0x02;
        m[2] = 0x11;
        m[531] = 0x80;
    }
    group_sync();
    uint32_t h[8];
    keccak256_coop(h, m, 532, lane);
    if (lane == 0) emit_hash(nd, bb, body, h);
    group_sync();
}

// One height below the fused top: generic nodes (one wave each) in the first gen_blocks workgroups
// so their latency-bound chains start first, then BOTTOM (height 1) or HFULL nodes one per lane in
// the same launch (they are independent of each other within a height).
struct LevelLaunch {
    int n0, nn;  // BOTTOM (BOT) or HFULL (!BOT) node range
    int g0, ng;  // generic node range
    uint32_t gen_blocks;
    int gen_lane;  // 1: one generic node per lane (gen_blocks of 256 lanes), 0: one per wave
};
// The level kernels keep the compiler's register budget (four waves per SIMD); five waves (96 VGPRs)
// measured within +-2 % (r03, r05: profiles/r05/ab/chunk_levels5_unroll2.txt).
template <bool BOT>
__global__ __launch_bounds__(256) void k_chunk_level(const PNode* __restrict__ nodes,
                                                     const PChild* __restrict__ children, LevelLaunch L,
                                                     BodyBatch bb) {
    __shared__ uint64_t sbuf[(BOT ? 256 * BOT_BUF : 8 * MSG_STRIDE) / 8];
    uint32_t blk = blockIdx.x;
    if (blk < L.gen_blocks && L.gen_lane) {
        uint64_t t = (uint64_t)blk * 256 + threadIdx.x;
        if (t >= (uint64_t)L.ng * bb.nbodies) return;
        const PNode nd = nodes[L.g0 + (int)(t % (uint64_t)L.ng)];
        do_generic_lane(nd, children, nodes, bb, (uint32_t)(t / (uint64_t)L.ng));
        return;
    }
    if (blk < L.gen_blocks) {
        uint64_t g = (uint64_t)blk * 8 + (threadIdx.x >> 5);  // one node per 32-lane group
        if (g >= (uint64_t)L.ng * bb.nbodies) return;         // uniform per group
        uint32_t body = (uint32_t)(g / (uint64_t)L.ng);
        const PNode nd = nodes[L.g0 + (int)(g % (uint64_t)L.ng)];
        do_generic_group(nd, children, nodes, bb, body, (uint8_t*)sbuf + (threadIdx.x >> 5) * MSG_STRIDE);
        return;
    }
    uint64_t t = (uint64_t)(blk - L.gen_blocks) * 256 + threadIdx.x;
    if (t >= (uint64_t)L.nn * bb.nbodies) return;
    uint32_t body = (uint32_t)(t / (uint64_t)L.nn);
    const PNode nd = nodes[L.n0 + (int)(t % (uint64_t)L.nn)];
    if constexpr (BOT) do_bottom(nd, bb, body, (uint8_t*)sbuf + threadIdx.x * BOT_BUF);
    else do_hfull(nd, bb, body);
}

// ---------------------------------------------------------------- fused top of the trie
struct TopLevels {
    int h0, h1;  // heights h0..h1 (inclusive), index h - 1 below
    int hb[TOP_MAX_H], he[TOP_MAX_H], gb[TOP_MAX_H], ge[TOP_MAX_H];
    uint32_t gen_lane;  // bit h - 1: that height's generic nodes one per lane (throughput form)
};
// The fused top is a short dependent chain (~17 permutations from height 3 to the root) that usually
// runs BESIDE bulk work: the next batch's bottom level (pipelined chunk roots) or k_notary_tx (the
// notary forks its chunk roots onto a side stream).  Running its waves at the highest wave priority
// (s_setprio 3) measured within noise (r04: configs[2] 91.7 vs 91.8 GB/s, the notary leg 9,844 vs 9,843
// shards/s; profiles/r04/ab/notary_sweep_top_prio{0,1}.txt), so they run at the default priority.
constexpr uint32_t TOP_MAX_BODIES = 256;  // one fused-top workgroup per CU at most
constexpr int TOP_HFULL_THREADS = 256;    // waves 0-3: HFULL nodes, one per lane (64 / 128: within +-2 %, r03)
constexpr int TOP_GEN_WAVES = 2;          // waves 4..: generic nodes, one per wave (never behind HFULL work)
constexpr int TOP_BLOCK = TOP_HFULL_THREADS + 64 * TOP_GEN_WAVES;

// one workgroup per body, a barrier between heights (children's hashes are in the CU's L1/L2).
// Per height: many HFULL nodes -> one per lane of waves 0-3 while the generic nodes go to the
// 32-lane groups of waves 4-5; few nodes (the chain up to the root) -> every node to a 32-lane group
// and the cooperative Keccak, which cuts each permutation's latency about threefold.
constexpr int TOP_GROUPS = TOP_BLOCK / 32;
constexpr int TOP_COOP_MAX = TOP_GROUPS;  // nodes per height up to which every node is group-hashed (one round)

// The fused top keeps the compiler's register budget (a smaller one, leaving the next batch's bottom
// level more of each SIMD's register file, measured null: profiles/r05/ab/top_register_budget.txt).
__global__ __launch_bounds__(TOP_BLOCK) void k_chunk_top(const PNode* __restrict__ nodes,
                                                         const PChild* __restrict__ children, TopLevels tl,
                                                         BodyBatch bb) {
    __shared__ uint64_t gbuf[TOP_GROUPS * MSG_STRIDE / 8];
    uint32_t body = blockIdx.x;
    int tid = threadIdx.x, grp = tid >> 5;
    uint8_t* m = (uint8_t*)gbuf + grp * MSG_STRIDE;
    for (int h = tl.h0; h <= tl.h1; h++) {
        int hb = tl.hb[h - 1], he = tl.he[h - 1];
        int gb = tl.gb[h - 1], ge = tl.ge[h - 1];
        int nh = he - hb, ng = ge - gb;
        if ((tl.gen_lane >> (h - 1)) & 1u) {  // many generic nodes: one per lane, after the HFULL lanes
            for (int i = hb + tid; i < he; i += TOP_BLOCK) do_hfull(nodes[i], bb, body);
            for (int i = gb + tid; i < ge; i += TOP_BLOCK) do_generic_lane(nodes[i], children, nodes, bb, body);
        } else if (nh + ng <= TOP_COOP_MAX) {  // the latency chain: every node to a group
            for (int k = grp; k < nh + ng; k += TOP_GROUPS) {
                if (k < nh) do_hfull_group(nodes[hb + k], bb, body, m);
                else do_generic_group(nodes[gb + k - nh], children, nodes, bb, body, m);
            }
        } else {  // HFULL nodes one per lane on waves 0-3, generic nodes on the groups of waves 4-5
            if (tid < TOP_HFULL_THREADS) {
                for (int i = hb + tid; i < he; i += TOP_HFULL_THREADS) do_hfull(nodes[i], bb, body);
            } else {
                int g = grp - TOP_HFULL_THREADS / 32;
                for (int i = gb + g; i < ge; i += TOP_GROUPS - TOP_HFULL_THREADS / 32)
                    do_generic_group(nodes[i], children, nodes, bb, body, m);
            }
        }
        __syncthreads();
    }
}

// ================================================================ launcher
size_t chunk_root_scratch_bytes(const TriePlan* plan, uint32_t nbodies) {
    size_t ms = (size_t)plan->h.n_msg * MSG_STRIDE;
    size_t rs = (size_t)plan->h.n_slots * REF_STRIDE;
    return (ms + rs) * nbodies + 512;
}

// Where a pipelined run's bulk kernels end (GSV_HOOK_TAIL: the next run on another instance starts its
// bulk kernels there): right after the bottom level (r05 default), so the next batch's bottom level
// runs beside this batch's HFULL level(s) as well as its fused top — the HFULL launch of a 100-body
// batch is ~400 waves, under half a wave per SIMD.  configs[2] 91.4-91.6 -> 93.4-94.2 GB/s at depth 2
// and 3 (profiles/r05/ab/chunk_tail_bottom.txt; through r04 the mark was before the top).
// all heights of the plan: per-height launches below top_h, then one fused launch
static hipError_t launch_levels(const TriePlan* plan, const BodyBatch& bb, hipStream_t st,
                                void (*timer_begin)(void*, int), void (*timer_end)(void*, int), void* tctx) {
    const TriePlanHost& p = plan->h;
    uint32_t nb = bb.nbodies;
    // the fused top is a latency tool: one workgroup per body, so it only pays while the bodies fit
    // on the CUs at once; a larger batch runs every height as a dense per-height launch instead
    const int top_h = nb <= TOP_MAX_BODIES ? p.top_h : p.height + 1;
    for (int h = 1; h < top_h; h++) {
        int b0 = p.lvl_bottom_begin[h - 1], b1 = p.lvl_bottom_end[h - 1];
        int f0 = p.lvl_hfull_begin[h - 1], f1 = p.lvl_hfull_end[h - 1];
        int g0 = p.lvl_gen_begin[h - 1], g1 = p.lvl_gen_end[h - 1];
        bool bot = b1 > b0;  // BOTTOM nodes only exist at height 1, where there is no HFULL node
        LevelLaunch L;
        L.n0 = bot ? b0 : f0;
        L.nn = bot ? b1 - b0 : f1 - f0;
        L.g0 = g0;
        L.ng = g1 - g0;
        L.gen_lane = (uint64_t)L.ng * nb >= GEN_LANE_MODE_MIN ? 1 : 0;
        L.gen_blocks = (uint32_t)(((uint64_t)L.ng * nb + (L.gen_lane ? 255 : 7)) / (L.gen_lane ? 256 : 8));
        uint64_t blocks = L.gen_blocks + ((uint64_t)L.nn * nb + 255) / 256;
        if (blocks == 0) continue;
        int kid = bot ? GSV_K_CHUNK_LEAF : GSV_K_CHUNK_LEVEL;
        if (timer_begin) timer_begin(tctx, kid);
        if (bot)
            hipLaunchKernelGGL(k_chunk_level<true>, dim3((unsigned)blocks), dim3(256), 0, st, plan->d_nodes,
                               plan->d_children, L, bb);
        else
            hipLaunchKernelGGL(k_chunk_level<false>, dim3((unsigned)blocks), dim3(256), 0, st, plan->d_nodes,
                               plan->d_children, L, bb);
        if (timer_end) timer_end(tctx, kid);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        if (bot && timer_begin) timer_begin(tctx, GSV_HOOK_TAIL);
    }
    if (top_h <= p.height) {
        if (p.height > TOP_MAX_H) return hipErrorInvalidValue;
        TopLevels tl{};
        tl.h0 = top_h;
        tl.h1 = p.height;
        for (int h = 1; h <= p.height; h++) {
            tl.hb[h - 1] = p.lvl_hfull_begin[h - 1];
            tl.he[h - 1] = p.lvl_hfull_end[h - 1];
            tl.gb[h - 1] = p.lvl_gen_begin[h - 1];
            tl.ge[h - 1] = p.lvl_gen_end[h - 1];
            if ((uint64_t)(tl.ge[h - 1] - tl.gb[h - 1]) * nb >= GEN_LANE_MODE_MIN) tl.gen_lane |= 1u << (h - 1);
        }
        if (timer_begin) timer_begin(tctx, GSV_K_CHUNK_LEVEL);
        hipLaunchKernelGGL(k_chunk_top, dim3(nb), dim3(TOP_BLOCK), 0, st, plan->d_nodes, plan->d_children, tl, bb);
        if (timer_end) timer_end(tctx, GSV_K_CHUNK_LEVEL);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_chunk_root_plan(const TriePlan* plan, const uint8_t* d_bodies, const uint64_t* d_body_off,
                                  uint32_t nbodies, uint8_t* d_scratch, uint8_t* d_roots, hipStream_t st,
                                  void (*timer_begin)(void*, int), void (*timer_end)(void*, int),
                                  void* tctx) {
    const TriePlanHost& p = plan->h;
    if (nbodies == 0 || p.nodes.empty()) return hipSuccess;
    BodyBatch bb;
    bb.bodies = d_bodies;
    bb.body_off = d_body_off;
    bb.msg_stride = (size_t)p.n_msg * MSG_STRIDE;
    bb.ref_stride = (size_t)p.n_slots * REF_STRIDE;
    bb.msg = d_scratch;
    bb.refs = d_scratch + bb.msg_stride * nbodies;
    bb.roots = d_roots;
    bb.nbodies = nbodies;
    bb.leafrefs = nullptr;
    bb.leaf_base = nullptr;
    bb.generic = 0;
    return launch_levels(plan, bb, st, timer_begin, timer_end, tctx);
}

// ================================================================ generic DeriveSha (any DerivableList)
// RLP length prefix for a string (base 0x80) or list (base 0xc0) of `len` bytes (rlp/encode.go:71-89)
template <class W>
GSV_DI void put_prefix(W& w, uint8_t base, uint32_t len) {
    if (len < 56) {
        w.put((uint8_t)(base + len));
        return;
    }
    int nb = len < 256 ? 1 : len < 65536 ? 2 : len < (1u << 24) ? 3 : 4;
    w.put((uint8_t)(base + 55 + nb));
    for (int k = nb - 1; k >= 0; k--) w.put((uint8_t)(len >> (8 * k)));
}
GSV_DI uint32_t prefix_len(uint32_t len) {
    return len < 56 ? 1u : len < 256 ? 2u : len < 65536 ? 3u : len < (1u << 24) ? 4u : 5u;
}

// A leaf's RLP header (<= 16 bytes) assembled in two registers, byte n at bits 8n
struct RegWriter {
    uint64_t w0 = 0, w1 = 0;
    uint32_t n = 0;
    GSV_DI void put(uint8_t b) {
        if (n < 8) w0 |= (uint64_t)b << (8 * n);
        else if (n < 16) w1 |= (uint64_t)b << (8 * (n - 8));
        n++;
    }
    GSV_DI void str(const uint8_t* s, int len) {  // RLP string, len < 56 (as Writer::str)
        if (len == 1 && s[0] < 0x80) {
            put(s[0]);
            return;
        }
        put((uint8_t)(0x80 + len));
        for (int k = 0; k < len; k++) put(s[k]);
    }
};
GSV_DI uint64_t low_bytes(int32_t n) { return n <= 0 ? 0ull : n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1ull); }
// Keccak-256 of header(H bytes in hw0/hw1) || v[0..L) without materialising the message: each rate
// block is read from v as <= 35 aligned dwords (only those holding a value byte) realigned with
// v_alignbyte, bytes outside the value masked, the header OR-ed into block 0's first two words.
typedef uint32_t u32x4a4_cr __attribute__((ext_vector_type(4), aligned(4)));
// whole (wave-uniform): each 16-byte group that holds a value byte is read as one dwordx4 — the up to 15
// bytes it reads outside the value belong to the batch's other values (the caller checks >= 32 bytes
// of the batch on both sides) and are masked like the per-dword path's (r06, as k_keccak256's final
// block: load_block_tail; k_derive_leaf 126.6 -> 118.7 us per tx-root step, the leg +3-5 %,
// profiles/r06/ab/derive_leaf.txt)
GSV_DI void keccak_hdr_value(uint32_t h[8], uint64_t hw0, uint64_t hw1, uint32_t H, const uint8_t* v, uint32_t L,
                             bool whole) {
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    uint32_t len = H + L, nfull = len / 136;
    for (uint32_t blk = 0; blk <= nfull; blk++) {
        int32_t base = (int32_t)(136 * blk);
        int32_t vlo = max((int32_t)H - base, 0), vhi = min((int32_t)len - base, 136);
        uintptr_t sa = (uintptr_t)v - H + (uintptr_t)base;  // source of block byte 0 (value coordinates)
        const uint32_t* q = (const uint32_t*)(sa & ~(uintptr_t)3);
        uint32_t sh = (uint32_t)(sa & 3u);
        uint32_t d[36];
        if (whole) {
#pragma unroll
            for (int g = 0; g < 9; g++) {
                int32_t b0 = 16 * g - (int32_t)sh;  // block position of the group's first byte
                u32x4a4_cr x = {0u, 0u, 0u, 0u};
                if (b0 + 16 > vlo && b0 < vhi) x = *(const u32x4a4_cr*)(q + 4 * g);
                d[4 * g] = x.x;
                d[4 * g + 1] = x.y;
                d[4 * g + 2] = x.z;
                d[4 * g + 3] = x.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 36; j++) {
                int32_t b0 = 4 * j - (int32_t)sh;  // block position of dword j's first byte
                d[j] = (j < 35 && b0 + 4 > vlo && b0 < vhi) ? q[j] : 0u;
            }
        }
        int32_t rem = (int32_t)len - base;  // in the final block: position of the 0x01 pad byte
#pragma unroll
        for (int k = 0; k < 17; k++) {
            uint32_t lo = __builtin_amdgcn_alignbyte(d[2 * k + 1], d[2 * k], sh);
            uint32_t hi = __builtin_amdgcn_alignbyte(d[2 * k + 2], d[2 * k + 1], sh);
            uint64_t x = ((uint64_t)lo | ((uint64_t)hi << 32)) & low_bytes(vhi - 8 * k) & ~low_bytes(vlo - 8 * k);
            if (blk == 0 && k == 0) x |= hw0;
            if (blk == 0 && k == 1) x |= hw1;
            if (blk == nfull) {
                if ((rem >> 3) == k) x ^= 0x01ull << (8 * (rem & 7));
                if (k == 16) x ^= 0x8000000000000000ULL;
            }
            a[k] ^= x;
        }
        keccakf(a);  // keccakf_digest on the last block: 162 -> 186 registers in k_derive_leaf
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        h[2 * k] = (uint32_t)a[k];
        h[2 * k + 1] = (uint32_t)(a[k] >> 32);
    }
}

// One lane per leaf: leaf j of list b = shortNode{hexToCompact(key(j)[depth:]), valueNode(GetRlp(j))}
// encoded [compact, string(value)] (trie/hasher.go:113-145 via node.go EncodeRLP); inlined into its
// parent when the RLP is < 32 bytes, else hashed; a list of one item is that leaf, hashed as root.
__global__ __launch_bounds__(256) void k_derive_leaf(const uint8_t* __restrict__ vals,
                                                     const uint64_t* __restrict__ voff, uint64_t vend,
                                                     uint8_t* lmsg,
                                                     const uint64_t* __restrict__ leaf_base,
                                                     const uint16_t* __restrict__ leaf_depth, uint32_t N,
                                                     uint32_t nlists, uint8_t* leafrefs, uint8_t* roots) {
    // leaves in permutation-count order within the workgroup (keccak_dev.cuh wg_bucket_order): a
    // leaf is its <= 16-byte header and the value, ~(L + 16) / 136 + 1 permutations
    uint64_t t0 = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    bool valid = t0 < (uint64_t)N * nlists;
    uint64_t blk = 0;
    if (valid) {
        uint64_t it0 = leaf_base[(uint32_t)(t0 / N)] + (uint32_t)(t0 % N);
        blk = (voff[it0 + 1] - voff[it0] + 16u) / 136u;
    }
    uint32_t tl = wg_bucket_order((uint32_t)(t0 - (uint64_t)blockIdx.x * 256), valid, blk);
    if (tl == ~0u) return;
    uint64_t t = (uint64_t)blockIdx.x * 256 + tl;
    uint32_t b = (uint32_t)(t / N), j = (uint32_t)(t % N);
    uint64_t item = leaf_base[b] + j;
    const uint8_t* v = vals + voff[item];
    uint32_t L = (uint32_t)(voff[item + 1] - voff[item]);
    int depth = leaf_depth[j];
    uint8_t ck[8];
    int cl = compact_key(ck, j, depth, key_len(j));
    uint32_t kenc = (cl == 1 && ck[0] < 0x80) ? 1u : 1u + cl;
    bool vbyte = (L == 1 && v[0] < 0x80);
    uint32_t venc = vbyte ? 1u : prefix_len(L) + L;
    uint8_t* s = leafrefs + item * REF_STRIDE;
    if (!vbyte) {  // hashed leaves (>= 32 bytes or the root): header in registers, value read in place
        RegWriter r;
        put_prefix(r, 0xc0, kenc + venc);
        r.str(ck, cl);
        put_prefix(r, 0x80, L);
        if (r.n <= 16 && (N == 1 || r.n + L >= 32)) {
            uint32_t h[8];
            // whole 16-byte groups when every lane's value has >= 32 bytes of the batch on both sides
            bool edge = voff[item] < voff[0] + 32 || voff[item + 1] + 32 > vend;
            keccak_hdr_value(h, r.w0, r.w1, r.n, v, L, __builtin_amdgcn_ballot_w64(edge) == 0);
            if (N == 1) store_hash32(roots + (size_t)b * 32, h);
            else store_hashref_slot(s, h);
            return;
        }
    }
    // this item's message buffer: 8-byte aligned, disjoint from its neighbours' (each needs <= L + 17
    // bytes and starts at least L + 25 bytes after the previous one)
    uint8_t* m = lmsg + (((voff[item] - voff[0]) + 7) & ~7ull) + 32ull * item;
    Writer w{m, 0};
    put_prefix(w, 0xc0, kenc + venc);
    w.str(ck, cl);
    if (vbyte) {
        w.put(v[0]);
    } else {
        put_prefix(w, 0x80, L);
        for (uint32_t k = 0; k < L; k++) w.put(v[k]);
    }
    uint32_t len = w.n;
    if (N == 1 || len >= 32) {
        uint32_t h[8];
        keccak_buf(h, m, len);
        if (N == 1) store_hash32(roots + (size_t)b * 32, h);
        else store_hashref_slot(s, h);
    } else {
        s[0] = (uint8_t)len;
        for (uint32_t k = 0; k < len; k++) s[8 + k] = m[k];
    }
}

size_t derive_sha_scratch_bytes(const TriePlan* plan, uint32_t nlists) {
    return plan->h.nodes.empty() ? 512 : chunk_root_scratch_bytes(plan, nlists);
}

hipError_t launch_derive_sha_plan(const TriePlan* plan, uint32_t nlists, const uint8_t* d_vals,
                                  const uint64_t* d_voff, uint64_t vend, const uint64_t* d_leaf_base, uint8_t* d_lmsg, uint8_t* d_leafrefs, uint8_t* d_scratch, uint8_t* d_roots,
                                  hipStream_t st, void (*timer_begin)(void*, int), void (*timer_end)(void*, int),
                                  void* tctx) {
    const TriePlanHost& p = plan->h;
    if (nlists == 0 || p.N == 0 || !p.generic) return hipSuccess;
    uint64_t total = (uint64_t)p.N * nlists;
    if (timer_begin) timer_begin(tctx, GSV_K_DERIVE_LEAF);
    hipLaunchKernelGGL(k_derive_leaf, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, d_vals, d_voff, vend,
                       d_lmsg, d_leaf_base, plan->d_leaf_depth, p.N, nlists, d_leafrefs, d_roots);
    if (timer_end) timer_end(tctx, GSV_K_DERIVE_LEAF);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || p.nodes.empty()) return e;
    BodyBatch bb;
    bb.bodies = nullptr;
    bb.body_off = nullptr;
    bb.msg_stride = (size_t)p.n_msg * MSG_STRIDE;
    bb.ref_stride = (size_t)p.n_slots * REF_STRIDE;
    bb.msg = d_scratch;
    bb.refs = d_scratch + bb.msg_stride * nlists;
    bb.roots = d_roots;
    bb.nbodies = nlists;
    bb.leafrefs = d_leafrefs;
    bb.leaf_base = d_leaf_base;
    bb.generic = 1;
    return launch_levels(plan, bb, st, timer_begin, timer_end, tctx);
}

// ================================================================ Proof of Custody body expansion
// sharding/collation.go:124-136: salted[k*(s+1) .. +s) = salt, salted[k*(s+1)+s] = body[k]; an empty
// body gives salted = salt.  grid.y = body; in_off holds (start, end) pairs per body, out_off the
// 16-byte aligned output starts.
//
// One thread per 16 output bytes, one dwordx4 store: the salted stream is the period-(s+1) pattern
// salt || 0 with body byte k in slot k*(s+1)+s.  Each workgroup stages the pattern (s + 1 + 24 bytes)
// in LDS; a thread reads its 16 bytes at phase r0 as five aligned LDS dwords (fewer than 64 dwords
// apart, so the lanes' different phases hit different banks) realigned with v_alignbyte, then ORs in
// the <= ceil(16 / (s+1)) body bytes of its window.  r05 wrote one dword per thread from per-byte
// salt and body loads: 1,583 -> 606 us per 100 x 1 MiB batch at a 20-byte salt (3.5 TB/s of writes), the
// POC leg 5,048-5,080 -> 5,309 bodies/s (r06, profiles/r06/ab/poc_expand.txt).
constexpr uint32_t POC_SALT_LDS = 8192;  // longer salts take k_poc_expand_bytes

__global__ __launch_bounds__(256) void k_poc_expand(const uint8_t* __restrict__ bodies,
                                                    const uint64_t* __restrict__ in_off,
                                                    const uint64_t* __restrict__ out_off,
                                                    const uint8_t* __restrict__ salt, uint32_t slen,
                                                    uint8_t* out) {
    __shared__ uint32_t s_pat[(POC_SALT_LDS + 1 + 24 + 3) / 4 + 1];
    const uint32_t per = slen + 1;
    uint8_t* pat8 = (uint8_t*)s_pat;
    for (uint32_t k = threadIdx.x; k < per + 24; k += 256) {
        uint32_t m = k % per;
        pat8[k] = m < slen ? salt[m] : 0;
    }
    __syncthreads();
    const uint32_t b = blockIdx.y;
    const uint64_t n_in = in_off[2 * b + 1] - in_off[2 * b];
    const uint64_t n_out = n_in ? n_in * per : slen;
    const uint64_t k0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    if (k0 >= n_out) return;
    const uint8_t* src = bodies + in_off[2 * b];
    uint8_t* dst = out + out_off[b];
    const uint64_t q0 = k0 / per;
    const uint32_t r0 = (uint32_t)(k0 - q0 * per);
    const uint32_t a = r0 >> 2, sh = r0 & 3u;
    uint32_t d[5];
#pragma unroll
    for (int j = 0; j < 5; j++) d[j] = s_pat[a + j];
    uint32_t w0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh), w1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
    uint32_t w2 = __builtin_amdgcn_alignbyte(d[3], d[2], sh), w3 = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
    if (n_in) {
        uint64_t q = q0;
        for (uint32_t u = slen - r0; u < 16u && q < n_in; u += per, q++) {  // the window's body bytes
            uint32_t v = (uint32_t)src[q] << (8u * (u & 3u));
            uint32_t i = u >> 2;
            w0 |= i == 0 ? v : 0u;
            w1 |= i == 1 ? v : 0u;
            w2 |= i == 2 ? v : 0u;
            w3 |= i == 3 ? v : 0u;
        }
    }
    if (k0 + 16 <= n_out) {
        *(uint4*)(dst + k0) = make_uint4(w0, w1, w2, w3);
    } else {
        uint32_t w[4] = {w0, w1, w2, w3};
        for (uint32_t u = 0; k0 + u < n_out; u++) dst[k0 + u] = (uint8_t)(w[u >> 2] >> (8u * (u & 3u)));
    }
}

// salts longer than POC_SALT_LDS: one thread per 4 output bytes, salt and body bytes read from HBM
__global__ __launch_bounds__(256) void k_poc_expand_bytes(const uint8_t* __restrict__ bodies,
                                                          const uint64_t* __restrict__ in_off,
                                                          const uint64_t* __restrict__ out_off,
                                                          const uint8_t* __restrict__ salt, uint32_t slen,
                                                          uint8_t* out) {
    uint32_t b = blockIdx.y;
    uint64_t n_in = in_off[2 * b + 1] - in_off[2 * b];
    uint64_t n_out = n_in ? n_in * (slen + 1) : slen;
    uint64_t k0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (k0 >= n_out) return;
    const uint8_t* src = bodies + in_off[2 * b];
    uint8_t* dst = out + out_off[b];
    uint64_t q = k0 / (slen + 1);
    uint32_t r = (uint32_t)(k0 - q * (slen + 1));
#pragma unroll
    for (int u = 0; u < 4; u++) {
        if (k0 + u < n_out) dst[k0 + u] = (!n_in || r < slen) ? salt[r] : src[q];
        if (++r > slen) {
            r = 0;
            q++;
        }
    }
}

hipError_t launch_poc_expand(const uint8_t* d_bodies, const uint64_t* d_in_off, const uint64_t* d_out_off,
                             uint32_t nbodies, uint64_t max_out, const uint8_t* d_salt, uint32_t slen, uint8_t* d_out,
                             hipStream_t st) {
    if (!nbodies || !max_out) return hipSuccess;
    if (slen <= POC_SALT_LDS) {
        uint64_t blocks = (max_out + 4095) / 4096;
        hipLaunchKernelGGL(k_poc_expand, dim3((unsigned)blocks, nbodies), dim3(256), 0, st, d_bodies, d_in_off,
                           d_out_off, d_salt, slen, d_out);
    } else {
        uint64_t blocks = (max_out + 1023) / 1024;
        hipLaunchKernelGGL(k_poc_expand_bytes, dim3((unsigned)blocks, nbodies), dim3(256), 0, st, d_bodies,
                           d_in_off, d_out_off, d_salt, slen, d_out);
    }
    return hipGetLastError();
}

}  // namespace gsv
