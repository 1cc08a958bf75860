// Host emulation of the chunk-root trie PLAN (geth-sharding_amd/csrc/chunk_root.hip build_trie_plan, the
// product's own host code in libgsv.so): every node the plan lists is encoded on the CPU the way the
// kernels encode it (BOTTOM: 16 inline leaves [0x20, rlp(b)]; HFULL: f9 02 11 | (a0 || H) x 16 | 80;
// BRANCH / EXT / LEAF from the plan's children, trie/hasher.go:153-165 inlining, root forced) and the
// root compared by the caller with the oracle restatement (oracle_derive_sha_bytes).  A plan that
// encodes the wrong trie fails here without a GPU; a plan that is right while the GPU disagrees
// points at the kernels.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../geth-sharding_amd/csrc/chunk_root.h"

extern "C" void oracle_keccak256(const uint8_t* in, size_t len, uint8_t* out32);

namespace {

using Bytes = std::vector<uint8_t>;

int key_nbytes(uint32_t i) { return i < 128 ? 1 : i < 256 ? 2 : i < 65536 ? 3 : i < (1u << 24) ? 4 : 5; }
uint8_t key_byte(uint32_t i, int b) {
    int nb = key_nbytes(i);
    if (nb == 1) return i == 0 ? 0x80 : (uint8_t)i;
    if (b == 0) return (uint8_t)(0x80 + nb - 1);
    return (uint8_t)(i >> (8 * (nb - 1 - b)));
}
// nibbles of keybytesToHex(rlp(i)) (trie/encoding.go:65-75), terminator 16 last
Bytes key_hex(uint32_t i) {
    Bytes h;
    for (int b = 0; b < key_nbytes(i); b++) {
        h.push_back(key_byte(i, b) >> 4);
        h.push_back(key_byte(i, b) & 15);
    }
    h.push_back(16);
    return h;
}
// hexToCompact (trie/encoding.go:37-52)
Bytes compact(const Bytes& hex) {
    Bytes n = hex;
    uint8_t term = 0;
    if (!n.empty() && n.back() == 16) {
        term = 1;
        n.pop_back();
    }
    Bytes out(n.size() / 2 + 1, 0);
    out[0] = term << 5;
    size_t k = 0;
    if (n.size() & 1) {
        out[0] |= 0x10 | n[0];
        k = 1;
    }
    for (size_t j = 1; j < out.size(); j++, k += 2) out[j] = (uint8_t)(n[k] << 4 | n[k + 1]);
    return out;
}
void put_len(Bytes& o, size_t len, uint8_t short_base, uint8_t long_base) {
    if (len < 56) {
        o.push_back((uint8_t)(short_base + len));
        return;
    }
    uint8_t t[8];
    int nb = 0;
    for (size_t v = len; v; v >>= 8) t[nb++] = (uint8_t)v;
    o.push_back((uint8_t)(long_base + nb));
    for (int j = nb - 1; j >= 0; j--) o.push_back(t[j]);
}
Bytes rlp_str(const Bytes& s) {
    Bytes o;
    if (s.size() == 1 && s[0] < 0x80) return s;
    put_len(o, s.size(), 0x80, 0xb7);
    o.insert(o.end(), s.begin(), s.end());
    return o;
}
Bytes rlp_list(const Bytes& payload) {
    Bytes o;
    put_len(o, payload.size(), 0xc0, 0xf7);
    o.insert(o.end(), payload.begin(), payload.end());
    return o;
}
Bytes value_of(uint8_t b) {  // Chunks.GetRlp(i) = rlp(body[i])
    return b == 0 ? Bytes{0x80} : b < 128 ? Bytes{b} : Bytes{0x81, b};
}
Bytes leaf_enc(uint32_t i, int depth, const uint8_t* body) {
    Bytes hex = key_hex(i);
    Bytes rem(hex.begin() + depth, hex.end());
    Bytes p = rlp_str(compact(rem));
    Bytes v = rlp_str(value_of(body[i]));
    p.insert(p.end(), v.begin(), v.end());
    return rlp_list(p);
}
// reference of an encoded node inside its parent (hasher.go:153-165): inline below 32 bytes
Bytes ref_of(const Bytes& enc, bool force) {
    if (enc.size() < 32 && !force) return enc;
    uint8_t h[32];
    oracle_keccak256(enc.data(), enc.size(), h);
    Bytes r{0xa0};
    r.insert(r.end(), h, h + 32);
    return r;
}

}  // namespace

// root of the trie the plan for N describes over body[0..N); returns 0, or -1 on a plan
// inconsistency (a child encoded after its parent, a missing slot owner)
extern "C" int plan_emu_root(const uint8_t* body, uint32_t N, uint8_t* root32, int* height, int* top_h) {
    gsv::TriePlanHost p;
    gsv::build_trie_plan(p, N, false);
    const int M = (int)p.nodes.size();
    *height = p.height;
    *top_h = p.top_h;
    std::vector<Bytes> ref(M);
    std::vector<char> done(M, 0);
    // HFULL children: msg buffer index -> node, then slot from the offset inside it
    std::vector<int> by_msg(p.n_msg, -1);
    for (int i = 0; i < M; i++)
        if (p.nodes[i].msg_off >= 0) by_msg[p.nodes[i].msg_off / gsv::MSG_STRIDE] = i;
    std::vector<std::vector<int>> hkids(M, std::vector<int>(16, -1));
    for (int i = 0; i < M; i++) {
        int pm = p.nodes[i].parent_msg;
        if (pm < 0) continue;
        int par = by_msg[pm / gsv::MSG_STRIDE];
        int slot = (pm % gsv::MSG_STRIDE) / 32;
        if (par < 0 || slot > 15 || hkids[par][slot] >= 0) return -1;
        hkids[par][slot] = i;
    }
    for (int i = 0; i < M; i++) {
        const gsv::PNode& n = p.nodes[i];
        bool force = i == p.root;
        Bytes enc;
        if (n.kind == gsv::PK_BOTTOM) {
            Bytes pay;
            for (int j = 0; j < 16; j++) {
                Bytes l = leaf_enc(n.first_i + j, n.depth + 1, body);
                pay.insert(pay.end(), l.begin(), l.end());
            }
            pay.push_back(0x80);
            enc = rlp_list(pay);
        } else if (n.kind == gsv::PK_HFULL) {
            Bytes pay;
            for (int s = 0; s < 16; s++) {
                int c = hkids[i][s];
                if (c < 0 || !done[c] || ref[c].size() != 33) return -1;
                pay.insert(pay.end(), ref[c].begin(), ref[c].end());
            }
            pay.push_back(0x80);
            enc = rlp_list(pay);
        } else if (n.kind == gsv::PK_BRANCH) {
            std::vector<Bytes> slots(16, Bytes{0x80});
            for (int k = 0; k < n.nchild; k++) {
                const gsv::PChild& c = p.children[n.child_begin + k];
                if (c.type == gsv::PC_LEAF) slots[c.slot] = ref_of(leaf_enc(c.idx, c.depth, body), false);
                else {
                    if (!done[c.idx]) return -1;
                    slots[c.slot] = ref[c.idx];
                }
            }
            Bytes pay;
            for (auto& s : slots) pay.insert(pay.end(), s.begin(), s.end());
            pay.push_back(0x80);
            enc = rlp_list(pay);
        } else if (n.kind == gsv::PK_EXT) {
            const gsv::PChild& c = p.children[n.child_begin];
            if (c.type != gsv::PC_NODE || !done[c.idx]) return -1;
            Bytes hex = key_hex(n.first_i);
            Bytes seg(hex.begin() + n.depth, hex.begin() + n.ext_end);
            Bytes pay = rlp_str(compact(seg));
            pay.insert(pay.end(), ref[c.idx].begin(), ref[c.idx].end());
            enc = rlp_list(pay);
        } else {  // PK_LEAF (N == 1)
            enc = leaf_enc(n.first_i, n.depth, body);
        }
        ref[i] = ref_of(enc, force);
        done[i] = 1;
    }
    if (p.root < 0 || ref[p.root].size() != 33) return -1;
    memcpy(root32, ref[p.root].data() + 1, 32);
    return 0;
}
