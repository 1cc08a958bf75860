// Host side of the batch types.Sender path: strict RLP decode of txdata and the signer's sighash
// preimage, mirroring
//   core/types/transaction.go:55-70,125-133    txdata layout, isProtectedV
//   core/types/transaction_signing.go:127-137  EIP155Signer.Sender (chainId check, V - 2*chainId - 8)
//   core/types/transaction_signing.go:155-165  EIP155Signer.Hash  = rlpHash([...6 fields, chainId, 0, 0])
//   core/types/transaction_signing.go:182-220  Homestead/Frontier Sender + Hash (6 fields)
//   core/types/transaction_signing.go:250-260  deriveChainId
//   rlp/decode.go canonical-integer / canonical-size rules
// The Keccak of each preimage and the recovery run on the GPU (keccak.hip, ecrecover.hip).
#include <cstring>
#include <vector>

#include "tx_host.h"

namespace gsv {

namespace {

struct Item {
    const uint8_t* p;
    size_t n;
    bool list;
};

// one RLP item at p[0..len); returns consumed bytes, 0 on error
size_t rlp_item(const uint8_t* p, size_t len, Item& it) {
    if (len == 0) return 0;
    uint8_t b0 = p[0];
    if (b0 < 0x80) {
        it = {p, 1, false};
        return 1;
    }
    if (b0 < 0xb8) {
        size_t n = b0 - 0x80;
        if (1 + n > len) return 0;
        if (n == 1 && p[1] < 0x80) return 0;  // non-canonical size
        it = {p + 1, n, false};
        return 1 + n;
    }
    if (b0 < 0xc0) {
        size_t nb = b0 - 0xb7, n = 0;
        if (nb > 8 || 1 + nb > len || p[1] == 0) return 0;
        for (size_t i = 0; i < nb; i++) n = (n << 8) | p[1 + i];
        if (n < 56 || n > len - 1 - nb) return 0;
        it = {p + 1 + nb, n, false};
        return 1 + nb + n;
    }
    if (b0 < 0xf8) {
        size_t n = b0 - 0xc0;
        if (1 + n > len) return 0;
        it = {p + 1, n, true};
        return 1 + n;
    }
    size_t nb = b0 - 0xf7, n = 0;
    if (nb > 8 || 1 + nb > len || p[1] == 0) return 0;
    for (size_t i = 0; i < nb; i++) n = (n << 8) | p[1 + i];
    if (n < 56 || n > len - 1 - nb) return 0;
    it = {p + 1 + nb, n, true};
    return 1 + nb + n;
}

bool uint_ok(const Item& it, size_t maxlen) {
    return !it.list && it.n <= maxlen && !(it.n > 0 && it.p[0] == 0);
}
uint64_t to_u64(const Item& it) {
    uint64_t v = 0;
    for (size_t i = 0; i < it.n; i++) v = (v << 8) | it.p[i];
    return v;
}
size_t bitlen(const uint8_t* p, size_t n) {
    while (n && p[0] == 0) {
        p++;
        n--;
    }
    if (!n) return 0;
    size_t b = 8 * (n - 1);
    for (uint8_t x = p[0]; x; x >>= 1) b++;
    return b;
}

void put_header(std::vector<uint8_t>& o, size_t len, uint8_t base) {
    if (len < 56) {
        o.push_back((uint8_t)(base + len));
        return;
    }
    int nb = 0;
    for (size_t t = len; t; t >>= 8) nb++;
    o.push_back((uint8_t)(base + 55 + nb));
    for (int i = nb - 1; i >= 0; i--) o.push_back((uint8_t)(len >> (8 * i)));
}
void put_string(std::vector<uint8_t>& o, const uint8_t* d, size_t n) {
    if (n == 1 && d[0] < 0x80) {
        o.push_back(d[0]);
        return;
    }
    put_header(o, n, 0x80);
    o.insert(o.end(), d, d + n);
}
void put_uint_be(std::vector<uint8_t>& o, const uint8_t* d, size_t n) {
    while (n && d[0] == 0) {
        d++;
        n--;
    }
    put_string(o, d, n);
}
void put_u64(std::vector<uint8_t>& o, uint64_t v) {
    uint8_t t[8];
    for (int i = 0; i < 8; i++) t[i] = (uint8_t)(v >> (56 - 8 * i));
    put_uint_be(o, t, 8);
}

// big-endian a - b into out[64]; false if negative
bool be_sub(uint8_t out[64], const uint8_t* a, size_t an, const uint8_t* b, size_t bn) {
    if (an > 64 || bn > 64) return false;
    uint8_t A[64] = {0}, B[64] = {0};
    memcpy(A + 64 - an, a, an);
    memcpy(B + 64 - bn, b, bn);
    int br = 0;
    for (int i = 63; i >= 0; i--) {
        int d = (int)A[i] - B[i] - br;
        br = d < 0;
        out[i] = (uint8_t)(d + (br ? 256 : 0));
    }
    return !br;
}

}  // namespace

int tx_prepare(const uint8_t* rlp, size_t len, const uint8_t* cid, size_t cidlen, int signer_kind,
               TxPrep& out) {
    out.pre.clear();
    memset(out.r32, 0, 32);
    memset(out.s32, 0, 32);
    out.v = 0;
    out.vbig = 0;
    out.homestead = 1;
    Item outer, f[9];
    size_t used = rlp_item(rlp, len, outer);
    if (!used || used != len || !outer.list) return GSV_ST_BAD_RLP;
    const uint8_t* p = outer.p;
    size_t rem = outer.n;
    for (int i = 0; i < 9; i++) {
        size_t u = rlp_item(p, rem, f[i]);
        if (!u) return GSV_ST_BAD_RLP;
        p += u;
        rem -= u;
    }
    if (rem) return GSV_ST_BAD_RLP;
    if (!uint_ok(f[0], 8) || !uint_ok(f[2], 8) || !uint_ok(f[1], 256) || !uint_ok(f[4], 256) ||
        !uint_ok(f[6], 256) || !uint_ok(f[7], 256) || !uint_ok(f[8], 256))
        return GSV_ST_BAD_RLP;
    if (f[3].list || (f[3].n != 0 && f[3].n != 20) || f[5].list) return GSV_ST_BAD_RLP;

    auto sighash_pre = [&](bool eip155) {
        std::vector<uint8_t> body;
        put_u64(body, to_u64(f[0]));
        put_uint_be(body, f[1].p, f[1].n);
        put_u64(body, to_u64(f[2]));
        if (f[3].n == 20) put_string(body, f[3].p, 20);
        else put_header(body, 0, 0x80);  // nil recipient (rlp:"nil")
        put_uint_be(body, f[4].p, f[4].n);
        put_string(body, f[5].p, f[5].n);
        if (eip155) {
            put_uint_be(body, cid, cidlen);
            put_u64(body, 0);
            put_u64(body, 0);
        }
        put_header(out.pre, body.size(), 0xc0);
        out.pre.insert(out.pre.end(), body.begin(), body.end());
    };
    const Item& V = f[6];
    std::vector<uint8_t> vprime(V.p, V.p + V.n);
    if (signer_kind == GSV_SIGNER_EIP155) {
        size_t vb = bitlen(V.p, V.n);
        bool prot = true;
        if (vb <= 8) {
            uint64_t v = to_u64(V);
            prot = (v != 27 && v != 28);
        }
        if (prot) {
            uint8_t chain[64] = {0}, want[64] = {0};
            if (vb <= 64) {  // uint64 arithmetic with wrap-around exactly as deriveChainId
                uint64_t c = (to_u64(V) - 35) / 2;
                for (int i = 0; i < 8; i++) chain[56 + i] = (uint8_t)(c >> (56 - 8 * i));
            } else {
                uint8_t t[64];
                const uint8_t k35 = 35;
                if (!be_sub(t, V.p, V.n, &k35, 1)) return GSV_ST_INVALID_CHAIN_ID;
                int r = 0;
                for (int i = 0; i < 64; i++) {
                    int cur = r * 256 + t[i];
                    chain[i] = (uint8_t)(cur / 2);
                    r = cur % 2;
                }
            }
            if (cidlen > 64) return GSV_ST_INVALID_CHAIN_ID;
            memcpy(want + 64 - cidlen, cid, cidlen);
            if (memcmp(chain, want, 64) != 0) return GSV_ST_INVALID_CHAIN_ID;
            uint8_t two_c[64], t[64], vv[64];
            int carry = 0;
            for (int i = 63; i >= 0; i--) {
                int d = want[i] * 2 + carry;
                two_c[i] = (uint8_t)d;
                carry = d >> 8;
            }
            const uint8_t eight = 8;
            if (!be_sub(t, V.p, V.n, two_c, 64) || !be_sub(vv, t, 64, &eight, 1)) return GSV_ST_INVALID_SIG;
            vprime.assign(vv, vv + 64);
            sighash_pre(true);
        } else {
            sighash_pre(false);
        }
        out.homestead = 1;
    } else {
        sighash_pre(false);
        out.homestead = signer_kind == GSV_SIGNER_HOMESTEAD ? 1 : 0;
    }
    // recoverPlain inputs (core/types/transaction_signing.go:222-234)
    if (bitlen(vprime.data(), vprime.size()) > 8) out.vbig = 1;
    uint64_t v = 0;
    for (uint8_t b : vprime) v = (v << 8) | b;  // only the low byte matters when bitlen <= 8
    out.v = v;
    const Item& R = f[7];
    const Item& S = f[8];
    if (bitlen(R.p, R.n) > 256 || bitlen(S.p, S.n) > 256) {
        out.vbig = 1;  // R or S >= 2^256 >= n: ValidateSignatureValues fails
    } else {
        size_t rn = R.n > 32 ? 32 : R.n, sn = S.n > 32 ? 32 : S.n;
        memcpy(out.r32 + 32 - rn, R.p + R.n - rn, rn);
        memcpy(out.s32 + 32 - sn, S.p + S.n - sn, sn);
    }
    return GSV_ST_OK;
}

}  // namespace gsv
