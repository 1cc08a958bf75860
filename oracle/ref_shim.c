/*
 * TEST INFRASTRUCTURE ONLY — never linked into the product (libgsv.so).
 *
 * Thin C shim that compiles the reference's OWN C sources straight from
 * /root/reference (nothing is copied into this repository) into
 * oracle/_ref/libgsvref.so, so the restated oracle (oracle/gsv_oracle.c) and the
 * HIP path can be checked against the real reference code, and so bench.py can
 * time the reference CPU path ("cpu_baseline.kind": "reference").
 *
 *   - libsecp256k1 exactly as geth's cgo preamble builds it
 *     (crypto/secp256k1/secp256.go:21-31: USE_NUM_NONE, USE_FIELD_10X26,
 *     USE_FIELD_INV_BUILTIN, USE_SCALAR_8X32, USE_SCALAR_INV_BUILTIN, NDEBUG)
 *     plus the cgo shim crypto/secp256k1/ext.h:30-47 (secp256k1_ext_ecdsa_recover).
 *   - Keccak-256 from vendor/github.com/ethereum/ethash/src/libethash/sha3.c
 *     (sha3_256 with delimiter 0x01, sha3.c:146) — compiled as its own TU.
 *
 * Build recipe: oracle/Makefile target `ref` (gcc on these files directly).
 */
#define USE_NUM_NONE
#define USE_FIELD_10X26
#define USE_FIELD_INV_BUILTIN
#define USE_SCALAR_8X32
#define USE_SCALAR_INV_BUILTIN
#define NDEBUG
#include "src/secp256k1.c"
#include "src/modules/recovery/main_impl.h"
#include "ext.h"

#include <pthread.h>

static secp256k1_context *g_ctx;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void ref_init_once(void) {
    /* crypto/secp256k1/secp256.go:45-52: one global SIGN|VERIFY context. */
    g_ctx = secp256k1_context_create_sign_verify();
}

__attribute__((visibility("default"))) int gsvref_init(void) {
    pthread_once(&g_once, ref_init_once);
    return g_ctx != NULL;
}

/* crypto/secp256k1/secp256.go:105-122 RecoverPubkey, minus the Go-side length
 * checks (callers pass fixed-size buffers); recid >= 4 is rejected here as
 * checkSignature (secp256.go:171-178) does.  Returns 1 ok / 0 fail / -1 bad recid. */
__attribute__((visibility("default"))) int gsvref_ecrecover(unsigned char *pub65,
                                                            const unsigned char *sig65,
                                                            const unsigned char *msg32) {
    gsvref_init();
    if (sig65[64] >= 4) return -1;
    return secp256k1_ext_ecdsa_recover(g_ctx, pub65, sig65, msg32);
}

/* Batch loop over the reference path (used only as the timed CPU baseline). */
__attribute__((visibility("default"))) int gsvref_ecrecover_many(unsigned char *pub65,
                                                                 const unsigned char *sig65,
                                                                 const unsigned char *msg32,
                                                                 long n) {
    int ok = 0;
    gsvref_init();
    for (long i = 0; i < n; i++) {
        if (sig65[65 * i + 64] >= 4) continue;
        ok += secp256k1_ext_ecdsa_recover(g_ctx, pub65 + 65 * i, sig65 + 65 * i, msg32 + 32 * i);
    }
    return ok;
}

/* crypto/secp256k1/secp256.go:70-101 Sign: RFC6979 recoverable signature,
 * serialized [R || S || V] with V = recid. */
__attribute__((visibility("default"))) int gsvref_sign(unsigned char *sig65,
                                                       const unsigned char *msg32,
                                                       const unsigned char *seckey32) {
    secp256k1_ecdsa_recoverable_signature s;
    int recid = 0;
    gsvref_init();
    if (secp256k1_ec_seckey_verify(g_ctx, seckey32) != 1) return 0;
    if (!secp256k1_ecdsa_sign_recoverable(g_ctx, &s, msg32, seckey32,
                                          secp256k1_nonce_function_rfc6979, NULL))
        return 0;
    secp256k1_ecdsa_recoverable_signature_serialize_compact(g_ctx, sig65, &recid, &s);
    sig65[64] = (unsigned char)recid;
    return 1;
}

/* Uncompressed public key of a secret key (for fixture generation). */
__attribute__((visibility("default"))) int gsvref_pubkey(unsigned char *pub65,
                                                         const unsigned char *seckey32) {
    secp256k1_pubkey pk;
    size_t len = 65;
    gsvref_init();
    if (!secp256k1_ec_pubkey_create(g_ctx, &pk, seckey32)) return 0;
    return secp256k1_ec_pubkey_serialize(g_ctx, pub65, &len, &pk, SECP256K1_EC_UNCOMPRESSED);
}

/* Signature with a caller-chosen nonce (libsecp256k1's nonce-function hook): reproduces the GPU's
 * synthetic signer (gsv_synth_sign) with the reference's own signing code, for the configs[1]
 * fixture.  Low-s normalised with the recid flipped, as secp256k1_ecdsa_sig_sign does. */
static int fixed_nonce(unsigned char *nonce32, const unsigned char *msg32, const unsigned char *key32,
                       const unsigned char *algo16, void *data, unsigned int attempt) {
    (void)msg32;
    (void)key32;
    (void)algo16;
    if (attempt) return 0;
    memcpy(nonce32, data, 32);
    return 1;
}

__attribute__((visibility("default"))) int gsvref_sign_nonce(unsigned char *sig65, const unsigned char *msg32,
                                                             const unsigned char *seckey32,
                                                             const unsigned char *nonce32) {
    secp256k1_ecdsa_recoverable_signature s;
    int recid = 0;
    gsvref_init();
    if (!secp256k1_ecdsa_sign_recoverable(g_ctx, &s, msg32, seckey32, fixed_nonce, (void *)nonce32)) return 0;
    secp256k1_ecdsa_recoverable_signature_serialize_compact(g_ctx, sig65, &recid, &s);
    sig65[64] = (unsigned char)recid;
    return 1;
}

int sha3_256(uint8_t *out, size_t outlen, uint8_t const *in, size_t inlen);

/* n signatures i = i0 .. i0+n-1 of the GPU's synthetic signer (gsv_synth_sign) made by the
 * reference's code: msg / key / nonce = ethash Keccak-256(le64(seed) || le64(i) || tag), key and
 * nonce reduced mod n by secp256k1_scalar_set_b32 (0 -> 1). */
__attribute__((visibility("default"))) long gsvref_synth_sign_many(uint64_t seed, long i0, long n,
                                                                   unsigned char *msg32, unsigned char *sig65) {
    long ok = 0;
    gsvref_init();
    for (long j = 0; j < n; j++) {
        uint64_t i = (uint64_t)(i0 + j);
        unsigned char in[19], key[32], nce[32];
        for (int b = 0; b < 8; b++) {
            in[b] = (unsigned char)(seed >> (8 * b));
            in[8 + b] = (unsigned char)(i >> (8 * b));
        }
        memcpy(in + 16, "msg", 3);
        sha3_256(msg32 + 32 * j, 32, in, 19);
        unsigned char *kk[2] = {key, nce};
        const char *tags[2] = {"key", "nce"};
        for (int t = 0; t < 2; t++) {
            secp256k1_scalar sc;
            int overflow = 0;
            memcpy(in + 16, tags[t], 3);
            sha3_256(kk[t], 32, in, 19);
            secp256k1_scalar_set_b32(&sc, kk[t], &overflow);
            if (secp256k1_scalar_is_zero(&sc)) secp256k1_scalar_set_int(&sc, 1);
            secp256k1_scalar_get_b32(kk[t], &sc);
        }
        ok += gsvref_sign_nonce(sig65 + 65 * j, msg32 + 32 * j, key, nce);
    }
    return ok;
}

/* ---- configs[3] synthetic collations, made with the reference's own signer ----
 * The bytes the GPU generator (notary.hip k_notary_synth) writes for shard `s`: tx j is an EIP-155
 * transaction (core/types/transaction.go:55-70 field order) signed by libsecp256k1 with the
 * generator's key and nonce (Keccak-256(le64(seed) || le64(gi) || tag), gi = s * txs + j), RLP-encoded
 * (rlp/encode.go) and blob-serialized into 4 chunks of [indicator | 31 bytes] at body offset 128 j
 * (sharding/utils/marshal.go:71-123).  Tx j with j % 128 == 127 is invalid by construction, class
 * (gi / 128) % 4: 0 high-s (s -> n - s, recid ^ 1), 1 V encodes chain 5, 2 r = 2^255 + 2 (no point
 * has that x), 3 recid flipped (a valid signature of ANOTHER key: only the sender tells). */
static unsigned put_be_uint(unsigned char *o, uint64_t v) { /* rlp of a uint64 (rlp/encode.go:390) */
    unsigned char t[8];
    unsigned n = 0;
    for (int i = 7; i >= 0; i--) {
        unsigned char b = (unsigned char)(v >> (8 * i));
        if (n || b) t[n++] = b;
    }
    if (n == 0) {
        o[0] = 0x80;
        return 1;
    }
    if (n == 1 && t[0] < 0x80) {
        o[0] = t[0];
        return 1;
    }
    o[0] = (unsigned char)(0x80 + n);
    memcpy(o + 1, t, n);
    return 1 + n;
}

static unsigned put_be_bytes(unsigned char *o, const unsigned char *b32) { /* rlp of a 256-bit big int */
    unsigned z = 0;
    while (z < 32 && b32[z] == 0) z++;
    unsigned n = 32 - z;
    if (n == 1 && b32[z] < 0x80) {
        o[0] = b32[z];
        return 1;
    }
    o[0] = (unsigned char)(0x80 + n);
    memcpy(o + 1, b32 + z, n);
    return 1 + n;
}

static void synth_tag(unsigned char out[32], uint64_t seed, uint64_t i, const char *tag, int tlen) {
    unsigned char in[19];
    for (int b = 0; b < 8; b++) {
        in[b] = (unsigned char)(seed >> (8 * b));
        in[8 + b] = (unsigned char)(i >> (8 * b));
    }
    memset(in + 16, 0, 3);
    memcpy(in + 16, tag, (size_t)tlen);
    sha3_256(out, 32, in, 19);
}

static void synth_scalar(unsigned char k[32]) { /* mod n, 0 -> 1 (as gsvref_synth_sign_many) */
    secp256k1_scalar sc;
    int overflow = 0;
    secp256k1_scalar_set_b32(&sc, k, &overflow);
    if (secp256k1_scalar_is_zero(&sc)) secp256k1_scalar_set_int(&sc, 1);
    secp256k1_scalar_get_b32(k, &sc);
}

/* body_out: txs * 128 bytes.  Returns the number of txs signed (txs on success). */
__attribute__((visibility("default"))) long gsvref_notary_synth_body(uint64_t seed, uint32_t shard, uint32_t txs,
                                                                     unsigned char *body_out) {
    long ok = 0;
    gsvref_init();
    for (uint32_t j = 0; j < txs; j++) {
        uint64_t gi = (uint64_t)shard * txs + j;
        unsigned char f[112], pre[124], h[32], key[32], nce[32], sig[65], tx[128];
        unsigned w = 0;
        w += put_be_uint(f + w, j % 128);
        w += put_be_uint(f + w, 20000000000ull);
        w += put_be_uint(f + w, 21000);
        synth_tag(h, seed, gi, "to", 2);
        f[w++] = 0x94;
        memcpy(f + w, h + 12, 20);
        w += 20;
        w += put_be_uint(f + w, gi);
        f[w++] = 0x80;
        /* sighash preimage rlp([6 fields, chainId 1, 0, 0]) (transaction_signing.go:155-165) */
        unsigned blen = w + 3, plen = 0;
        if (blen < 56) pre[plen++] = (unsigned char)(0xc0 + blen);
        else {
            pre[plen++] = 0xf8;
            pre[plen++] = (unsigned char)blen;
        }
        memcpy(pre + plen, f, w);
        plen += w;
        pre[plen++] = 0x01;
        pre[plen++] = 0x80;
        pre[plen++] = 0x80;
        unsigned char msg[32];
        sha3_256(msg, 32, pre, plen);
        synth_tag(key, seed, gi, "key", 3);
        synth_tag(nce, seed, gi, "nce", 3);
        synth_scalar(key);
        synth_scalar(nce);
        if (!gsvref_sign_nonce(sig, msg, key, nce)) continue;
        ok++;
        unsigned chain = 1, recid = sig[64];
        if (j % 128 == 127) {
            unsigned cls = (unsigned)((gi / 128) % 4);
            if (cls == 0) { /* high-s */
                secp256k1_scalar s;
                int of = 0;
                secp256k1_scalar_set_b32(&s, sig + 32, &of);
                secp256k1_scalar_negate(&s, &s);
                secp256k1_scalar_get_b32(sig + 32, &s);
                recid ^= 1u;
            } else if (cls == 1) {
                chain = 5;
            } else if (cls == 2) {
                memset(sig, 0, 32);
                sig[0] = 0x80;
                sig[31] = 0x02;
            } else {
                recid ^= 1u;
            }
        }
        w += put_be_uint(f + w, (recid & 1u) + 35 + 2 * chain);
        w += put_be_bytes(f + w, sig);
        w += put_be_bytes(f + w, sig + 32);
        unsigned tlen = 0;
        tx[tlen++] = 0xf8;
        tx[tlen++] = (unsigned char)w;
        memcpy(tx + tlen, f, w);
        tlen += w;
        unsigned char *out = body_out + (size_t)j * 128;
        for (unsigned c = 0; c < 4; c++) {
            unsigned lo = c * 31;
            out[c * 32] = (unsigned char)(c == 3 ? tlen - 93 : 0);
            for (unsigned q = 0; q < 31; q++) out[c * 32 + 1 + q] = lo + q < tlen ? tx[lo + q] : 0;
        }
    }
    return ok;
}
