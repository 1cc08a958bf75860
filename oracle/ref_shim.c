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
