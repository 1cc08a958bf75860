/*
 * TEST INFRASTRUCTURE ONLY. Second translation unit of oracle/_ref/libgsvref.so:
 * the reference's vendored ethash Keccak (vendor/github.com/ethereum/ethash/src/
 * libethash/sha3.c, delimiter 0x01 at sha3.c:146), compiled from /root/reference
 * by oracle/Makefile. Exposes it under a stable name for ctypes.
 */
#include <stddef.h>
#include <stdint.h>

int sha3_256(uint8_t *out, size_t outlen, uint8_t const *in, size_t inlen);

__attribute__((visibility("default"))) int gsvref_keccak256(uint8_t *out32, const uint8_t *in,
                                                            size_t len) {
    return sha3_256(out32, 32, in, len);
}

/* Many messages laid out back to back with offsets off[0..n] (timed CPU baseline). */
__attribute__((visibility("default"))) void gsvref_keccak256_many(uint8_t *out32, const uint8_t *data,
                                                                  const uint64_t *off, long n) {
    for (long i = 0; i < n; i++) sha3_256(out32 + 32 * i, 32, data + off[i], off[i + 1] - off[i]);
}
