// Batched Keccak-256 over variable-length messages (crypto.Keccak256, crypto/crypto.go:43-49;
// sponge crypto/sha3/sha3.go:98-157, rate 136, dsbyte 0x01).  One message per lane; each lane
// absorbs its own 136-byte blocks.  Used for transaction sighashes (RLP preimages) and as the
// generic batch hash entry point.
#include "gsv_internal.h"
#include "keccak_dev.cuh"

namespace gsv {

GSV_DI uint64_t load_le64_bytes(const uint8_t* p, uint32_t avail) {
    // avail >= 8: full lane; otherwise partial (zero-filled)
    uint64_t v = 0;
    if (avail >= 8 && ((uintptr_t)p & 7u) == 0) return *(const uint64_t*)p;
#pragma unroll
    for (int b = 0; b < 8; b++)
        if ((uint32_t)b < avail) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

__global__ __launch_bounds__(256) void k_keccak256(const uint8_t* __restrict__ data,
                                                   const uint64_t* __restrict__ off, uint32_t n,
                                                   uint8_t* __restrict__ out32) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = data + off[i];
    uint64_t len = off[i + 1] - off[i];
    uint64_t a[25];
#pragma unroll
    for (int k = 0; k < 25; k++) a[k] = 0;
    while (len >= 136) {
#pragma unroll
        for (int k = 0; k < 17; k++) a[k] ^= load_le64_bytes(p + 8 * k, 8);
        keccakf(a);
        p += 136;
        len -= 136;
    }
    // final block: remaining len bytes, then 0x01 at len, 0x80 at 135
    uint32_t rem = (uint32_t)len;
#pragma unroll
    for (int k = 0; k < 17; k++) {
        int32_t avail = (int32_t)rem - 8 * k;
        uint64_t w = avail > 0 ? load_le64_bytes(p + 8 * k, (uint32_t)(avail > 8 ? 8 : avail)) : 0;
        if ((uint32_t)(rem >> 3) == (uint32_t)k) w ^= 0x01ull << (8 * (rem & 7u));
        if (k == 16) w ^= 0x8000000000000000ULL;
        a[k] ^= w;
    }
    keccakf(a);
    uint8_t* o = out32 + (size_t)i * 32;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int b = 0; b < 8; b++) o[8 * k + b] = (uint8_t)(a[k] >> (8 * b));
}

hipError_t launch_keccak256(const uint8_t* data, const uint64_t* off, uint32_t n, uint8_t* out32,
                            hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_keccak256, dim3((n + 255) / 256), dim3(256), 0, st, data, off, n, out32);
    return hipGetLastError();
}

}  // namespace gsv
