// Operation counters of the instrumented build (tools/count_ops.py builds libgsv.so with
// -DGSV_OPCOUNT into variants/opcount/): how many 256-bit field / scalar products, inversions
// and Keccak-f permutations the kernels execute, summed over executing lanes (one wave-level
// atomic per counted operation).  The product build compiles every GSV_OPC() to nothing.
#pragma once

namespace gsv {
enum OpKind : int {
    OPC_FE_MUL = 0,  // secp256k1 field product (fe9 / 8x32)
    OPC_FE_SQR = 1,  // secp256k1 field squaring
    OPC_SC_MUL = 2,  // scalar (mod n) product, incl. the GLV split's 256x256 products
    OPC_SC_SQR = 3,
    OPC_BN_MUL = 4,  // BN254 F_p Montgomery product
    OPC_MODINV = 5,  // safegcd inversion (mod p, mod n, BN254 p)
    OPC_BN_REDC = 6, // BN254 Montgomery reduction (one per fq_mul / fq_mul2 / fq_dot)
    OPC_FE_DOT = 7,  // secp256k1 a*b + c*d with one reduction (fe9_dot: 162 + 19 mads)
    OPC_N = 8
};
}  // namespace gsv

#if defined(GSV_OPCOUNT) && defined(__HIPCC__)
#include <hip/hip_runtime.h>
static __device__ unsigned long long gsv_opc_counts[gsv::OPC_N];
__device__ __forceinline__ void gsv_opc(int k) {
    unsigned long long m = __ballot(1);
    if ((int)__lane_id() == __ffsll((long long)m) - 1) atomicAdd(&gsv_opc_counts[k], (unsigned long long)__popcll(m));
}
#define GSV_OPC(k) gsv_opc(k)
// host reader of this translation unit's counters: extern "C" gsv_opcount_<name>(out[OPC_N], reset)
#define GSV_OPCOUNT_READER(name)                                                                       \
    extern "C" int gsv_opcount_##name(unsigned long long* out, int reset) {                            \
        if (hipDeviceSynchronize() != hipSuccess) return -1;                                           \
        if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gsv_opc_counts), sizeof(gsv_opc_counts)) != hipSuccess) \
            return -1;                                                                                 \
        if (reset) {                                                                                   \
            unsigned long long z[gsv::OPC_N] = {0};                                                    \
            if (hipMemcpyToSymbol(HIP_SYMBOL(gsv_opc_counts), z, sizeof(z)) != hipSuccess) return -1;  \
        }                                                                                              \
        return 0;                                                                                      \
    }
#else
#define GSV_OPC(k) ((void)0)
#define GSV_OPCOUNT_READER(name)
#endif
