// Batched secp256k1 public-key recovery on gfx950 — one signature per lane.
//
// Semantics restated from the reference (bit-exact outputs and success/failure classes):
//   crypto/secp256k1/ext.h:30-47            secp256k1_ext_ecdsa_recover (parse -> recover -> serialize)
//   libsecp256k1/src/modules/recovery/main_impl.h:38-58   parse_compact: r, s >= n -> fail
//   main_impl.h:170-191   m = msg32 mod n
//   main_impl.h:87-121    r == 0 || s == 0 -> fail; recid & 2 -> x = r + n (r >= p - n -> fail);
//                         lift x with y parity recid & 1 (non-residue -> fail);
//                         Q = (s/r) R + (-m/r) G; Q == infinity -> fail
//   core/types/transaction_signing.go:222-247 recoverPlain + crypto/crypto.go:181-192 (sender kernel)
//
// Algorithm (ours, MI355X-first — not libsecp256k1's Strauss-wNAF, which branches per digit and
// wastes SIMD lanes).  Field arithmetic: 9 x 29-bit limbs with lazy reduction (secp256k1_fe9.cuh).
//   * u2*R: GLV split u2 = k1 + k2*lambda (|k1|,|k2| < 2^128), fixed-schedule odd-digit w = 4
//     recoding (recover_dev.cuh GSV_GLV_W: an add every 4th bit, identical across the wave: no
//     divergence), 8-entry table {1,3,...,15}R (entries 0..3 in LDS, 4..7 in per-lane scratch: the
//     LDS of two waves per SIMD holds four), built on an isomorphic curve
//     (libsecp-style "global z") so all table points are affine without an inversion; the lambda
//     half uses (beta x, y).  128 doublings + 65 mixed additions (w = 3 with the 4-entry table in
//     LDS: 129 + 88, measured 6 % slower: 15.5 -> 14.5 ms per 2^20 recoveries).
//   * u1*G: fixed-base comb, 13 windows of 20 bits from a 1.09 GB affine table in HBM (one random
//     80-byte entry per window, prefetched a window ahead), 12 mixed additions (window 0 starts the sum), no doublings
//     (gsv_internal.h COMB_BITS; 16-bit windows from the Infinity Cache were 1.3 % slower).
//   * no square root up front: u2*R runs on the curve y^2 = x^3 + 7 c^3 (c = x^3 + 7) where R is
//     (c x, c^2); one general add to combine, carried as a + t b (t = y_R); one exponentiation by
//     (p-3)/4 then gives both y_R and Z^-1 (recover_dev.cuh GSV_RECOVER_TWIST); fused Keccak-256
//     address.
#include "opcount.cuh"
#include "recover_dev.cuh"

namespace gsv {

// ---------------------------------------------------------------------------- kernels
// 2 waves/SIMD: two 256-thread blocks per CU share its 160 KiB LDS (72 KiB GLV table each)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSV_ECR_WAVES, GSV_ECR_WAVES))) void k_ecrecover(const uint8_t* __restrict__ msg32,
                                                   const uint8_t* __restrict__ sig65, uint32_t n,
                                                   const uint4* __restrict__ gtab,
                                                   uint8_t* __restrict__ pub65,
                                                   uint8_t* __restrict__ addr20,
                                                   uint8_t* __restrict__ status) {
    GSV_LTAB_DECL;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* sg = sig65 + (size_t)i * 65;
    uint32_t msg[8], r[8], s[8];
    load32_be(msg, msg32 + (size_t)i * 32);
    load32_be(r, sg);
    load32_be(s, sg + 32);
    uint32_t recid = sg[64];
    fe qx, qy;
    uint32_t st = recover_core(qx, qy, msg, r, s, recid & 3u, gtab, GSV_LTAB_LANE);
    if (recid >= 4) st = GSV_ST_INVALID_RECID;
    bool ok = st == GSV_ST_OK;
    store_pub_addr(pub65 ? pub65 + (size_t)i * 65 : nullptr, addr20 ? addr20 + (size_t)i * 20 : nullptr,
                   ok, qx, qy);
    status[i] = (uint8_t)st;
}

// recoverPlain (core/types/transaction_signing.go:222-247) + ValidateSignatureValues
// (crypto/crypto.go:181-192) + address = Keccak256(pub[1:])[12:]
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSV_ECR_WAVES, GSV_ECR_WAVES))) void k_sender(const uint8_t* __restrict__ sighash32,
                                                const uint8_t* __restrict__ r32,
                                                const uint8_t* __restrict__ s32,
                                                const uint64_t* __restrict__ v,
                                                const uint8_t* __restrict__ vbig, uint32_t n,
                                                int homestead, const uint4* __restrict__ gtab,
                                                uint8_t* __restrict__ addr20,
                                                uint8_t* __restrict__ status) {
    GSV_LTAB_DECL;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t msg[8], r[8], s[8];
    load32_be(msg, sighash32 + (size_t)i * 32);
    load32_be(r, r32 + (size_t)i * 32);
    load32_be(s, s32 + (size_t)i * 32);
    uint8_t V = (uint8_t)(v[i] - 27u);  // byte(Vb.Uint64() - 27)
    // Vb.BitLen() > 8 -> ErrInvalidSig, whatever the caller's v_big flag says
    bool valid = vbig[i] == 0 && v[i] <= 0xFFu;
    sc rs, ss;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        rs.v[k] = r[k];
        ss.v[k] = s[k];
    }
    valid = valid && !sc_is_zero(rs) && !sc_is_zero(ss);
    valid = valid && !(homestead && limbs_lt(HALF_N, s));
    valid = valid && limbs_lt(r, SN) && limbs_lt(s, SN) && (V == 0 || V == 1);
    fe qx, qy;
    uint32_t st = recover_core(qx, qy, msg, r, s, V & 1u, gtab, GSV_LTAB_LANE);
    if (!valid) st = GSV_ST_INVALID_SIG;
    store_pub_addr(nullptr, addr20 + (size_t)i * 20, st == GSV_ST_OK, qx, qy);
    status[i] = (uint8_t)st;
}

// The ecrecover precompile (core/vm/contracts.go:78-101): input = hash(32) || v(32) || r(32) || s(32),
// right-padded to 128 bytes by the caller (common.RightPadBytes).  ok[i] = 1 and out32 = the
// left-padded signer address (LeftPadBytes(Keccak256(pub[1:])[12:], 32)) on success; ok[i] = 0 and
// out32 zero where the reference returns (nil, nil): input[32:63] not all zero, or
// ValidateSignatureValues(v - 27, r, s, homestead = false) false, or Ecrecover failing.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GSV_ECR_WAVES, GSV_ECR_WAVES))) void k_ecrecover_precompile(
    const uint8_t* __restrict__ in128, uint32_t n, const uint4* __restrict__ gtab, uint8_t* __restrict__ out32,
    uint8_t* __restrict__ ok) {
    GSV_LTAB_DECL;
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = in128 + (size_t)i * 128;
    uint32_t msg[8], r[8], s[8];
    load32_be(msg, p);
    load32_be(r, p + 64);
    load32_be(s, p + 96);
    uint32_t hi = 0;  // allZero(input[32:63])
#pragma unroll
    for (int k = 32; k < 63; k++) hi |= p[k];
    uint8_t V = (uint8_t)(p[63] - 27u);  // byte arithmetic, wraps like the reference
    sc rs, ss;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        rs.v[k] = r[k];
        ss.v[k] = s[k];
    }
    bool valid = hi == 0 && !sc_is_zero(rs) && !sc_is_zero(ss) && limbs_lt(r, SN) && limbs_lt(s, SN) &&
                 (V == 0 || V == 1);
    fe qx, qy;
    uint32_t st = recover_core(qx, qy, msg, r, s, V & 1u, gtab, GSV_LTAB_LANE);
    bool good = valid && st == GSV_ST_OK;
    uint8_t* o = out32 + (size_t)i * 32;
#pragma unroll
    for (int k = 0; k < 12; k++) o[k] = 0;
    store_pub_addr(nullptr, o + 12, good, qx, qy);
    ok[i] = good ? 1 : 0;
}

// Fixed-base comb table: entry (w, d) = d * 2^(COMB_BITS w) * G, affine, canonical fe9 limbs
// (x[9] y[9] + 2 pad words, recover_dev.cuh gtab_load).  Built once per context in two launches:
// k_gtable_base writes each window's base B_w = 2^(COMB_BITS w) G into its unused d = 0 slot, then
// k_gtable_init computes d * B_w (COMB_BITS-bit double-and-add) for every d >= 1.
GSV_DI void gtab_store(uint4* e, const gej9& acc) {
    fe9 zi, zi2, x, y;
    fe9_inv(zi, acc.z);
    fe9_sqr(zi2, zi);
    fe9_mul(x, acc.x, zi2);
    fe9_mul(zi2, zi2, zi);
    fe9_mul(y, acc.y, zi2);
    fe9_normalize_full(x);
    fe9_normalize_full(y);
    e[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    e[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
    e[2] = make_uint4(x.v[8], y.v[0], y.v[1], y.v[2]);
    e[3] = make_uint4(y.v[3], y.v[4], y.v[5], y.v[6]);
    e[4] = make_uint4(y.v[7], y.v[8], 0u, 0u);
}

__global__ __launch_bounds__(64) void k_gtable_base(uint4* __restrict__ gtab) {
    uint32_t w = threadIdx.x;
    if (w >= (uint32_t)COMB_WINDOWS) return;
    gej9 acc;
    fe9_from_const(acc.x, GX);
    fe9_from_const(acc.y, GY);
    fe9_set_u32(acc.z, 1);
    for (uint32_t k = 0; k < (uint32_t)COMB_BITS * w; k++) gej9_dbl(acc, acc);
    gtab_store(gtab + ((size_t)w << COMB_BITS) * GTAB_ENTRY_U4, acc);
}

__global__ __launch_bounds__(256) void k_gtable_init(uint4* __restrict__ gtab) {
    size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= GTAB_ENTRIES) return;
    uint32_t w = (uint32_t)(id >> COMB_BITS), d = (uint32_t)(id & ((1u << COMB_BITS) - 1u));
    if (d == 0) return;  // holds B_w
    ge9 B;
    gtab_load(B, gtab + ((size_t)w << COMB_BITS) * GTAB_ENTRY_U4);
    gej9 acc;
    bool inf = true;
    acc.x = B.x;
    acc.y = B.y;
    fe9_set_u32(acc.z, 1);
    for (int b = COMB_BITS - 1; b >= 0; b--) {
        if (!inf) gej9_dbl(acc, acc);
        if ((d >> b) & 1u) gej9_add_ge(acc, inf, acc, B);
    }
    gtab_store(gtab + id * GTAB_ENTRY_U4, acc);
}

// ---------------------------------------------------------------------------- synthetic signer
__global__ __launch_bounds__(256) void k_synth_sign(uint64_t seed, uint32_t n,
                                                    const uint4* __restrict__ gtab,
                                                    uint8_t* __restrict__ msg32,
                                                    uint8_t* __restrict__ sig65,
                                                    uint8_t* __restrict__ pub65,
                                                    uint8_t* __restrict__ addr20) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sc d, k, m;
    derive32(d.v, seed, i, 0x79656bu);  // "key"
    derive32(m.v, seed, i, 0x67736du);  // "msg"
    derive32(k.v, seed, i, 0x65636eu);  // "nce"
    uint32_t r[8], s[8], recid;
    fe px, py;
    ecdsa_sign(r, s, recid, px, py, d, k, m.v, gtab);
    uint8_t* sg = sig65 + (size_t)i * 65;
    limbs_to_be(sg, r);
    limbs_to_be(sg + 32, s);
    sg[64] = (uint8_t)recid;
    limbs_to_be(msg32 + (size_t)i * 32, m.v);
    store_pub_addr(pub65 ? pub65 + (size_t)i * 65 : nullptr, addr20 ? addr20 + (size_t)i * 20 : nullptr,
                   true, px, py);
}

// ---------------------------------------------------------------------------- launchers
hipError_t launch_gtable_init(uint4* gtab, hipStream_t st) {
    hipLaunchKernelGGL(k_gtable_base, dim3(1), dim3(64), 0, st, gtab);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gtable_init, dim3((unsigned)((GTAB_ENTRIES + 255) / 256)), dim3(256), 0, st, gtab);
    return hipGetLastError();
}

hipError_t launch_ecrecover(const uint8_t* msg32, const uint8_t* sig65, uint32_t n, const uint4* gtab,
                            uint8_t* pub65, uint8_t* addr20, uint8_t* status, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ecrecover, dim3((n + 255) / 256), dim3(256), 0, st, msg32, sig65, n, gtab,
                       pub65, addr20, status);
    return hipGetLastError();
}

hipError_t launch_sender(const uint8_t* sighash32, const uint8_t* r32, const uint8_t* s32,
                         const uint64_t* v, const uint8_t* vbig, uint32_t n, int homestead,
                         const uint4* gtab, uint8_t* addr20, uint8_t* status, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_sender, dim3((n + 255) / 256), dim3(256), 0, st, sighash32, r32, s32, v, vbig,
                       n, homestead, gtab, addr20, status);
    return hipGetLastError();
}

hipError_t launch_ecrecover_precompile(const uint8_t* in128, uint32_t n, const uint4* gtab, uint8_t* out32,
                                       uint8_t* ok, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ecrecover_precompile, dim3((n + 255) / 256), dim3(256), 0, st, in128, n, gtab, out32, ok);
    return hipGetLastError();
}

hipError_t launch_synth_sign(uint64_t seed, uint32_t n, const uint4* gtab, uint8_t* msg32,
                             uint8_t* sig65, uint8_t* pub65, uint8_t* addr20, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth_sign, dim3((n + 255) / 256), dim3(256), 0, st, seed, n, gtab, msg32,
                       sig65, pub65, addr20);
    return hipGetLastError();
}

}  // namespace gsv

GSV_OPCOUNT_READER(ecrecover)
