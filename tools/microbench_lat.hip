// Issue cost and dependent latency of the integer VALU patterns a 256-bit modular product is
// built from, on gfx950.  Each kernel runs LOOP iterations of ONE asm statement holding 32
// instructions (no compiler padding inside), timed per wave with s_memtime (shader clock), at
// W = 1, 2, 4, 8 waves per SIMD.  Reported: shader cycles per instruction per wave, and per SIMD
// (= per-wave / W): the SIMD throughput cost once enough waves hide the latency.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include "../geth-sharding_amd/csrc/secp256k1_dev.cuh"
#include "../geth-sharding_amd/csrc/secp256k1_fe9.cuh"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int LOOP = 256;

#define R4(x) x x x x
#define R8(x) R4(x) R4(x)
#define R16(x) R8(x) R8(x)
#define R32(x) R16(x) R16(x)

#define KERNEL_BEGIN(name)                                                                   \
    __global__ __launch_bounds__(256) void name(uint64_t* cyc, uint32_t* out, uint32_t seed) { \
        uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 7u + seed;                          \
        uint64_t x0 = ((uint64_t)a << 3) + 1, x1 = x0 + 3, x2 = x0 + 5, x3 = x0 + 7;          \
        uint64_t x4 = x0 + 9, x5 = x0 + 11, x6 = x0 + 13, x7 = x0 + 15;                        \
        uint32_t y0 = a, y1 = a + 1, y2 = a + 2, y3 = a + 3, y4 = a + 4, y5 = a + 5, y6 = a + 6, y7 = a + 7; \
        uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0;               \
        uint64_t t0 = __builtin_readcyclecounter();                                          \
        for (int it = 0; it < LOOP; it++) {
#define KERNEL_END                                                                           \
        }                                                                                    \
        uint64_t t1 = __builtin_readcyclecounter();                                          \
        uint64_t z = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7; \
        uint32_t w = y0 ^ y1 ^ y2 ^ y3 ^ y4 ^ y5 ^ y6 ^ y7;                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)z ^ (uint32_t)(z >> 32) ^ w;   \
        if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0; \
    }

#define IO64 "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
#define IO32 "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3), "+v"(y4), "+v"(y5), "+v"(y6), "+v"(y7)
#define IOS "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)
// operand numbering: %0-%7 x (64-bit VGPR pairs), %8-%15 y (32-bit), %16-%23 s (SGPR pairs), %24 a, %25 b

// 1. v_mad_u64_u32 dependent through the 64-bit accumulator (carry-out to an unread SGPR pair)
KERNEL_BEGIN(k_mad_dep)
    asm volatile(R32("v_mad_u64_u32 %0, %16, %24, %25, %0\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 2. v_mad_u64_u32, 8 independent accumulators
KERNEL_BEGIN(k_mad_ind)
    asm volatile(R4("v_mad_u64_u32 %0, %16, %24, %25, %0\n\tv_mad_u64_u32 %1, %17, %24, %25, %1\n\tv_mad_u64_u32 %2, %18, %24, %25, %2\n\tv_mad_u64_u32 %3, %19, %24, %25, %3\n\tv_mad_u64_u32 %4, %20, %24, %25, %4\n\tv_mad_u64_u32 %5, %21, %24, %25, %5\n\tv_mad_u64_u32 %6, %22, %24, %25, %6\n\tv_mad_u64_u32 %7, %23, %24, %25, %7\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 3. v_addc chain through vcc and the destination
KERNEL_BEGIN(k_addc_dep)
    asm volatile(R32("v_addc_co_u32_e64 %8, vcc, %8, %24, vcc\n\t") : IO64, IO32, IOS : "v"(a), "v"(b) : "vcc");
KERNEL_END
// 4. v_addc, 8 independent destinations and carries (own SGPR pair each)
KERNEL_BEGIN(k_addc_ind)
    asm volatile(R4("v_addc_co_u32_e64 %8, %16, %8, %24, %16\n\tv_addc_co_u32_e64 %9, %17, %9, %24, %17\n\tv_addc_co_u32_e64 %10, %18, %10, %24, %18\n\tv_addc_co_u32_e64 %11, %19, %11, %24, %19\n\tv_addc_co_u32_e64 %12, %20, %12, %24, %20\n\tv_addc_co_u32_e64 %13, %21, %13, %24, %21\n\tv_addc_co_u32_e64 %14, %22, %14, %24, %22\n\tv_addc_co_u32_e64 %15, %23, %15, %24, %23\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 5. v_add_u32, 8 independent
KERNEL_BEGIN(k_add_ind)
    asm volatile(R4("v_add_u32 %8, %8, %24\n\tv_add_u32 %9, %9, %24\n\tv_add_u32 %10, %10, %24\n\tv_add_u32 %11, %11, %24\n\tv_add_u32 %12, %12, %24\n\tv_add_u32 %13, %13, %24\n\tv_add_u32 %14, %14, %24\n\tv_add_u32 %15, %15, %24\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 6. v_add_u32 dependent
KERNEL_BEGIN(k_add_dep)
    asm volatile(R32("v_add_u32 %8, %8, %24\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 7. v_lshl_add_u64 (64-bit add, shift 0), 8 independent
KERNEL_BEGIN(k_add64_ind)
    asm volatile(R4("v_lshl_add_u64 %0, %0, 0, %1\n\tv_lshl_add_u64 %1, %1, 0, %2\n\tv_lshl_add_u64 %2, %2, 0, %3\n\tv_lshl_add_u64 %3, %3, 0, %4\n\tv_lshl_add_u64 %4, %4, 0, %5\n\tv_lshl_add_u64 %5, %5, 0, %6\n\tv_lshl_add_u64 %6, %6, 0, %7\n\tv_lshl_add_u64 %7, %7, 0, %0\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 8. v_lshl_add_u64 dependent
KERNEL_BEGIN(k_add64_dep)
    asm volatile(R32("v_lshl_add_u64 %0, %0, 0, %1\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 9. product-scanning pattern: mad (carry -> vcc) + addc overflow word, one chain
KERNEL_BEGIN(k_madaddc_1)
    asm volatile(R16("v_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e64 %8, vcc, 0, %8, vcc\n\t") : IO64, IO32, IOS : "v"(a), "v"(b) : "vcc");
KERNEL_END
// 10. the same pattern, two interleaved chains (carries in vcc and in an SGPR pair)
KERNEL_BEGIN(k_madaddc_2)
    asm volatile(R8("v_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_mad_u64_u32 %1, %16, %24, %25, %1\n\tv_addc_co_u32_e64 %8, vcc, 0, %8, vcc\n\tv_addc_co_u32_e64 %9, %16, 0, %9, %16\n\t") : IO64, IO32, IOS : "v"(a), "v"(b) : "vcc");
KERNEL_END
// 11. v_add3_u32, 8 independent
KERNEL_BEGIN(k_add3_ind)
    asm volatile(R4("v_add3_u32 %8, %8, %24, %25\n\tv_add3_u32 %9, %9, %24, %25\n\tv_add3_u32 %10, %10, %24, %25\n\tv_add3_u32 %11, %11, %24, %25\n\tv_add3_u32 %12, %12, %24, %25\n\tv_add3_u32 %13, %13, %24, %25\n\tv_add3_u32 %14, %14, %24, %25\n\tv_add3_u32 %15, %15, %24, %25\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 12. v_cndmask_b32 on an SGPR-pair mask, 8 independent
KERNEL_BEGIN(k_cndmask_ind)
    asm volatile(R4("v_cndmask_b32_e64 %8, %8, %24, %16\n\tv_cndmask_b32_e64 %9, %9, %24, %17\n\tv_cndmask_b32_e64 %10, %10, %24, %18\n\tv_cndmask_b32_e64 %11, %11, %24, %19\n\tv_cndmask_b32_e64 %12, %12, %24, %20\n\tv_cndmask_b32_e64 %13, %13, %24, %21\n\tv_cndmask_b32_e64 %14, %14, %24, %22\n\tv_cndmask_b32_e64 %15, %15, %24, %23\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 13. v_mul_hi_u32 + v_mul_lo_u32, 8 independent (4 of each)
KERNEL_BEGIN(k_mullohi_ind)
    asm volatile(R4("v_mul_lo_u32 %8, %8, %24\n\tv_mul_hi_u32 %9, %9, %24\n\tv_mul_lo_u32 %10, %10, %24\n\tv_mul_hi_u32 %11, %11, %24\n\tv_mul_lo_u32 %12, %12, %24\n\tv_mul_hi_u32 %13, %13, %24\n\tv_mul_lo_u32 %14, %14, %24\n\tv_mul_hi_u32 %15, %15, %24\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 14. v_mad_u32_u24 (24-bit multiply-add, 32-bit result), 8 independent
KERNEL_BEGIN(k_mad24_ind)
    asm volatile(R4("v_mad_u32_u24 %8, %8, %24, %25\n\tv_mad_u32_u24 %9, %9, %24, %25\n\tv_mad_u32_u24 %10, %10, %24, %25\n\tv_mad_u32_u24 %11, %11, %24, %25\n\tv_mad_u32_u24 %12, %12, %24, %25\n\tv_mad_u32_u24 %13, %13, %24, %25\n\tv_mad_u32_u24 %14, %14, %24, %25\n\tv_mad_u32_u24 %15, %15, %24, %25\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 15. v_pk_mov_b32 (column hand-off), 8 independent
KERNEL_BEGIN(k_pkmov_ind)
    asm volatile(R4("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]\n\tv_pk_mov_b32 %1, %1, %2 op_sel:[1,0]\n\tv_pk_mov_b32 %2, %2, %3 op_sel:[1,0]\n\tv_pk_mov_b32 %3, %3, %4 op_sel:[1,0]\n\tv_pk_mov_b32 %4, %4, %5 op_sel:[1,0]\n\tv_pk_mov_b32 %5, %5, %6 op_sel:[1,0]\n\tv_pk_mov_b32 %6, %6, %7 op_sel:[1,0]\n\tv_pk_mov_b32 %7, %7, %0 op_sel:[1,0]\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 16. v_mad_u64_u32 dependent, carry-out to vcc (unread)
KERNEL_BEGIN(k_mad_dep_vcc)
    asm volatile(R32("v_mad_u64_u32 %0, vcc, %24, %25, %0\n\t") : IO64, IO32, IOS : "v"(a), "v"(b) : "vcc");
KERNEL_END

// 17. v_addc_co_u32_e32 (VOP2 encoding, implicit vcc), 8 destinations, carry chain through vcc
KERNEL_BEGIN(k_addc32_vcc)
    asm volatile(R4("v_addc_co_u32_e32 %8, vcc, %24, %8, vcc\n\tv_addc_co_u32_e32 %9, vcc, %24, %9, vcc\n\tv_addc_co_u32_e32 %10, vcc, %24, %10, vcc\n\tv_addc_co_u32_e32 %11, vcc, %24, %11, vcc\n\tv_addc_co_u32_e32 %12, vcc, %24, %12, vcc\n\tv_addc_co_u32_e32 %13, vcc, %24, %13, vcc\n\tv_addc_co_u32_e32 %14, vcc, %24, %14, vcc\n\tv_addc_co_u32_e32 %15, vcc, %24, %15, vcc\n\t") : IO64, IO32, IOS : "v"(a), "v"(b) : "vcc");
KERNEL_END
// 18. v_add_u32 with a 32-bit literal (VOP2 + literal = 8 bytes)
KERNEL_BEGIN(k_add_lit)
    asm volatile(R4("v_add_u32 %8, 0x12345, %8\n\tv_add_u32 %9, 0x12345, %9\n\tv_add_u32 %10, 0x12345, %10\n\tv_add_u32 %11, 0x12345, %11\n\tv_add_u32 %12, 0x12345, %12\n\tv_add_u32 %13, 0x12345, %13\n\tv_add_u32 %14, 0x12345, %14\n\tv_add_u32 %15, 0x12345, %15\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 19. v_add_u32_e64 (VOP3 encoding of a VOP2 op)
KERNEL_BEGIN(k_add_e64)
    asm volatile(R4("v_add_u32_e64 %8, %8, %24\n\tv_add_u32_e64 %9, %9, %24\n\tv_add_u32_e64 %10, %10, %24\n\tv_add_u32_e64 %11, %11, %24\n\tv_add_u32_e64 %12, %12, %24\n\tv_add_u32_e64 %13, %13, %24\n\tv_add_u32_e64 %14, %14, %24\n\tv_add_u32_e64 %15, %15, %24\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 20. alternating v_mad_u64_u32 (VOP3) and v_addc_co_u32_e32 (VOP2): the product-scanning pair
KERNEL_BEGIN(k_mad_addc32)
    asm volatile(R16("v_mad_u64_u32 %0, vcc, %24, %25, %0\n\tv_addc_co_u32_e32 %8, vcc, 0, %8, vcc\n\t") : IO64, IO32, IOS : "v"(a), "v"(b) : "vcc");
KERNEL_END
// 21. alternating v_mad_u64_u32 and independent v_add_u32
KERNEL_BEGIN(k_mad_add)
    asm volatile(R16("v_mad_u64_u32 %0, %16, %24, %25, %0\n\tv_add_u32 %8, %8, %24\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 22. v_mov_b32 (VOP1), 8 independent
KERNEL_BEGIN(k_mov_ind)
    asm volatile(R4("v_mov_b32 %8, %9\n\tv_mov_b32 %9, %10\n\tv_mov_b32 %10, %11\n\tv_mov_b32 %11, %12\n\tv_mov_b32 %12, %13\n\tv_mov_b32 %13, %14\n\tv_mov_b32 %14, %15\n\tv_mov_b32 %15, %8\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 23. s_nop 0
KERNEL_BEGIN(k_snop)
    asm volatile(R32("s_nop 0\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 24. v_bitop3_b32 (VOP3), 8 independent
KERNEL_BEGIN(k_bitop3)
    asm volatile(R4("v_bitop3_b32 %8, %8, %24, %25 bitop3:0x96\n\tv_bitop3_b32 %9, %9, %24, %25 bitop3:0x96\n\tv_bitop3_b32 %10, %10, %24, %25 bitop3:0x96\n\tv_bitop3_b32 %11, %11, %24, %25 bitop3:0x96\n\tv_bitop3_b32 %12, %12, %24, %25 bitop3:0x96\n\tv_bitop3_b32 %13, %13, %24, %25 bitop3:0x96\n\tv_bitop3_b32 %14, %14, %24, %25 bitop3:0x96\n\tv_bitop3_b32 %15, %15, %24, %25 bitop3:0x96\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END
// 25. v_xor_b32 (VOP2) 8 independent
KERNEL_BEGIN(k_xor)
    asm volatile(R4("v_xor_b32 %8, %24, %8\n\tv_xor_b32 %9, %24, %9\n\tv_xor_b32 %10, %24, %10\n\tv_xor_b32 %11, %24, %11\n\tv_xor_b32 %12, %24, %12\n\tv_xor_b32 %13, %24, %13\n\tv_xor_b32 %14, %24, %14\n\tv_xor_b32 %15, %24, %15\n\t") : IO64, IO32, IOS : "v"(a), "v"(b));
KERNEL_END

// clock calibration: s_memtime vs s_memrealtime (100 MHz)
__global__ void k_clock(uint64_t* o) {
    uint64_t t0 = __builtin_readcyclecounter(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (int i = 0; i < 200000; i++) asm volatile("v_add_u32 %0, %0, %0" : "+v"(x));
    uint64_t t1 = __builtin_readcyclecounter(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) { o[0] = t1 - t0; o[1] = r1 - r0; o[2] = x; }
}

// whole field products in a dependent loop: 8x32 (secp256k1_dev.cuh) vs 9x29 (secp256k1_fe9.cuh)
template <int MODE>
__global__ __launch_bounds__(256) void k_field(uint64_t* cyc, uint32_t* out, uint32_t seed) {
    gsv::fe a, b;
    gsv::fe9 a9, b9;
#pragma unroll
    for (int i = 0; i < 8; i++) { a.v[i] = (threadIdx.x + i * 0x9E3779B9u) ^ seed; b.v[i] = (blockIdx.x * 13 + i * 0x85EBCA6Bu) ^ seed; }
    a.v[7] &= 0x7FFFFFFFu; b.v[7] &= 0x7FFFFFFFu;
    gsv::fe9_from_words(a9, a.v); gsv::fe9_from_words(b9, b.v);
    uint64_t t0 = __builtin_readcyclecounter();
    for (int it = 0; it < 64; it++) {
        if (MODE == 0) gsv::fe_mul(a, a, b);
        else if (MODE == 1) gsv::fe_sqr(a, a);
        else if (MODE == 2) gsv::fe9_mul(a9, a9, b9);
        else if (MODE == 3) gsv::fe9_sqr(a9, a9);
        else if (MODE == 4) gsv::fe_add(a, a, b);
        else if (MODE == 5) { gsv::fe9_add(a9, a9, b9); gsv::fe9_normalize_weak(a9); }
        else if (MODE == 6) { gsv::gej g; g.x = a; g.y = b; g.z = a; gsv::gej_dbl(g, g); a = g.x; b = g.y; }
        else { gsv::gej9 g; g.x = a9; g.y = b9; g.z = a9; gsv::gej9_dbl(g, g); a9 = g.x; b9 = g.y; }
    }
    uint64_t t1 = __builtin_readcyclecounter();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= a.v[i] ^ b.v[i];
#pragma unroll
    for (int i = 0; i < 9; i++) s ^= a9.v[i] ^ b9.v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = (t1 - t0) * 128;  // printed as cycles per field op (64 ops; the table divides by 256 x 32)
}

typedef void (*kfn)(uint64_t*, uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    printf("device %s CUs %d nominal clock %.0f MHz\n", prop.gcnArchName, cus, prop.clockRate / 1e3);
    uint32_t* d;
    uint64_t* dc;
    int maxw = 8;
    CHECK(hipMalloc(&d, sizeof(uint32_t) * cus * 256 * maxw));
    CHECK(hipMalloc(&dc, sizeof(uint64_t) * cus * 4 * maxw));
    struct { const char* name; kfn f; } ks[] = {
        {"mad dep (acc chain)", k_mad_dep}, {"mad dep, sdst=vcc", k_mad_dep_vcc}, {"mad x8 independent", k_mad_ind},
        {"addc dep (vcc chain)", k_addc_dep}, {"addc x8 indep (own SGPR)", k_addc_ind},
        {"add_u32 dep", k_add_dep}, {"add_u32 x8 indep", k_add_ind}, {"add3_u32 x8 indep", k_add3_ind},
        {"lshl_add_u64 dep", k_add64_dep}, {"lshl_add_u64 x8 indep", k_add64_ind},
        {"mad+addc 1 chain", k_madaddc_1}, {"mad+addc 2 chains", k_madaddc_2},
        {"cndmask x8 indep", k_cndmask_ind}, {"mul_lo/hi x8 indep", k_mullohi_ind}, {"mad_u32_u24 x8 indep", k_mad24_ind},
        {"pk_mov_b32 x8 indep", k_pkmov_ind},
        {"addc_e32 x8 (vcc chain)", k_addc32_vcc}, {"add_u32 + literal x8", k_add_lit}, {"add_u32_e64 x8", k_add_e64},
        {"mad / addc_e32 pairs", k_mad_addc32}, {"mad / add_u32 pairs", k_mad_add}, {"mov_b32 x8", k_mov_ind},
        {"s_nop 0", k_snop}, {"bitop3 x8", k_bitop3}, {"xor_b32 x8", k_xor},
        {"FIELD fe_mul 8x32 per op", k_field<0>}, {"FIELD fe_sqr 8x32 (x256)", k_field<1>},
        {"FIELD fe9_mul per op", k_field<2>}, {"FIELD fe9_sqr (x256)", k_field<3>},
        {"FIELD fe_add 8x32 per op", k_field<4>}, {"FIELD fe9_add+norm (x256)", k_field<5>},
        {"FIELD gej_dbl 8x32 per op", k_field<6>}, {"FIELD gej9_dbl (x256)", k_field<7>},
    };
    {
        hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, dc);
        CHECK(hipDeviceSynchronize());
        uint64_t hc[3];
        CHECK(hipMemcpy(hc, dc, sizeof(hc), hipMemcpyDeviceToHost));
        printf("s_memtime ticks %llu over %llu x 10 ns -> %.0f MHz\n", (unsigned long long)hc[0], (unsigned long long)hc[1], hc[0] / (hc[1] * 10e-3));
    }
    std::vector<uint64_t> h(cus * 4 * maxw);
    for (int w : {1, 2, 3, 4, 8}) {
        int grid = cus * w;  // 256-thread blocks = one wave per SIMD each
        printf("--- %d wave(s)/SIMD\n", w);
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, dc, d, 1u);
            CHECK(hipDeviceSynchronize());
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), 0, 0, dc, d, 2u);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(h.data(), dc, sizeof(uint64_t) * grid * 4, hipMemcpyDeviceToHost));
            std::vector<uint64_t> v(h.begin(), h.begin() + grid * 4);
            std::sort(v.begin(), v.end());
            double med = (double)v[v.size() / 2];
            double per = med / (LOOP * 32.0);
            printf("  %-26s %6.2f cycles/instr per wave   %6.2f per SIMD\n", k.name, per, per / w);
        }
    }
    return 0;
}
