// Throughput of secp256k1 field / group code on gfx950 as a function of waves per SIMD, with the
// occupancy FORCED by each workgroup's LDS allocation (160 KiB / W per 256-thread block, so at
// most W blocks = W waves per SIMD fit on a CU) and timed over the whole launch with HIP events
// (many blocks per CU: dispatch skew averages out).  microbench_lat.hip times each wave with
// s_memtime at a nominal occupancy it does not enforce; this one measures what a kernel gets.
//
// Reported per kernel and W: SIMD-cycles per operation at the nominal 2.4 GHz
// (= elapsed x 2.4e9 x SIMDs / total wave-operations) and the lane-operation rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../geth-sharding_amd/csrc/secp256k1_fe9.cuh"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int OPS = 64;

#define R4(x) x x x x
#define R8(x) R4(x) R4(x)
#define R32(x) R8(x) R8(x) R8(x) R8(x)

// MODE 0: fe9_mul chain, 1: fe9_sqr chain, 2: gej9_dbl chain, 3: 32 independent v_mad_u64_u32 (asm),
// 4: 32 independent v_add_u32 (asm), 5: mixed-add gej9_add_ge_core chain, 6: v_lshrrev_b64,
// 7: v_alignbit_b32, 8: v_and_b32 with a literal, 9: a dependent mad / 64-bit shift chain
template <int MODE>
__global__ __launch_bounds__(256) void k_occ(uint32_t* out, uint32_t seed) {
    extern __shared__ uint32_t lds[];
    if (threadIdx.x == 0) lds[0] = seed;  // the allocation holds the occupancy; touch it once
    gsv::fe9 a9, b9;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        a9.v[i] = ((threadIdx.x + i * 0x9E3779B9u) ^ seed) & gsv::M29;
        b9.v[i] = ((blockIdx.x * 13 + i * 0x85EBCA6Bu) ^ seed) & gsv::M29;
    }
    uint64_t x0 = a9.v[0], x1 = a9.v[1], x2 = a9.v[2], x3 = a9.v[3], x4 = a9.v[4], x5 = a9.v[5], x6 = a9.v[6], x7 = a9.v[7];
    uint32_t y0 = b9.v[0], y1 = b9.v[1];
    for (int it = 0; it < OPS; it++) {
        if (MODE == 0) gsv::fe9_mul(a9, a9, b9);
        else if (MODE == 1) gsv::fe9_sqr(a9, a9);
        else if (MODE == 2) { gsv::gej9 g; g.x = a9; g.y = b9; g.z = a9; gsv::gej9_dbl(g, g); a9 = g.x; b9 = g.y; }
        else if (MODE == 3) {
            asm volatile(R4("v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_mad_u64_u32 %1, vcc, %8, %9, %1\n\t"
                            "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\tv_mad_u64_u32 %3, vcc, %8, %9, %3\n\t"
                            "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\tv_mad_u64_u32 %5, vcc, %8, %9, %5\n\t"
                            "v_mad_u64_u32 %6, vcc, %8, %9, %6\n\tv_mad_u64_u32 %7, vcc, %8, %9, %7\n\t")
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
                         : "v"(y0), "v"(y1) : "vcc");
        } else if (MODE == 4) {
            asm volatile(R4("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                            "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t")
                         : "+v"(a9.v[0]), "+v"(a9.v[1]), "+v"(a9.v[2]), "+v"(a9.v[3]), "+v"(a9.v[4]), "+v"(a9.v[5]),
                           "+v"(a9.v[6]), "+v"(a9.v[7])
                         : "v"(y0));
        } else if (MODE == 6) {
            asm volatile(R4("v_lshrrev_b64 %0, 29, %0\n\tv_lshrrev_b64 %1, 29, %1\n\tv_lshrrev_b64 %2, 29, %2\n\tv_lshrrev_b64 %3, 29, %3\n\t"
                            "v_lshrrev_b64 %4, 29, %4\n\tv_lshrrev_b64 %5, 29, %5\n\tv_lshrrev_b64 %6, 29, %6\n\tv_lshrrev_b64 %7, 29, %7\n\t")
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
        } else if (MODE == 7) {
            asm volatile(R4("v_alignbit_b32 %0, %0, %8, 29\n\tv_alignbit_b32 %1, %1, %8, 29\n\tv_alignbit_b32 %2, %2, %8, 29\n\tv_alignbit_b32 %3, %3, %8, 29\n\t"
                            "v_alignbit_b32 %4, %4, %8, 29\n\tv_alignbit_b32 %5, %5, %8, 29\n\tv_alignbit_b32 %6, %6, %8, 29\n\tv_alignbit_b32 %7, %7, %8, 29\n\t")
                         : "+v"(a9.v[0]), "+v"(a9.v[1]), "+v"(a9.v[2]), "+v"(a9.v[3]), "+v"(a9.v[4]), "+v"(a9.v[5]),
                           "+v"(a9.v[6]), "+v"(a9.v[7])
                         : "v"(y0));
        } else if (MODE == 8) {
            asm volatile(R4("v_and_b32_e32 %0, 0x1fffffff, %8\n\tv_and_b32_e32 %1, 0x1fffffff, %8\n\tv_and_b32_e32 %2, 0x1fffffff, %8\n\tv_and_b32_e32 %3, 0x1fffffff, %8\n\t"
                            "v_and_b32_e32 %4, 0x1fffffff, %8\n\tv_and_b32_e32 %5, 0x1fffffff, %8\n\tv_and_b32_e32 %6, 0x1fffffff, %8\n\tv_and_b32_e32 %7, 0x1fffffff, %8\n\t")
                         : "+v"(a9.v[0]), "+v"(a9.v[1]), "+v"(a9.v[2]), "+v"(a9.v[3]), "+v"(a9.v[4]), "+v"(a9.v[5]),
                           "+v"(a9.v[6]), "+v"(a9.v[7])
                         : "v"(y0));
        } else if (MODE >= 10 && MODE <= 17) {  // 32-bit bit ops of the Keccak rounds and their alternatives
#define OP8(ins) asm volatile(R4(ins " %0, %0, %8, %9\n\t" ins " %1, %1, %8, %9\n\t" ins " %2, %2, %8, %9\n\t"   \
                                     ins " %3, %3, %8, %9\n\t" ins " %4, %4, %8, %9\n\t" ins " %5, %5, %8, %9\n\t"   \
                                     ins " %6, %6, %8, %9\n\t" ins " %7, %7, %8, %9\n\t")                             \
                              : "+v"(a9.v[0]), "+v"(a9.v[1]), "+v"(a9.v[2]), "+v"(a9.v[3]), "+v"(a9.v[4]),        \
                                "+v"(a9.v[5]), "+v"(a9.v[6]), "+v"(a9.v[7])                                       \
                              : "v"(y0), "v"(y1))
#define OP8_2(ins) asm volatile(R4(ins " %0, %0, %8\n\t" ins " %1, %1, %8\n\t" ins " %2, %2, %8\n\t"             \
                                     ins " %3, %3, %8\n\t" ins " %4, %4, %8\n\t" ins " %5, %5, %8\n\t"             \
                                     ins " %6, %6, %8\n\t" ins " %7, %7, %8\n\t")                                   \
                              : "+v"(a9.v[0]), "+v"(a9.v[1]), "+v"(a9.v[2]), "+v"(a9.v[3]), "+v"(a9.v[4]),        \
                                "+v"(a9.v[5]), "+v"(a9.v[6]), "+v"(a9.v[7])                                       \
                              : "v"(y0))
            if (MODE == 10) OP8_2("v_xor_b32_e32");
            else if (MODE == 11) OP8_2("v_xor_b32_e64");
            else if (MODE == 12) {
                asm volatile(R4("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %9 bitop3:0x96\n\t"
                                "v_bitop3_b32 %2, %2, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %3, %3, %8, %9 bitop3:0x96\n\t"
                                "v_bitop3_b32 %4, %4, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %8, %9 bitop3:0x96\n\t"
                                "v_bitop3_b32 %6, %6, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %8, %9 bitop3:0x96\n\t")
                             : "+v"(a9.v[0]), "+v"(a9.v[1]), "+v"(a9.v[2]), "+v"(a9.v[3]), "+v"(a9.v[4]), "+v"(a9.v[5]),
                               "+v"(a9.v[6]), "+v"(a9.v[7])
                             : "v"(y0), "v"(y1));
            } else if (MODE == 13) OP8("v_or3_b32");
            else if (MODE == 14) OP8("v_bfi_b32");
            else if (MODE == 15) OP8("v_perm_b32");
            else if (MODE == 16) OP8("v_alignbyte_b32");
            else OP8("v_add3_u32");
#undef OP8
#undef OP8_2
        } else if (MODE == 9) {  // the mul's mix: 4 mads + 1 64-bit shift + 1 and, dependent as in a column
            asm volatile(R4("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %0, vcc, %3, %2, %0\n\t"
                            "v_mad_u64_u32 %0, vcc, %2, %2, %0\n\tv_mad_u64_u32 %0, vcc, %3, %3, %0\n\t"
                            "v_lshrrev_b64 %1, 29, %0\n\tv_mad_u64_u32 %1, vcc, %2, %3, %1\n\t"
                            "v_mad_u64_u32 %1, vcc, %3, %2, %1\n\tv_lshrrev_b64 %0, 29, %1\n\t")
                         : "+v"(x0), "+v"(x1) : "v"(y0), "v"(y1) : "vcc");
        } else {
            gsv::gej9 p, o; gsv::ge9 q; gsv::fe9 h, rr;
            p.x = a9; p.y = b9; p.z = a9; q.x = b9; q.y = a9;
            gsv::gej9_add_ge_core(o, h, rr, p, q);
            a9 = o.x; b9 = o.z;
        }
    }
    uint32_t s = (uint32_t)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7) ^ (uint32_t)((x0 ^ x7) >> 32);
#pragma unroll
    for (int i = 0; i < 9; i++) s ^= a9.v[i] ^ b9.v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    int simds = cus * 4;
    printf("device %s CUs %d  LDS/CU 160 KiB; occupancy forced by dynamic LDS per 256-thread block\n", prop.gcnArchName, cus);
    struct { const char* name; kfn f; double ops_per_iter; } ks[] = {
        {"fe9_mul chain", k_occ<0>, 1}, {"fe9_sqr chain", k_occ<1>, 1}, {"gej9_dbl chain", k_occ<2>, 1},
        {"gej9 mixed add (core)", k_occ<5>, 1},
        {"v_mad_u64_u32 x8 indep", k_occ<3>, 32}, {"v_add_u32 x8 indep", k_occ<4>, 32},
        {"v_lshrrev_b64 x8 indep", k_occ<6>, 32}, {"v_alignbit_b32 x8 indep", k_occ<7>, 32},
        {"v_and_b32 lit x8 indep", k_occ<8>, 32}, {"mad/lshr64 dep chain", k_occ<9>, 32},
        {"v_xor_b32 (VOP2) x8", k_occ<10>, 32}, {"v_xor_b32_e64 (VOP3) x8", k_occ<11>, 32},
        {"v_bitop3_b32 x8", k_occ<12>, 32}, {"v_or3_b32 x8", k_occ<13>, 32}, {"v_bfi_b32 x8", k_occ<14>, 32},
        {"v_perm_b32 x8", k_occ<15>, 32}, {"v_alignbyte_b32 x8", k_occ<16>, 32}, {"v_add3_u32 x8", k_occ<17>, 32},
    };
    for (auto& k : ks) CHECK(hipFuncSetAttribute((const void*)k.f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    int rounds = 16;
    uint32_t* d;
    CHECK(hipMalloc(&d, sizeof(uint32_t) * (size_t)cus * 8 * rounds * 256));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto& k : ks) {
        printf("%-24s", k.name);
        for (int w : {1, 2, 3, 4, 5, 6, 8}) {
            size_t lds = (160 * 1024) / w - 512;
            int grid = cus * w * rounds;
            hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), lds, 0, d, 1u);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(256), lds, 0, d, 2u + rep);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            double wave_ops = 3.0 * grid * 4 * OPS * k.ops_per_iter;
            double cyc = ms * 1e-3 * 2.4e9 * simds / wave_ops;
            printf("  W%d %8.2f", w, cyc);
        }
        printf("   (SIMD-cycles per op)\n");
    }
    return 0;
}
