// Cycles per wave-instruction of the VALU ops the secp256k1 / BN254 field code is made of, on gfx950,
// measured in shader cycles (s_memtime around the loop, so DVFS does not enter) at 1, 2 and 3 waves
// per SIMD, 8 independent chains per lane on random operands.  The per-SIMD cost of one
// wave-instruction = wave cycles x waves per SIMD / instructions per wave (the co-resident waves share
// the SIMD's issue).  Used to price instruction choices in tools/gen_fe9_asm.py.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_mix.hip -o tools/microbench_mix
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);        \
            return 1;                                                              \
        }                                                                          \
    } while (0)

constexpr int ITERS = 2048;
constexpr int CH = 8;

// OP(d, a, b): one instruction on 32-bit (or 64-bit pair) chain values
#define BENCH32(NAME, ASM)                                                                         \
    __global__ void NAME(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,             \
                         uint64_t* __restrict__ cyc) {                                             \
        uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;                                         \
        uint32_t x[CH], b = in[(t * 7 + 3) & 4095] | 1u;                                            \
        for (int c = 0; c < CH; c++) x[c] = in[(t + 97 * c) & 4095];                                \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                                 \
        for (int i = 0; i < ITERS; i++) {                                                           \
            _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(x[c]) : "v"(b)); \
        }                                                                                           \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                                 \
        uint32_t s = 0;                                                                             \
        for (int c = 0; c < CH; c++) s ^= x[c];                                                     \
        out[t] = s;                                                                                 \
        if ((threadIdx.x & 63) == 0) cyc[t >> 6] = t1 - t0;                                         \
    }
#define BENCH64(NAME, ASM)                                                                         \
    __global__ void NAME(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,             \
                         uint64_t* __restrict__ cyc) {                                             \
        uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;                                         \
        uint64_t x[CH];                                                                             \
        uint32_t b = in[(t * 7 + 3) & 4095] | 1u;                                                   \
        for (int c = 0; c < CH; c++) x[c] = ((uint64_t)in[(t + 31 * c) & 4095] << 32) | in[(t + 97 * c) & 4095]; \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                                 \
        for (int i = 0; i < ITERS; i++) {                                                           \
            _Pragma("unroll") for (int c = 0; c < CH; c++) asm volatile(ASM : "+v"(x[c]) : "v"(b)); \
        }                                                                                           \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                                 \
        uint64_t s = 0;                                                                             \
        for (int c = 0; c < CH; c++) s ^= x[c];                                                     \
        out[t] = (uint32_t)s ^ (uint32_t)(s >> 32);                                                 \
        if ((threadIdx.x & 63) == 0) cyc[t >> 6] = t1 - t0;                                         \
    }

__global__ void k_mad64(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint64_t* __restrict__ cyc) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t x[CH];
    uint32_t b = in[(t * 7 + 3) & 4095] | 1u, a = in[(t * 5 + 1) & 4095];
    for (int c = 0; c < CH; c++) x[c] = ((uint64_t)in[(t + 31 * c) & 4095] << 32) | in[(t + 97 * c) & 4095];
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(x[c]) : "v"(a), "v"(b) : "s0", "s1");
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint64_t s = 0;
    for (int c = 0; c < CH; c++) s ^= x[c];
    out[t] = (uint32_t)s ^ (uint32_t)(s >> 32);
    if ((threadIdx.x & 63) == 0) cyc[t >> 6] = t1 - t0;
}
BENCH64(k_shr64, "v_lshrrev_b64 %0, 29, %0")
BENCH64(k_shl64, "v_lshlrev_b64 %0, 13, %0")
BENCH64(k_lshladd64, "v_lshl_add_u64 %0, %0, 2, %0")
BENCH64(k_mov64, "v_mov_b64 %0, %0")
BENCH32(k_and32, "v_and_b32 %0, 0x1fffffff, %0")
BENCH32(k_add32, "v_add_u32 %0, %0, %1")
BENCH32(k_add3, "v_add3_u32 %0, %0, %1, %0")
BENCH32(k_mov32, "v_mov_b32 %0, %0")
BENCH32(k_shr32, "v_lshrrev_b32 %0, 29, %0")
BENCH32(k_alignbit, "v_alignbit_b32 %0, %1, %0, 29")
BENCH32(k_mad24, "v_mad_u32_u24 %0, %0, %1, %0")
BENCH32(k_mullo, "v_mul_lo_u32 %0, %0, %1")
BENCH32(k_bfe, "v_bfe_u32 %0, %0, 3, 29")
BENCH32(k_bitop3, "v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96")
BENCH32(k_cndmask, "v_cmp_gt_u32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc")
BENCH32(k_pkadd16, "v_pk_add_u16 %0, %0, %1")
BENCH32(k_dot2u16, "v_dot2_u32_u16 %0, %0, %1, %0")

typedef void (*kfn)(const uint32_t*, uint32_t*, uint64_t*);

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    printf("device %s CUs %d\n", prop.gcnArchName, cus);
    std::vector<uint32_t> h(4096);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    for (auto& v : h) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        v = (uint32_t)s;
    }
    uint32_t *d_in, *d_out;
    uint64_t* d_cyc;
    const int maxw = 3, block = 256;
    const int maxblocks = cus * maxw;  // 256-thread block = 4 waves = one per SIMD
    CHECK(hipMalloc(&d_in, 4096 * 4));
    CHECK(hipMalloc(&d_out, (size_t)maxblocks * block * 4));
    CHECK(hipMalloc(&d_cyc, (size_t)maxblocks * 4 * 8));
    CHECK(hipMemcpy(d_in, h.data(), 4096 * 4, hipMemcpyHostToDevice));
    struct {
        const char* name;
        kfn f;
        int instr;  // VALU instructions per chain step
    } ks[] = {
        {"v_mad_u64_u32", k_mad64, 1}, {"v_lshrrev_b64", k_shr64, 1}, {"v_lshlrev_b64", k_shl64, 1},
        {"v_lshl_add_u64", k_lshladd64, 1}, {"v_mov_b64", k_mov64, 1}, {"v_and_b32", k_and32, 1},
        {"v_add_u32", k_add32, 1}, {"v_add3_u32", k_add3, 1}, {"v_mov_b32", k_mov32, 1},
        {"v_lshrrev_b32", k_shr32, 1}, {"v_alignbit_b32", k_alignbit, 1}, {"v_mad_u32_u24", k_mad24, 1},
        {"v_mul_lo_u32", k_mullo, 1}, {"v_bfe_u32", k_bfe, 1}, {"v_bitop3_b32", k_bitop3, 1},
        {"v_cmp+v_cndmask", k_cndmask, 2}, {"v_pk_add_u16", k_pkadd16, 1}, {"v_dot2_u32_u16", k_dot2u16, 1},
    };
    std::vector<uint64_t> cyc((size_t)maxblocks * 4);
    printf("%-18s %s\n", "instruction", "SIMD cycles per wave-instruction at 1 / 2 / 3 waves per SIMD (median wave)");
    for (auto& k : ks) {
        printf("%-18s", k.name);
        for (int w = 1; w <= maxw; w++) {
            int blocks = cus * w;
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(block), 0, 0, d_in, d_out, d_cyc);  // warm
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(block), 0, 0, d_in, d_out, d_cyc);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(cyc.data(), d_cyc, (size_t)blocks * 4 * 8, hipMemcpyDeviceToHost));
            std::vector<uint64_t> v(cyc.begin(), cyc.begin() + (size_t)blocks * 4);
            std::sort(v.begin(), v.end());
            double med = (double)v[v.size() / 2];
            double per = med * w / ((double)ITERS * CH * k.instr);
            printf("  %6.2f", per);
        }
        printf("\n");
    }
    return 0;
}
