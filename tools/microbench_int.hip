// Integer VALU throughput micro-benchmark for gfx950 (MI355X).
// Measures per-instruction issue rate of the ops a 256-bit modular multiply is built from:
//   v_mad_u64_u32 (32x32+64 -> 64), v_mul_lo_u32, v_mul_hi_u32, v_add_co/addc chains,
//   v_bitop3_b32 / v_alignbit (Keccak), and a full 8x32-limb schoolbook product.
// Output: one line per op: lane-ops/s and ratio to the full-rate lane-op peak
// (256 CU x 4 SIMD x 32 lanes/clk x f_clk).  Used to fix roofline.peak in bench.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int CH = 8; // independent chains per lane

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 7 + seed;
    uint64_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = (uint64_t)(a + c) << 7;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint64_t t;
            asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %3" : "=v"(t) : "v"(a + c), "v"(b), "v"(acc[c]) : "s0", "s1");
            acc[c] = t;
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_mullo(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed | 1;
    uint32_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = a + c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint32_t t;
            asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(t) : "v"(acc[c]), "v"(a));
            acc[c] = t;
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed | 0x80000001u;
    uint32_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = a + c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint32_t t;
            asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(t) : "v"(acc[c]), "v"(a));
            acc[c] = t ^ a;
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_add32(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed;
    uint32_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = a + c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint32_t t;
            asm volatile("v_add_u32 %0, %1, %2" : "=v"(t) : "v"(acc[c]), "v"(a));
            acc[c] = t;
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addc(uint32_t* out, uint32_t seed) {
    // v_add_co_u32 + v_addc_co_u32 pairs (64-bit add), CH independent chains
    uint32_t a = threadIdx.x ^ seed;
    uint64_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = a + c;
    uint64_t b = ((uint64_t)seed << 32) | a;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) acc[c] += b;
    }
    uint64_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_bitop3(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed, b = seed * 3;
    uint32_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = a + c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint32_t t;
            asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(t) : "v"(acc[c]), "v"(a), "v"(b));
            acc[c] = t;
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_alignbit(uint32_t* out, uint32_t seed) {
    uint32_t a = threadIdx.x ^ seed;
    uint32_t acc[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = a + c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
            uint32_t t;
            asm volatile("v_alignbit_b32 %0, %1, %2, 7" : "=v"(t) : "v"(acc[c]), "v"(a));
            acc[c] = t;
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s ^= acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// full 8x8-limb schoolbook 256x256 -> 512, operand scanning in plain C (compiler codegen)
__global__ void k_mul256(uint32_t* out, uint32_t seed) {
    uint32_t a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; i++) { a[i] = (threadIdx.x + i * 0x9E3779B9u) ^ seed; b[i] = (blockIdx.x * 13 + i * 0x85EBCA6Bu) ^ seed; }
    for (int it = 0; it < ITERS / 64; it++) {
        uint32_t t[16];
#pragma unroll
        for (int i = 0; i < 16; i++) t[i] = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint64_t c = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) {
                uint64_t p = (uint64_t)a[i] * b[j] + t[i + j] + c;
                t[i + j] = (uint32_t)p;
                c = p >> 32;
            }
            t[i + 8] = (uint32_t)c;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) a[i] = t[i] ^ t[i + 8];
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint32_t*, uint32_t);

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    int cus = prop.multiProcessorCount;
    double clk = prop.clockRate * 1e3; // Hz
    printf("device %s CUs %d clock %.0f MHz\n", prop.gcnArchName, cus, clk / 1e6);
    const int block = 256, grid = cus * 8;
    uint32_t* d;
    CHECK(hipMalloc(&d, sizeof(uint32_t) * grid * block));
    struct { const char* name; kfn f; double ops_per_iter; } ks[] = {
        {"v_mad_u64_u32", k_mad64, (double)CH},
        {"v_mul_lo_u32", k_mullo, (double)CH},
        {"v_mul_hi_u32(+xor)", k_mulhi, (double)CH},
        {"v_add_u32", k_add32, (double)CH},
        {"add64(co+addc)", k_addc, (double)CH},
        {"v_bitop3_b32", k_bitop3, (double)CH},
        {"v_alignbit_b32", k_alignbit, (double)CH},
        {"mul256x256 (64 mads/iter)", k_mul256, 64.0 / 64.0},
    };
    double peak = (double)cus * 4 * 32 * clk;
    printf("full-rate lane-op peak at nominal clock: %.3e lane-ops/s\n", peak);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, d, 1u);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        const int reps = 5;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(block), 0, 0, d, (uint32_t)r);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        double ops = (double)grid * block * ITERS * k.ops_per_iter * reps;
        double rate = ops / (ms * 1e-3);
        printf("%-28s %.3e lane-ops/s  = %.3f of full-rate peak  (%.3f ms/launch)\n", k.name, rate, rate / peak, ms / reps);
    }
    return 0;
}
