// Microbenchmark: issue cost of the integer instructions the counter-based RNG (Philox4x32-10) uses
// on gfx950, and of whole Philox blocks as compiled vs with v_bitop3_b32 (xor3): 16 independent chains per
// lane, 8 waves per SIMD.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_int tools/probe/ubench_int.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int OP> __device__ __forceinline__ uint32_t op(uint32_t x, uint32_t k) {
    if constexpr (OP == 0) { uint64_t r; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "s"(k) : "vcc"); return (uint32_t)r ^ (uint32_t)(r >> 32); }
    if constexpr (OP == 1) { asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "s"(k)); return x; }
    if constexpr (OP == 2) { asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "s"(k)); return x; }
    if constexpr (OP == 3) { asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(x) : "s"(k)); return x; }
    if constexpr (OP == 4) { asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "s"(k)); return x; }
    if constexpr (OP == 5) { asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(x) : "s"(k)); return x; }
    if constexpr (OP == 6) { uint64_t r; asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(x), "s"(k) : "vcc"); return (uint32_t)r; }
    return x;
}

template <int OP>
__global__ __launch_bounds__(256) void chains(uint32_t* out, int iters, uint32_t k) {
    uint32_t x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = threadIdx.x * 16 + j;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = op<OP>(x[j], k);
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

struct U4 { uint32_t a, b, c, d; };
template <bool X3>
__device__ __forceinline__ U4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0, n2;
        if constexpr (X3) {
            n0 = __builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c1, k0, 0x96);   // a ^ b ^ c
            n2 = __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c3, k1, 0x96);
        } else {
            n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
            n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        }
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return U4{c0, c1, c2, c3};
}
template <bool X3>
__global__ __launch_bounds__(256) void blocks(uint32_t* out, int iters, uint32_t k0, uint32_t k1) {
    U4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = U4{threadIdx.x, (uint32_t)j, blockIdx.x, 0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = philox<X3>(acc[j].a, acc[j].b, acc[j].c, acc[j].d, k0 + i, k1);
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) s ^= acc[j].a ^ acc[j].b ^ acc[j].c ^ acc[j].d;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const int kBlocks = 256 * 8, kThreads = 256;
template <typename F>
static void timeit(const char* name, F launch, double wave_insts) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double cyc = 2.4e9 * ms / 1e3;
    printf("%-22s %8.3f ms  %7.2f SIMD-cycles per wave-unit (at 2.4 GHz)\n", name, ms, cyc * 1024.0 / (5.0 * wave_insts));
}

int main() {
    uint32_t* out;
    (void)hipMalloc(&out, sizeof(uint32_t) * kBlocks * kThreads);
    const int iters = 4096;
    const double n = (double)kBlocks * kThreads / 64.0 * iters * 16;   // wave-instructions per launch
    timeit("v_mad_u64_u32 (+xor)", [&] { chains<0><<<kBlocks, kThreads>>>(out, iters, 0xD2511F53u); }, n);
    timeit("v_mad_u64_u32", [&] { chains<6><<<kBlocks, kThreads>>>(out, iters, 0xD2511F53u); }, n);
    timeit("v_mul_lo_u32", [&] { chains<1><<<kBlocks, kThreads>>>(out, iters, 0xD2511F53u); }, n);
    timeit("v_mul_hi_u32", [&] { chains<2><<<kBlocks, kThreads>>>(out, iters, 0xD2511F53u); }, n);
    timeit("v_bitop3_b32 (xor3)", [&] { chains<3><<<kBlocks, kThreads>>>(out, iters, 0xD2511F53u); }, n);
    timeit("v_xor_b32", [&] { chains<4><<<kBlocks, kThreads>>>(out, iters, 0xD2511F53u); }, n);
    timeit("v_mul_u32_u24", [&] { chains<5><<<kBlocks, kThreads>>>(out, iters, 0xD2511F53u); }, n);
    const int bi = 256;
    const double nb = (double)kBlocks * kThreads / 64.0 * bi * 4;   // wave Philox blocks per launch
    timeit("philox block (xor)", [&] { blocks<false><<<kBlocks, kThreads>>>(out, bi, 1u, 2u); }, nb);
    timeit("philox block (bitop3)", [&] { blocks<true><<<kBlocks, kThreads>>>(out, bi, 1u, 2u); }, nb);
    (void)hipFree(out);
    return 0;
}
