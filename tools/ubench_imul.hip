// Issue cost of the 32x32->64 integer multiply Philox uses (v_mad_u64_u32) on gfx950, against
// v_fma_f32 and a plain integer add: 8 independent chains per lane, 8 waves per SIMD on every CU,
// timed with HIP events.  Each chain step is one op of the kind measured plus one v_xor_b32.
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_imul tools/ubench_imul.hip && tools/bin/ubench_imul
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr int kIters = 8192;

__global__ __launch_bounds__(256) void k_mad64(uint32_t* out, uint32_t seed) {
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * 8u + (uint32_t)j;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint64_t p = (uint64_t)x[j] * 0xD2511F53u;   // v_mad_u64_u32
            x[j] = (uint32_t)(p >> 32) ^ (uint32_t)p;
        }
    }
    uint32_t s = 0;
    for (int j = 0; j < 8; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(uint32_t* out, uint32_t seed) {
    uint32_t x[8];
    for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * 8u + (uint32_t)j;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t p = x[j] + 0xD2511F53u;   // v_add_u32
            x[j] = (p >> 7) ^ p;                     // v_lshrrev + v_xor (v_xad / v_lshr_xor)
        }
    }
    uint32_t s = 0;
    for (int j = 0; j < 8; ++j) s ^= x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma(float* out, float seed) {
    float x[8];
    for (int j = 0; j < 8; ++j) x[j] = seed + threadIdx.x * 1e-3f + (float)j;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = __builtin_fmaf(x[j], 0.999f, 1e-4f);   // v_fma_f32
    }
    float s = 0;
    for (int j = 0; j < 8; ++j) s += x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    int dev = 0, ncu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = ncu * 8;   // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    uint32_t* buf = nullptr;
    hipMalloc(&buf, (size_t)blocks * 256 * sizeof(uint32_t));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch, double ops_per_step) {
        launch();   // warm-up
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double wave_steps = 5.0 * blocks * 4 * (double)kIters * 8;   // per wave: kIters x 8 chain steps
        const double ns_per_step_per_simd = ms * 1e6 / (wave_steps / (ncu * 4.0));
        printf("%-6s %8.3f ms  %.3f ns per wave chain-step per SIMD (%.0f instr per step)\n", name, ms,
               ns_per_step_per_simd, ops_per_step);
    };
    run("mad64", [&] { k_mad64<<<blocks, 256>>>(buf, 1u); }, 2);
    run("add", [&] { k_add<<<blocks, 256>>>(buf, 1u); }, 3);
    run("fma", [&] { k_fma<<<blocks, 256>>>((float*)buf, 1.0f); }, 1);
    hipFree(buf);
    return 0;
}
