// Microbenchmark: sustained VALU FMA throughput on gfx950 for v_fma_f32, v_pk_fma_f32 and
// v_fma_f64 (16 independent chains per lane, 8 waves per SIMD), to calibrate the roofline the
// sample loop is judged against.  Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_valu.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

// Inline asm pins the instruction form (hipcc would SLP-pack plain scalar fmaf chains).
__device__ __forceinline__ f2 fmaT(f2 a, f2 b, f2 c) {
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    return c;
}
__device__ __forceinline__ float fmaT(float a, float b, float c) {
    asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    return c;
}
__device__ __forceinline__ double fmaT(double a, double b, double c) {
    asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
    return c;
}

template <typename T>
__global__ __launch_bounds__(256) void chains(T* out, int iters, T a, T b) {
    T x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = (T)(threadIdx.x + j);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = fmaT(a, b, x[j]);
    }
    T s = x[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) s = s + x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename T>
static void run(const char* name, T a, T b, double flop_per_fma) {
    const int blocks = 256 * 8, threads = 256, iters = 4096;
    T* out;
    (void)hipMalloc(&out, sizeof(T) * blocks * threads);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    chains<T><<<blocks, threads>>>(out, iters, a, b);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) chains<T><<<blocks, threads>>>(out, iters, a, b);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double fmas = 5.0 * blocks * threads * (double)iters * 16;
    const double cyc = 2.4e9 * ms / 1e3;  // at 2.4 GHz
    printf("%-14s %8.3f ms  %8.2f TFLOP/s  %6.2f SIMD-cycles per wave-instruction (at 2.4 GHz)\n", name, ms,
           fmas * flop_per_fma / ms / 1e9, cyc * 1024.0 / (fmas / 64.0));
    (void)hipFree(out);
}

int main() {
    run<float>("v_fma_f32", 0.999f, 0.001f, 2.0);
    run<f2>("v_pk_fma_f32", f2{0.999f, 0.999f}, f2{0.001f, 0.001f}, 4.0);
    run<double>("v_fma_f64", 0.999, 0.001, 2.0);
    return 0;
}
