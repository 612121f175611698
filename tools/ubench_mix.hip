// Microbenchmark: sustained issue cost (SIMD-cycles per wave-instruction) of the VALU instruction kinds the
// sample loop issues, on gfx950: 16 independent chains per lane, 8 waves per SIMD, one kernel per kind, so
// a rocprofv3 --pmc pass over it also shows which SQ_INSTS_VALU_* class counts each kind and how often
// (tools/mix_pass.sh).  Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_mix tools/ubench_mix.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

#define KIND(NAME, T, ASM, CON)                                                                        \
    struct NAME {                                                                                      \
        typedef T type;                                                                                \
        static constexpr const char* name = #NAME;                                                     \
        __device__ __forceinline__ static void op(T& x, T a) { asm volatile(ASM : "+v"(x) : CON(a)); } \
    };
#define VC(a) "v"(a)
KIND(fma_f32, float, "v_fma_f32 %0, %1, %0, %1", VC)
KIND(pk_fma_f32, f2, "v_pk_fma_f32 %0, %1, %0, %1", VC)
KIND(fma_f64, double, "v_fma_f64 %0, %1, %0, %1", VC)
KIND(mul_f32, float, "v_mul_f32 %0, %1, %0", VC)
KIND(sqrt_f32, float, "v_sqrt_f32 %0, %0", VC)
KIND(rsq_f32, float, "v_rsq_f32 %0, %0", VC)
KIND(rsq_f64, double, "v_rsq_f64 %0, %0", VC)
KIND(add_u32, uint32_t, "v_add_u32 %0, %1, %0", VC)
KIND(bitop3, uint32_t, "v_bitop3_b32 %0, %1, %0, %1 bitop3:0x96", VC)
KIND(cvt_f32_u32, float, "v_cvt_f32_u32 %0, %0", VC)
KIND(cndmask, uint32_t, "v_cndmask_b32 %0, %1, %0, vcc", VC)
KIND(mov_b32, uint32_t, "v_mov_b32 %0, %1", VC)
KIND(and_b32, uint32_t, "v_and_b32 %0, %1, %0", VC)
KIND(max3_f32, float, "v_max3_f32 %0, %1, %0, %0", VC)
KIND(add_f32, float, "v_add_f32 %0, %1, %0", VC)
KIND(pk_add_f32, f2, "v_pk_add_f32 %0, %1, %0", VC)
KIND(pk_mul_f32, f2, "v_pk_mul_f32 %0, %1, %0", VC)
KIND(fma_f64_abc, double, "v_fma_f64 %0, %1, %0, %0", VC)
KIND(add_f64, double, "v_add_f64 %0, %1, %0", VC)

struct fma_f32_abc {   // three distinct source registers (no repeated operand)
    typedef float type;
    static constexpr const char* name = "fma_f32_abc";
    __device__ __forceinline__ static void op(float& x, float a) {
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(a * 0.5f));
    }
};
struct cndmask_s {   // the mask from an SGPR pair (e64), as the kernel's selects
    typedef uint32_t type;
    static constexpr const char* name = "cndmask_sgpr";
    __device__ __forceinline__ static void op(uint32_t& x, uint32_t a) {
        asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(x) : "v"(a), "s"(0x5555555555555555ull));
    }
};
struct cmp_e64 {   // a compare into an SGPR pair (the kernel's lane-mask compares)
    typedef float type;
    static constexpr const char* name = "cmp_e64";
    __device__ __forceinline__ static void op(float& x, float a) {
        asm volatile("v_cmp_gt_f32_e64 s[2:3], %0, %1" : "+v"(x) : "v"(a) : "s2", "s3");
    }
};
struct mad_u64 {
    typedef uint64_t type;
    static constexpr const char* name = "mad_u64_u32";
    __device__ __forceinline__ static void op(uint64_t& x, uint64_t a) {
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(x) : "v"((uint32_t)a) : "s0", "s1");
    }
};

template <typename K>
__global__ __launch_bounds__(256) void chains(typename K::type* out, int iters, typename K::type a) {
    typedef typename K::type T;
    T x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = a;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) K::op(x[j], a);
    }
    T s = x[0];
#pragma unroll
    for (int j = 1; j < 16; ++j) s = s + x[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(typename K::type a) {
    typedef typename K::type T;
    const int blocks = 256 * 8, threads = 256, iters = 8192;
    T* out;
    (void)hipMalloc(&out, sizeof(T) * blocks * threads);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    chains<K><<<blocks, threads>>>(out, iters, a);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) chains<K><<<blocks, threads>>>(out, iters, a);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winst = 3.0 * blocks * threads / 64.0 * iters * 16;   // wave-instructions
    printf("%-12s %8.3f ms  %6.2f SIMD-cycles per wave-instruction (at 2.4 GHz, 1024 SIMDs)\n", K::name, ms,
           2.4e9 * ms / 1e3 * 1024.0 / winst);
    (void)hipFree(out);
}

int main() {
    for (int w = 0; w < 4; ++w) run<fma_f32>(0.999f);   // clocks up (the first lines read low)
    run<fma_f32>(0.999f);
    run<pk_fma_f32>(f2{0.999f, 0.999f});
    run<fma_f64>(0.999);
    run<mul_f32>(0.999f);
    run<sqrt_f32>(1.5f);
    run<rsq_f32>(1.5f);
    run<rsq_f64>(1.5);
    run<add_u32>(3u);
    run<bitop3>(3u);
    run<cvt_f32_u32>(3.0f);
    run<cndmask>(3u);
    run<cndmask_s>(3u);
    run<fma_f32_abc>(0.999f);
    run<mad_u64>(3ull);
    run<mov_b32>(3u);
    run<and_b32>(3u);
    run<max3_f32>(0.5f);
    run<add_f32>(0.5f);
    run<pk_add_f32>(f2{0.5f, 0.5f});
    run<pk_mul_f32>(f2{0.999f, 0.999f});
    run<fma_f64_abc>(0.999);
    run<add_f64>(0.5);
    run<cmp_e64>(0.5f);
    return 0;
}
