// Microbenchmark: VGPR operand-read cost of 3-source VALU ops on gfx950 (SIMD-cycles per wave-instruction):
// one asm block of 16 independent instructions on fixed registers per loop step, 8 waves per SIMD.
// Distinct source banks (register index mod 4) against a repeated source (a square: x * x + y) and sources
// in one bank.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_bank tools/ubench_bank.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R16(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7) I(8) I(9) I(10) I(11) I(12) I(13) I(14) I(15)
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67",  \
             "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79"
// destinations v44 + 2j (j = 0..15: v44..v74, banks 0 and 2); sources v41 (bank 1), v42 (bank 2), v43 (bank 3), v40 (bank 0)
#define I_ABC(j) "v_fma_f32 v" #j "0, v41, v43, v" #j "0\n"
template <int K>
__global__ __launch_bounds__(256) void bank(float* out, int iters) {
    asm volatile("v_mov_b32 v40, 1.0\n v_mov_b32 v41, 1.0\n v_mov_b32 v42, 1.0\n v_mov_b32 v43, 1.0\n"
                 "v_mov_b32 v44, 1.0\n v_mov_b32 v46, 1.0\n v_mov_b32 v48, 1.0\n v_mov_b32 v50, 1.0\n"
                 "v_mov_b32 v52, 1.0\n v_mov_b32 v54, 1.0\n v_mov_b32 v56, 1.0\n v_mov_b32 v58, 1.0\n"
                 "v_mov_b32 v60, 1.0\n v_mov_b32 v62, 1.0\n v_mov_b32 v64, 1.0\n v_mov_b32 v66, 1.0\n"
                 "v_mov_b32 v68, 1.0\n v_mov_b32 v70, 1.0\n v_mov_b32 v72, 1.0\n v_mov_b32 v74, 1.0\n"
                 "v_mov_b32 v45, 1.0\n v_mov_b32 v47, 1.0\n v_mov_b32 v49, 1.0\n v_mov_b32 v51, 1.0\n"
                 "v_mov_b32 v53, 1.0\n v_mov_b32 v55, 1.0\n v_mov_b32 v57, 1.0\n v_mov_b32 v59, 1.0\n"
                 "v_mov_b32 v61, 1.0\n v_mov_b32 v63, 1.0\n v_mov_b32 v65, 1.0\n v_mov_b32 v67, 1.0\n"
                 "v_mov_b32 v69, 1.0\n v_mov_b32 v71, 1.0\n v_mov_b32 v73, 1.0\n v_mov_b32 v75, 1.0\n" ::: CLOB);
    for (int i = 0; i < iters; ++i) {
#define D(j) "v" #j
        if constexpr (K == 0)   // fma, sources in banks 1, 3 + accumulator (bank 0/2)
            asm volatile(
#define X(j) "v_fma_f32 v[44+2*" #j "], v41, v43, v[44+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 1)   // square-accumulate: x * x + acc (one source read twice)
            asm volatile(
#define X(j) "v_fma_f32 v[44+2*" #j "], v41, v41, v[44+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 2)   // all three sources in bank 0 (v40, v44+4k, v48+4k)
            asm volatile(
#define X(j) "v_fma_f32 v[44+2*" #j "], v40, v40, v[44+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 3)   // packed, distinct banks: {v44,v45}.. = {v42,v43} * {v40,v41} + acc
            asm volatile(
#define X(j) "v_pk_fma_f32 v[44+2*" #j ":45+2*" #j "], v[42:43], v[40:41], v[44+2*" #j ":45+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 4)   // packed square-accumulate
            asm volatile(
#define X(j) "v_pk_fma_f32 v[44+2*" #j ":45+2*" #j "], v[42:43], v[42:43], v[44+2*" #j ":45+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 5)   // mul square: x * x (two sources, one register)
            asm volatile(
#define X(j) "v_mul_f32 v[44+2*" #j "], v41, v41\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 6)   // mul, distinct
            asm volatile(
#define X(j) "v_mul_f32 v[44+2*" #j "], v41, v42\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 7)   // fma with the accumulator read in the same bank as a source (v44.. bank 0, v40 bank 0)
            asm volatile(
#define X(j) "v_fma_f32 v[44+2*" #j "], v40, v41, v[44+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 8)   // select on an SGPR-pair mask, distinct sources
            asm volatile(
#define X(j) "v_cndmask_b32_e64 v[44+2*" #j "], v41, v42, s[20:21]\n"
                R16(X) ::: CLOB, "s20", "s21");
#undef X
        if constexpr (K == 9)   // compare into an SGPR pair
            asm volatile(
#define X(j) "v_cmp_lt_f32_e64 s[20+2*(" #j "&3):21+2*(" #j "&3)], v41, v[44+2*" #j "]\n"
                R16(X) ::: CLOB, "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
#undef X
        if constexpr (K == 10)   // move
            asm volatile(
#define X(j) "v_mov_b32 v[44+2*" #j "], v41\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 11)   // two-source logic
            asm volatile(
#define X(j) "v_and_b32 v[44+2*" #j "], v41, v[44+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 12)   // three-source logic, distinct banks
            asm volatile(
#define X(j) "v_bitop3_b32 v[44+2*" #j "], v41, v43, v[44+2*" #j "] bitop3:0x96\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 13)   // fp64 add
            asm volatile(
#define X(j) "v_add_f64 v[44+2*" #j ":45+2*" #j "], v[42:43], v[44+2*" #j ":45+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 14)   // fp64 mul
            asm volatile(
#define X(j) "v_mul_f64 v[44+2*" #j ":45+2*" #j "], v[42:43], v[44+2*" #j ":45+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 15)   // fp64 fma, distinct banks
            asm volatile(
#define X(j) "v_fma_f64 v[44+2*" #j ":45+2*" #j "], v[42:43], v[40:41], v[44+2*" #j ":45+2*" #j "]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 16)   // compare into VCC (VOP2/VOPC encoding)
            asm volatile(
#define X(j) "v_cmp_lt_f32_e32 vcc, v41, v[44+2*" #j "]\n"
                R16(X) ::: CLOB, "vcc");
#undef X
        if constexpr (K == 17)   // compare into VCC, then a select on it (the pair, one instruction each)
            asm volatile(
#define X(j) "v_cmp_lt_f32_e32 vcc, v41, v[44+2*" #j "]\n v_cndmask_b32_e32 v[45+2*" #j "], v41, v[45+2*" #j "], vcc\n"
                R16(X) ::: CLOB, "vcc");
#undef X
        if constexpr (K == 18)   // compare into an SGPR pair, then a select on it
            asm volatile(
#define X(j) "v_cmp_lt_f32_e64 s[20+2*(" #j "&3):21+2*(" #j "&3)], v41, v[44+2*" #j "]\n v_cndmask_b32_e64 v[45+2*" #j "], v41, v[45+2*" #j "], s[20+2*(" #j "&3):21+2*(" #j "&3)]\n"
                R16(X) ::: CLOB, "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
#undef X
    }
    float r;
    asm volatile("v_mov_b32 %0, v44" : "=v"(r)::CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static const char* names[] = {"fma b1,b3,acc", "fma x*x+acc", "fma b0,b0,acc", "pk_fma distinct", "pk_fma x*x+acc",
                              "mul x*x", "mul distinct", "fma b0,b1,acc(b0)", "cndmask_e64 sgpr", "cmp_e64",
                              "mov", "and", "bitop3 distinct", "add_f64", "mul_f64", "fma_f64 distinct",
                              "cmp_e32 vcc", "cmp_e32+cndmask_e32 (2)", "cmp_e64+cndmask_e64 (2)"};
template <int K>
static void run() {
    const int blocks = 256 * 8, threads = 256, iters = 8192;
    float* out;
    (void)hipMalloc(&out, sizeof(float) * blocks * threads);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    bank<K><<<blocks, threads>>>(out, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) bank<K><<<blocks, threads>>>(out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winst = 3.0 * blocks * threads / 64.0 * iters * 16;
    printf("%-20s %8.3f ms  %6.2f SIMD-cycles per wave-instruction (at 2.4 GHz, 1024 SIMDs)\n", names[K], ms,
           2.4e9 * ms / 1e3 * 1024.0 / winst);
    (void)hipFree(out);
}

int main() {
    for (int w = 0; w < 3; ++w) run<0>();
    run<0>(); run<1>(); run<2>(); run<3>(); run<4>(); run<5>(); run<6>(); run<7>();
    run<8>(); run<9>(); run<10>(); run<11>(); run<12>(); run<13>(); run<14>(); run<15>();
    run<16>(); run<17>(); run<18>();
    return 0;
}
