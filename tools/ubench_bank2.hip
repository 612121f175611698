// Microbenchmark (round 6): VGPR bank sensitivity of the packed FP32 ops the sweep's filter and box tests
// issue (v_pk_fma_f32 with an SGPR-pair broadcast and two VGPR pairs, op_sel), of the 3-source VOP3 ops
// (max3, bitop3) and of fma_f32 with an SGPR operand: SIMD-cycles per wave-instruction, one asm block of 16
// independent instructions on fixed registers per loop step, 8 waves per SIMD.  A register's bank is its
// index mod 4.  Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_bank2 tools/ubench_bank2.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R16(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7) I(8) I(9) I(10) I(11) I(12) I(13) I(14) I(15)
#define CLOB "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", \
             "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", \
             "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76", \
             "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91", \
             "v92", "v93", "v94", "v95", "s20", "s21"
// destinations: v[64+2j : 65+2j] (j = 0..15; banks 0,1 for even j, 2,3 for odd j)
// constant pairs: v[32:33] (banks 0,1), v[34:35] (2,3), v[36:37] (0,1), v[38:39] (2,3); s[20:21] an SGPR pair
template <int K>
__global__ __launch_bounds__(256) void bank(float* out, int iters) {
    asm volatile("s_mov_b32 s20, 1.0\n s_mov_b32 s21, 1.0\n"
                 "v_mov_b32 v32, 1.0\n v_mov_b32 v33, 1.0\n v_mov_b32 v34, 1.0\n v_mov_b32 v35, 1.0\n"
                 "v_mov_b32 v36, 1.0\n v_mov_b32 v37, 1.0\n v_mov_b32 v38, 1.0\n v_mov_b32 v39, 1.0\n" ::: CLOB);
#define INIT(j) "v_mov_b32 v[64+2*" #j "], 1.0\n v_mov_b32 v[65+2*" #j "], 1.0\n v_mov_b32 v[40+" #j "], 1.0\n"
    asm volatile(R16(INIT) ::: CLOB);
    for (int i = 0; i < iters; ++i) {
        if constexpr (K == 0)   // pk_fma d = s * v(2,3) + v(0,1)   distinct banks (the filter's cz*K0 + K3 form)
            asm volatile(
#define X(j) "v_pk_fma_f32 v[64+2*" #j ":65+2*" #j "], s[20:21], v[34:35], v[32:33] op_sel_hi:[1,0,1]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 1)   // pk_fma d = s * v(0,1) + v(0,1)   same banks
            asm volatile(
#define X(j) "v_pk_fma_f32 v[64+2*" #j ":65+2*" #j "], s[20:21], v[36:37], v[32:33] op_sel_hi:[1,0,1]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 2)   // pk_fma d = s * v(2,3) + d   accumulate (the filter's chained form), distinct
            asm volatile(
#define X(j) "v_pk_fma_f32 v[64+2*" #j ":65+2*" #j "], s[20:21], v[34:35], v[64+2*" #j ":65+2*" #j "] op_sel_hi:[1,0,1]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 3)   // pk_fma d = s * v(0,1) + d   accumulate; d in banks 0,1 for even j
            asm volatile(
#define X(j) "v_pk_fma_f32 v[64+2*" #j ":65+2*" #j "], s[20:21], v[32:33], v[64+2*" #j ":65+2*" #j "] op_sel_hi:[1,0,1]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 4)   // pk_fma d = v * v + s (the r2f - y^2 form: x*x with an SGPR addend)
            asm volatile(
#define X(j) "v_pk_fma_f32 v[64+2*" #j ":65+2*" #j "], v[32:33], v[32:33], s[20:21] neg_lo:[1,0,0] neg_hi:[1,0,0]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 5)   // pk_fma three VGPR pairs, all banks 0,1
            asm volatile(
#define X(j) "v_pk_fma_f32 v[64+2*" #j ":65+2*" #j "], v[32:33], v[36:37], v[32:33]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 6)   // pk_mul s * v
            asm volatile(
#define X(j) "v_pk_mul_f32 v[64+2*" #j ":65+2*" #j "], s[20:21], v[34:35]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 7)   // fma_f32 s * v + v, distinct banks
            asm volatile(
#define X(j) "v_fma_f32 v[64+2*" #j "], s20, v33, v34\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 8)   // fma_f32 s * v + v, same bank (v32, v36)
            asm volatile(
#define X(j) "v_fma_f32 v[64+2*" #j "], s20, v32, v36\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 9)   // max3 distinct banks (v33, v34, v35)
            asm volatile(
#define X(j) "v_max3_f32 v[64+2*" #j "], v33, v34, v35\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 10)   // max3 two sources in one bank (v32, v36, v33)
            asm volatile(
#define X(j) "v_max3_f32 v[64+2*" #j "], v32, v36, v33\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 11)   // max with an inline constant (VOP2)
            asm volatile(
#define X(j) "v_max_f32 v[64+2*" #j "], 0, v33\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 12)   // fma_f32 v*v+v with one source each bank 1,2,3 (distinct, no SGPR)
            asm volatile(
#define X(j) "v_fma_f32 v[64+2*" #j "], v33, v34, v35\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 13)   // fma_f32 two of three sources in one bank (v33, v37, v34)
            asm volatile(
#define X(j) "v_fma_f32 v[64+2*" #j "], v33, v37, v34\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 14)   // v_and3 / v_bitop3 distinct
            asm volatile(
#define X(j) "v_and_or_b32 v[64+2*" #j "], v33, v34, v35\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 15)   // sub_f32 (VOP2) v - v
            asm volatile(
#define X(j) "v_sub_f32 v[64+2*" #j "], v33, v34\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 16)   // pk_add v + v distinct
            asm volatile(
#define X(j) "v_pk_add_f32 v[64+2*" #j ":65+2*" #j "], v[32:33], v[34:35]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 17)   // pk_add v + v same banks
            asm volatile(
#define X(j) "v_pk_add_f32 v[64+2*" #j ":65+2*" #j "], v[32:33], v[36:37]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 18)   // cvt_f32_u32 (VOP1)
            asm volatile(
#define X(j) "v_cvt_f32_u32 v[64+2*" #j "], v33\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 19)   // cndmask_e32 with vcc (set once)
            asm volatile(
#define X(j) "v_cndmask_b32_e32 v[64+2*" #j "], v33, v34, vcc\n"
                R16(X) ::: CLOB, "vcc");
#undef X
        if constexpr (K == 20)   // mul_f32 with an SGPR
            asm volatile(
#define X(j) "v_mul_f32 v[64+2*" #j "], s20, v33\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 22)   // 32-bit integer multiply (the scratch records' slot offset)
            asm volatile(
#define X(j) "v_mul_lo_u32 v[64+2*" #j "], s20, v33\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 23)   // 64-bit shift-add (pointer arithmetic)
            asm volatile(
#define X(j) "v_lshl_add_u64 v[64+2*" #j ":65+2*" #j "], s[20:21], 0, v[32:33]\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 24)   // 24-bit multiply
            asm volatile(
#define X(j) "v_mul_u32_u24 v[64+2*" #j "], s20, v33\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 25)   // shift-or, all VGPRs
            asm volatile(
#define X(j) "v_lshl_or_b32 v[64+2*" #j "], v33, v34, v35\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 26)   // max, all VGPRs
            asm volatile(
#define X(j) "v_max_f32 v[64+2*" #j "], v33, v34\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 27)   // add_u32 with an SGPR
            asm volatile(
#define X(j) "v_add_u32 v[64+2*" #j "], s20, v33\n"
                R16(X) ::: CLOB);
#undef X
        if constexpr (K == 21)   // readfirstlane-free v_lshlrev (VOP2 shift)
            asm volatile(
#define X(j) "v_lshlrev_b32 v[64+2*" #j "], 2, v33\n"
                R16(X) ::: CLOB);
#undef X
    }
    float r;
    asm volatile("v_mov_b32 %0, v64" : "=v"(r)::CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

static const char* names[] = {"pk_fma s,v23,v01", "pk_fma s,v01,v01", "pk_fma s,v23,acc", "pk_fma s,v01,acc",
                              "pk_fma v01*v01+s", "pk_fma v01,v01,v01", "pk_mul s,v23", "fma s,v1,v2",
                              "fma s,v0,v0'", "max3 v1,v2,v3", "max3 v0,v0',v1", "max 0,v1", "fma v1,v2,v3",
                              "fma v1,v1',v2", "and_or v1,v2,v3", "sub v1,v2", "pk_add v01,v23", "pk_add v01,v01'",
                              "cvt_f32_u32", "cndmask_e32 vcc", "mul s,v", "lshlrev 2,v", "mul_lo_u32 s,v",
                              "lshl_add_u64 s,0,v", "mul_u32_u24 s,v", "lshl_or v,v,v", "max v,v", "add_u32 s,v"};
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

template <int... K> static void all(std::integer_sequence<int, K...>) { (run<K>(), ...); }
int main() {
    for (int w = 0; w < 3; ++w) run<0>();
    all(std::make_integer_sequence<int, 28>{});
    return 0;
}
