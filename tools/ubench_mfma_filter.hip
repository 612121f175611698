// Microbenchmark (round 6): the general sweep's sphere filter for one 16-sphere cluster and 64 rays, as the product
// runs it (4 groups x 14 v_pk_fma_f32 with SGPR sphere operands, then the sign test and a ballot) against the same
// distances on the matrix cores: X = E1 . C and Y = E2 . C (rays x 4) . (4 x spheres) with v_mfma_f32_16x16x4_f32
// (4 tiles of 16 rays, X and Y: 8 MFMAs), D = r2 - X^2 - Y^2 on the VALU, the signs ANDed and one ballot.
// 6 waves per SIMD (the product's occupancy), every wave walking the same clusters (L1/K$-resident).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_mfma_filter tools/ubench_mfma_filter.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
#define NCL 64   // clusters in the table

__device__ __forceinline__ uint32_t filter_group(const float* v, f2 K0, f2 K1, f2 K2, f2 K3) {
    const f2 cx0 = {v[0], v[1]}, cy0 = {v[2], v[3]}, cz0 = {v[4], v[5]}, rr0 = {v[6], v[7]};
    const f2 cx1 = {v[8], v[9]}, cy1 = {v[10], v[11]}, cz1 = {v[12], v[13]}, rr1 = {v[14], v[15]};
    f2 a0, b0, a1, b1, r0, r1;
    asm volatile(
        "v_pk_fma_f32 %[a0], %[cz0], %[K0], %[K3] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
        "v_pk_fma_f32 %[b0], %[cz0], %[K2], %[K3] op_sel:[0,0,1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[a1], %[cz1], %[K0], %[K3] op_sel:[0,1,0] op_sel_hi:[1,1,0]\n\t"
        "v_pk_fma_f32 %[b1], %[cz1], %[K2], %[K3] op_sel:[0,0,1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[a0], %[cx0], %[K0], %[a0] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[b0], %[cy0], %[K1], %[b0] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[a1], %[cx1], %[K0], %[a1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[b1], %[cy1], %[K1], %[b1] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[b0], %[cx0], %[K1], %[b0] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[b1], %[cx1], %[K1], %[b1] op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %[r0], %[b0], %[b0], %[rr0] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
        "v_pk_fma_f32 %[r1], %[b1], %[b1], %[rr1] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
        "v_pk_fma_f32 %[r0], %[a0], %[a0], %[r0] neg_lo:[1,0,0] neg_hi:[1,0,0]\n\t"
        "v_pk_fma_f32 %[r1], %[a1], %[a1], %[r1] neg_lo:[1,0,0] neg_hi:[1,0,0]"
        : [a0] "=&v"(a0), [b0] "=&v"(b0), [a1] "=&v"(a1), [b1] "=&v"(b1), [r0] "=&v"(r0), [r1] "=&v"(r1)
        : [cx0] "s"(cx0), [cy0] "s"(cy0), [cz0] "s"(cz0), [rr0] "s"(rr0), [cx1] "s"(cx1), [cy1] "s"(cy1),
          [cz1] "s"(cz1), [rr1] "s"(rr1), [K0] "v"(K0), [K1] "v"(K1), [K2] "v"(K2), [K3] "v"(K3));
    const uint32_t s0 = __float_as_uint(r0.x) & __float_as_uint(r0.y), s1 = __float_as_uint(r1.x) & __float_as_uint(r1.y);
    return ~(s0 & s1);
}

// VALU: per cluster, 4 groups (64 B each, scalar loads) -> 4 ballots
template <int MODE>
__global__ __launch_bounds__(256, 6) void sweep(const float* __restrict__ sph, const float* __restrict__ mcl, int iters,
                                                uint32_t* out, float seed) {
    const uint32_t lane = threadIdx.x & 63u;
    // per-lane ray constants (arbitrary, distinct per lane)
    const float e1x = 0.6f + 0.001f * lane, e1z = 0.8f - 0.001f * lane, e2x = 0.3f, e2y = 0.9f - 0.0005f * lane,
                e2z = 0.1f, oe1 = seed * lane, oe2 = -seed * lane;
    uint32_t acc = 0;
    if constexpr (MODE == 0) {
        const f2 K0 = {e1x, e1z}, K1 = {e2x, e2y}, K2 = {e2z, 0.0f}, K3 = {-oe1, -oe2};
        for (int it = 0; it < iters; ++it) {
            const uint32_t c = __builtin_amdgcn_readfirstlane((uint32_t)it % NCL);
            float sv[4][16];   // the cluster's 4 groups, all requested before the first filter (64 SGPRs)
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int j = 0; j < 16; ++j) sv[g][j] = sph[64u * c + 16u * g + j];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint32_t m = filter_group(sv[g], K0, K1, K2, K3);
                const unsigned long long b = __ballot((int32_t)m < 0);
                acc += (uint32_t)b;
            }
        }
    } else {
        // A operands: tile t (rays 16t .. 16t+15): lane l supplies ray 16t + (l & 15)'s component l >> 4
        const uint32_t k = lane >> 4;
        const float c1 = k == 0 ? e1x : (k == 1 ? 0.0f : (k == 2 ? e1z : -oe1));
        const float c2 = k == 0 ? e2x : (k == 1 ? e2y : (k == 2 ? e2z : -oe2));
        float A1[4], A2[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int src = (16 * t + (int)(lane & 15u)) * 4;
            A1[t] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(c1)));
            A2[t] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(c2)));
        }
        // cluster block: [k][j] k = 0..2 centre components, k = 3: r2 (B uses 1.0 there)
        float bn = mcl[lane], r2n = mcl[48u + (lane & 15u)];
        for (int it = 0; it < iters; ++it) {
            const float b = bn, r2 = r2n;
            const uint32_t cn = (uint32_t)(it + 1) % NCL;
            bn = mcl[64u * cn + lane];
            r2n = mcl[64u * cn + 48u + (lane & 15u)];
            const float B = k == 3u ? 1.0f : b;
            uint32_t s = 0xFFFFFFFFu;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
                const f4 X = __builtin_amdgcn_mfma_f32_16x16x4f32(A1[t], B, z, 0, 0, 0);
                const f4 Y = __builtin_amdgcn_mfma_f32_16x16x4f32(A2[t], B, z, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float D = __builtin_fmaf(-X[r], X[r], __builtin_fmaf(-Y[r], Y[r], r2));
                    s &= __float_as_uint(D);
                }
            }
            const unsigned long long bb = __ballot((int32_t)s >= 0);   // lane l: sphere l & 15 passes for a ray of its 16
            acc += (uint32_t)(bb | (bb >> 16) | (bb >> 32) | (bb >> 48));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
static void run(const float* sph, const float* mcl, uint32_t* out) {
    const int blocks = 256 * 6, threads = 256, iters = 4096;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    sweep<MODE><<<blocks, threads>>>(sph, mcl, iters, out, 1e-3f);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) sweep<MODE><<<blocks, threads>>>(sph, mcl, iters, out, 1e-3f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wc = 3.0 * blocks * threads / 64.0 * iters;   // wave-clusters
    printf("%s  %8.3f ms  %7.1f SIMD-cycles per wave-cluster (2.4 GHz, 1024 SIMDs)\n",
           MODE == 0 ? "VALU filter (4 groups, 56 pk_fma)" : "MFMA filter (8 x 16x16x4 f32)   ", ms,
           2.4e9 * ms / 1e3 * 1024.0 / wc);
}

int main() {
    float *sph, *mcl;
    uint32_t* out;
    (void)hipMalloc(&sph, sizeof(float) * 64 * NCL);
    (void)hipMalloc(&mcl, sizeof(float) * 64 * NCL);
    (void)hipMalloc(&out, sizeof(uint32_t) * 256 * 6 * 256);
    float h[64 * NCL];
    for (int i = 0; i < 64 * NCL; ++i) h[i] = 0.01f * (float)((i * 37) % 101) - 0.5f;
    (void)hipMemcpy(sph, h, sizeof(h), hipMemcpyHostToDevice);
    (void)hipMemcpy(mcl, h, sizeof(h), hipMemcpyHostToDevice);
    for (int w = 0; w < 2; ++w) run<0>(sph, mcl, out);
    run<0>(sph, mcl, out);
    run<1>(sph, mcl, out);
    run<0>(sph, mcl, out);
    run<1>(sph, mcl, out);
    return 0;
}
