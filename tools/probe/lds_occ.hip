// How many 256-thread workgroups per CU the runtime allows for a given static LDS size (is the
// allocation byte-granular?).  Prints one line per size.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int B> __global__ __launch_bounds__(256, 1) void k(float* o) {
    __shared__ float s[B / 4];
    s[threadIdx.x] = (float)threadIdx.x;
    __syncthreads();
    o[threadIdx.x] = s[(threadIdx.x * 7) % (B / 4)];
}
template <int B> void probe() {
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)k<B>, 256, 0);
    printf("lds %6d B: %d workgroups/CU\n", B, n);
}
int main() {
    probe<20480>(); probe<23096>(); probe<23552>(); probe<26168>(); probe<27192>(); probe<27304>(); probe<27308>();
    probe<27648>(); probe<32768>(); probe<32772>(); probe<40960>();
    return 0;
}
