// Microbenchmark (diagnostic, not part of the library): cycles per Jacobi round of
// the ordered-choice kernel's inner loop on one wavefront, and of its parts.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_jacobi.hip -o tools/ubench_jacobi && tools/ubench_jacobi
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned int mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned int)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned int)m, 0u));
}

constexpr int TB = 4, WL = 256, ITERS = 4096;

// variant 0: the loop as in seg_solve_small (forced to run ITERS rounds)
// variant 1: the same with the LDS reads replaced by register arithmetic
// variant 2: only the dependent LDS reads (address from the previous value)
// variant 3: ballot/mbcnt chain only
__global__ void k(int variant, unsigned long long *out, int *sink) {
    __shared__ unsigned int win[TB * WL + 64];
    const int lane = threadIdx.x;
    for (int i = lane; i < TB * WL + 64; i += 64) win[i] = (i < TB * WL) ? ((i % WL) << 6 | (i / WL)) : ~0u;
    __syncthreads();
    int base[TB];
    for (int q = 0; q < TB; q++) base[q] = q * WL + (lane & 7);
    int ch = lane & 3;
    int acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (variant == 0) {
        for (int it = 0; it < ITERS; it++) {
            unsigned int v[TB];
#pragma unroll
            for (int q = 0; q < TB; q++) v[q] = win[base[q] + (int)mbcnt64(__ballot(ch == q))];
            unsigned int best = v[0];
#pragma unroll
            for (int q = 1; q < TB; q++) best = min(best, v[q]);
            ch = (int)(best & 63u);
            if (__ballot(ch == 77)) acc++;
        }
    } else if (variant == 1) {
        for (int it = 0; it < ITERS; it++) {
            unsigned int v[TB];
#pragma unroll
            for (int q = 0; q < TB; q++) v[q] = (unsigned int)(base[q] + (int)mbcnt64(__ballot(ch == q))) * 2654435761u;
            unsigned int best = v[0];
#pragma unroll
            for (int q = 1; q < TB; q++) best = min(best, v[q]);
            ch = (int)(best & 3u);
            if (__ballot(ch == 77)) acc++;
        }
    } else if (variant == 2) {
        unsigned int x = lane;
        for (int it = 0; it < ITERS; it++) {
            x = win[(x & 255)];
            if (__ballot(x == 0xdeadbeefu)) acc++;
        }
        ch = x;
    } else {
        for (int it = 0; it < ITERS; it++) {
            ch = (int)mbcnt64(__ballot(ch == 3)) & 3;
            if (__ballot(ch == 77)) acc++;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[variant] = t1 - t0;
    sink[lane] = ch + acc;
}

int main() {
    unsigned long long *d;
    int *sink;
    hipMalloc(&d, 8 * sizeof(unsigned long long));
    hipMalloc(&sink, 64 * sizeof(int));
    for (int v = 0; v < 4; v++) {
        for (int rep = 0; rep < 2; rep++) k<<<1, 64>>>(v, d, sink);
        hipDeviceSynchronize();
        unsigned long long c;
        hipMemcpy(&c, d + v, sizeof(c), hipMemcpyDeviceToHost);
        printf("variant %d: %.1f cycles per round\n", v, (double)c / ITERS);
    }
    return 0;
}
