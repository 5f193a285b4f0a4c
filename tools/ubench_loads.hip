// Microbenchmark (diagnostic, not part of the library): the latency of one
// round of independent global loads per lane, issued by 256 single-wave
// workgroups right after another kernel wrote the data (the ordered-choice
// kernel's prologue shape).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_loads.hip -o tools/ubench_loads && tools/ubench_loads
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_write(unsigned int *buf, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) buf[i] = i * 2654435761u;
}

// mode 0: NL dword loads per lane; mode 1: NL/4 dwordx4 loads per lane; mode 2: one dword load per lane
template <int NL>
__global__ void k_read(const unsigned int *buf, int mode, unsigned long long *st, unsigned int *sink) {
    const int lane = threadIdx.x, b = blockIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned int acc = 0;
    if (mode == 0) {
        unsigned int v[NL];
#pragma unroll
        for (int i = 0; i < NL; i++) v[i] = buf[(b * NL + i) * 64 + lane];
#pragma unroll
        for (int i = 0; i < NL; i++) acc += v[i];
    } else if (mode == 1) {
        const uint4 *b4 = reinterpret_cast<const uint4 *>(buf);
        uint4 v[NL / 4];
#pragma unroll
        for (int i = 0; i < NL / 4; i++) v[i] = b4[(b * NL / 4 + i) * 64 + lane];
#pragma unroll
        for (int i = 0; i < NL / 4; i++) acc += v[i].x + v[i].y + v[i].z + v[i].w;
    } else {
        acc = buf[b * 64 + lane];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) st[b] = (t1 - t0) * 10;
    sink[b * 64 + lane] = acc;
}

int main() {
    const int n = 1 << 22;
    unsigned int *buf, *sink;
    unsigned long long *st;
    hipMalloc(&buf, n * 4);
    hipMalloc(&sink, 256 * 64 * 4);
    hipMalloc(&st, 256 * 8);
    unsigned long long h[256];
    for (int mode = 0; mode < 3; mode++) {
        for (int rep = 0; rep < 3; rep++) {
            k_write<<<1024, 256>>>(buf, n);
            k_read<48><<<256, 64>>>(buf, mode, st, sink);
            hipDeviceSynchronize();
        }
        hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost);
        unsigned long long mn = ~0ull, mx = 0, sum = 0;
        for (int i = 0; i < 256; i++) {
            mn = h[i] < mn ? h[i] : mn;
            mx = h[i] > mx ? h[i] : mx;
            sum += h[i];
        }
        printf("mode %d (%s): min %llu ns, mean %llu ns, max %llu ns\n", mode,
               mode == 0 ? "48 dword loads/lane" : mode == 1 ? "12 dwordx4 loads/lane" : "1 dword load/lane", mn,
               sum / 256, mx);
    }
    return 0;
}
