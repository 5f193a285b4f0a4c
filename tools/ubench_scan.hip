// Microbenchmark (diagnostic, not part of the library): where pass 1 of the
// reserve batch (k_prep_hist's page role) spends its time at the metric size
// (10M units = 2442 pages of 4096, 4 B of meta per unit, 4 types, prio
// U[0,1024)).  Variants of one workgroup-per-page kernel:
//   0  loads only (16 KB per page, 4 x uint4 per lane), one store per block
//   1  + per-unit LDS histogram atomics (4 lane-interleaved copies, 64 bins per type)
//   2  + the epilogue: per-page u16 column row (T x 64) and per-chunk global atomics
//   3  cut-limited: only units at or above a per-type cut are counted (and listed)
//   4  variant 3 with a persistent grid (256 x 4 workgroups stride over the pages,
//      next page's loads in flight while the current one is counted)
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_scan.hip -o tools/ubench_scan && tools/ubench_scan
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int PAGE = 4096, T = 4, NB = 64, C = T * NB, HK = 4, CHUNK = 8;

__device__ __forceinline__ int bin_of(unsigned int d) {
    return d < 32 ? (int)d : min(63, 32 + (31 - __clz((int)d)) - 4);
}

template <int V>
__global__ __launch_bounds__(256) void k_page(const uint32_t *meta, int npages, unsigned short *gh, unsigned int *csum,
                                              unsigned int *spec, int *specn, unsigned int *sink, int cut) {
    __shared__ unsigned int hist[C * HK];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nblk = V == 4 ? gridDim.x : npages;
    for (int p = blockIdx.x; p < npages; p += nblk) {
        const uint4 *M4 = reinterpret_cast<const uint4 *>(meta + (long long)p * PAGE);
        uint4 mv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) mv[k] = M4[(w * 4 + k) * 64 + lane];
        if (V >= 1)
            for (int c = threadIdx.x; c < C * HK; c += 256) hist[c] = 0;
        if (V >= 1) __syncthreads();
        unsigned int acc = 0;
        int sn = 0;
        unsigned int *my = hist + (lane % HK);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t mm[4] = {mv[k].x, mv[k].y, mv[k].z, mv[k].w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int t = mm[q] & 3, pr = (int)(mm[q] >> 8);
                acc += mm[q];
                if (V == 1 || V == 2) atomicAdd(&my[(t * NB + bin_of(1023u - (unsigned)pr)) * HK], 1u);
                if (V >= 3 && pr >= cut) {
                    atomicAdd(&my[(t * NB + bin_of(1023u - (unsigned)pr)) * HK], 1u);
                    spec[((long long)p * 4 + w) * 256 + (sn++ & 255)] = (unsigned)(k * 4 + q);
                }
            }
        }
        if (V >= 3 && lane == 0) specn[p * 4 + w] = sn;
        if (V >= 1) __syncthreads();
        if (V >= 2) {
            unsigned int *cs = csum + (long long)(p / CHUNK) * C;
            unsigned short *g = gh + (long long)p * C;
            for (int c = threadIdx.x; c < C; c += 256) {
                unsigned int v = 0;
#pragma unroll
                for (int k = 0; k < HK; k++) v += hist[c * HK + k];
                if (V == 2 || (c % NB) < 20) g[c] = (unsigned short)v;
                if (v) atomicAdd(&cs[c], v);
            }
            __syncthreads();
        }
        if (V == 0 || V == 1) sink[p * 256 + threadIdx.x] = acc + (V == 1 ? hist[threadIdx.x] : 0);
        if (V == 1) __syncthreads();
    }
}

int main() {
    const int npages = 2442;
    const long long n = (long long)npages * PAGE;
    std::vector<uint32_t> h(n);
    unsigned long long x = 88172645463325252ull;
    for (long long i = 0; i < n; i++) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        h[i] = (uint32_t)((x & 3) | (((x >> 8) % 1024) << 8));
    }
    uint32_t *meta;
    unsigned short *gh;
    unsigned int *csum, *spec, *sink;
    int *specn;
    hipMalloc(&meta, n * 4);
    hipMemcpy(meta, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMalloc(&gh, (size_t)npages * C * 2);
    hipMalloc(&csum, (size_t)(npages / CHUNK + 1) * C * 4);
    hipMalloc(&spec, (size_t)npages * 4 * 256 * 4);
    hipMalloc(&specn, (size_t)npages * 4 * 4);
    hipMalloc(&sink, (size_t)npages * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](int v) {
        for (int rep = 0; rep < 25; rep++) {
            if (rep == 5) hipEventRecord(a, 0);
            switch (v) {
            case 0: k_page<0><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            case 1: k_page<1><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            case 2: k_page<2><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            case 3: k_page<3><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            case 4: k_page<4><<<1024, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            }
        }
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1000.0 / 20;
        printf("variant %d: %.2f us per launch, %.0f GB/s on %lld MB of meta\n", v, us, n * 4 / us / 1e3, n * 4 >> 20);
    };
    for (int v = 0; v <= 4; v++) run(v);
    // the same variants with the infinity cache flushed before each launch (1 GiB written in between):
    // the scan as it runs inside a reserve batch, where other kernels' traffic sits between two scans
    void *junk;
    hipMalloc(&junk, 1ll << 30);
    hipEvent_t c, d;
    hipEventCreate(&c);
    hipEventCreate(&d);
    for (int v = 0; v <= 3; v++) {
        double tot = 0;
        for (int rep = 0; rep < 12; rep++) {
            hipMemsetAsync(junk, rep, 1ll << 30, 0);
            hipEventRecord(c, 0);
            switch (v) {
            case 0: k_page<0><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            case 1: k_page<1><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            case 2: k_page<2><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            case 3: k_page<3><<<npages, 256>>>(meta, npages, gh, csum, spec, specn, sink, 1008); break;
            }
            hipEventRecord(d, 0);
            hipEventSynchronize(d);
            float ms = 0;
            hipEventElapsedTime(&ms, c, d);
            if (rep >= 2) tot += ms;
        }
        const double us = tot * 1000.0 / 10;
        printf("variant %d, cache flushed: %.2f us per launch, %.0f GB/s\n", v, us, n * 4 / us / 1e3);
    }
    return 0;
}
