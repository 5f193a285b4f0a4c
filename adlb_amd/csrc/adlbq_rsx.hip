// adlbq_rsx.hip -- hand-written LSD radix sort of (u64 key, int value) pairs
// (see adlbq_rsx.h).  gfx950: 64-wide waves, 256-thread workgroups of 2048
// keys, 8-bit digits.
#include "adlbq_rsx.h"

#include "adlbq_impl.h"

namespace adlbq {

__device__ __forceinline__ unsigned int rsx_digit(unsigned long long k, int sh, unsigned int mask, int desc) {
    return (unsigned int)((desc ? ~k : k) >> sh) & mask;  // descending = ascending on the complement
}

// lanes of this wave holding the same digit (valid lanes only)
__device__ __forceinline__ unsigned long long rsx_peers(unsigned int d, bool valid) {
    unsigned long long m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const unsigned long long bb = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    return m;
}

__global__ __launch_bounds__(RSX_THREADS) void k_rsx_hist(const unsigned long long *__restrict__ K, long long n,
                                                         int sh, unsigned int mask, int desc, int *__restrict__ hist,
                                                         int ntiles) {
    static_assert(RSX_THREADS == 256, "one thread per digit");
    __shared__ unsigned int sc[256];
    sc[threadIdx.x] = 0u;
    const long long base = (long long)blockIdx.x * RSX_TILE;
    constexpr int PER = RSX_TILE / RSX_THREADS;
    unsigned long long k[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const long long i = base + q * RSX_THREADS + threadIdx.x;
        k[q] = i < n ? K[i] : 0ull;
    }
    __syncthreads();
    const unsigned long long lt = (1ull << (threadIdx.x & 63)) - 1ull;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const bool valid = base + q * RSX_THREADS + threadIdx.x < n;
        const unsigned int d = rsx_digit(k[q], sh, mask, desc);
        const unsigned long long pe = rsx_peers(d, valid);
        if (valid && (pe & lt) == 0ull) atomicAdd(&sc[d], (unsigned int)__popcll(pe));  // one add per digit and wave
    }
    __syncthreads();
    hist[(long long)threadIdx.x * ntiles + blockIdx.x] = (int)sc[threadIdx.x];
}

// row d of hist (one digit over the tiles): exclusive prefix in place, total to rowtot[d]
__global__ __launch_bounds__(RSX_THREADS) void k_rsx_scan(int *__restrict__ hist, int ntiles, int *__restrict__ rowtot) {
    __shared__ int wsum[RSX_THREADS / 64];
    int *row = hist + (long long)blockIdx.x * ntiles;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int carry = 0;
    for (int c0 = 0; c0 < ntiles; c0 += RSX_THREADS) {
        const int i = c0 + threadIdx.x;
        const int v = i < ntiles ? row[i] : 0;
        int x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int pre = carry;
        for (int q = 0; q < w; q++) pre += wsum[q];
        if (i < ntiles) row[i] = pre + x - v;
#pragma unroll
        for (int q = 0; q < RSX_THREADS / 64; q++) carry += wsum[q];
        __syncthreads();
    }
    if (threadIdx.x == 0) rowtot[blockIdx.x] = carry;
}

__global__ __launch_bounds__(RSX_THREADS) void k_rsx_scatter(const unsigned long long *__restrict__ Kin,
                                                            const int *__restrict__ Vin,
                                                            unsigned long long *__restrict__ Kout,
                                                            int *__restrict__ Vout, long long n, int sh,
                                                            unsigned int mask, int desc, const int *__restrict__ hist,
                                                            const int *__restrict__ rowtot, int ntiles) {
    constexpr int NW = RSX_THREADS / 64;
    __shared__ unsigned int wc[NW][256];
    __shared__ unsigned int wsum[NW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long long base = (long long)blockIdx.x * RSX_TILE + (long long)w * RSX_STEPS * 64;
    // this wave's keys, a contiguous run in input order, in flight with the prologue's loads
    unsigned long long key[RSX_STEPS];
    int val[RSX_STEPS];
#pragma unroll
    for (int st = 0; st < RSX_STEPS; st++) {
        const long long i = base + st * 64 + lane;
        key[st] = i < n ? Kin[i] : 0ull;
        val[st] = i < n ? Vin[i] : 0;
    }
    // digit d's first output position for this tile: the totals of the lower digits + the earlier tiles' counts
    const int d0 = threadIdx.x;
    const int tot = rowtot[d0], tpre = hist[(long long)d0 * ntiles + blockIdx.x];
    int x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = (unsigned int)x;
#pragma unroll
    for (int q = 0; q < NW; q++) wc[q][d0] = 0u;
    __syncthreads();
    unsigned int dbase = (unsigned int)(x - tot + tpre);
    for (int q = 0; q < w; q++) dbase += wsum[q];
    // ranks within the wave's run: a running count per digit (one wave's LDS ops complete in order)
    unsigned int pos[RSX_STEPS], dig[RSX_STEPS];
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int st = 0; st < RSX_STEPS; st++) {
        const bool valid = base + st * 64 + lane < n;
        const unsigned int d = rsx_digit(key[st], sh, mask, desc);
        const unsigned long long pe = rsx_peers(d, valid);
        const unsigned int before = wc[w][d];
        pos[st] = before + (unsigned int)__popcll(pe & lt);
        dig[st] = d;
        __builtin_amdgcn_wave_barrier();
        if (valid && (pe & lt) == 0ull) wc[w][d] = before + (unsigned int)__popcll(pe);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {  // per digit: the tile's base plus the counts of the earlier waves
        unsigned int run = dbase;
#pragma unroll
        for (int q = 0; q < NW; q++) {
            const unsigned int c = wc[q][d0];
            wc[q][d0] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < RSX_STEPS; st++) {
        if (base + st * 64 + lane < n) {
            const unsigned int o = wc[w][dig[st]] + pos[st];
            Kout[o] = key[st];
            Vout[o] = val[st];
        }
    }
}

static size_t rsx_align(size_t b) { return (b + 255) & ~(size_t)255; }

size_t rsx_temp_bytes(long long n) {
    const long long nt = (n + RSX_TILE - 1) / RSX_TILE;
    return rsx_align(sizeof(unsigned long long) * (size_t)n) + rsx_align(sizeof(int) * (size_t)n) +
           rsx_align(sizeof(int) * 256 * (size_t)nt) + rsx_align(sizeof(int) * 256);
}

int rsx_sort_pairs(void *tmp, size_t tmp_bytes, const unsigned long long *kin, unsigned long long *kout,
                   const int *vin, int *vout, long long n, int lo_bit, int hi_bit, bool descending, hipStream_t s) {
    if (n <= 0) return ADLBQ_OK;
    if (lo_bit < 0 || hi_bit > 64 || n >= (1ll << 31) || tmp_bytes < rsx_temp_bytes(n))
        return fail(ADLBQ_ERR_ARG, "rsx_sort_pairs: bad arguments or scratch too small");
    const int nt = (int)((n + RSX_TILE - 1) / RSX_TILE);
    char *p = static_cast<char *>(tmp);
    auto *kt = reinterpret_cast<unsigned long long *>(p);
    p += rsx_align(sizeof(unsigned long long) * (size_t)n);
    auto *vt = reinterpret_cast<int *>(p);
    p += rsx_align(sizeof(int) * (size_t)n);
    auto *hist = reinterpret_cast<int *>(p);
    p += rsx_align(sizeof(int) * 256 * (size_t)nt);
    auto *rowtot = reinterpret_cast<int *>(p);
    const int P = hi_bit > lo_bit ? (hi_bit - lo_bit + 7) / 8 : 0;
    if (P == 0) {
        if (kout != kin) AQ_HIP(hipMemcpyAsync(kout, kin, sizeof(unsigned long long) * n, hipMemcpyDeviceToDevice, s));
        if (vout != vin) AQ_HIP(hipMemcpyAsync(vout, vin, sizeof(int) * n, hipMemcpyDeviceToDevice, s));
        return ADLBQ_OK;
    }
    const unsigned long long *ks = kin;
    const int *vs = vin;
    for (int q = 0; q < P; q++) {
        const int sh = lo_bit + 8 * q, nb = std::min(8, hi_bit - sh);
        const unsigned int mask = (1u << nb) - 1u;
        // the last pass writes the output: passes alternate output / scratch backwards from it
        const bool to_out = ((P - 1 - q) & 1) == 0;
        unsigned long long *kd = to_out ? kout : kt;
        int *vd = to_out ? vout : vt;
        k_rsx_hist<<<nt, RSX_THREADS, 0, s>>>(ks, n, sh, mask, descending ? 1 : 0, hist, nt);
        k_rsx_scan<<<256, RSX_THREADS, 0, s>>>(hist, nt, rowtot);
        k_rsx_scatter<<<nt, RSX_THREADS, 0, s>>>(ks, vs, kd, vd, n, sh, mask, descending ? 1 : 0, hist, rowtot, nt);
        ks = kd;
        vs = vd;
    }
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

}  // namespace adlbq
