// adlbq_keyrank.hip -- candidate ranking for 8 < T <= 64 work types ("keyrank").
//
// After k_select_open every type t has its candidate list at candoff[t] (in
// column order; inside a multi-priority column not yet in key order).  The
// ordered choice needs every list in key order (prio desc, open-bucket
// position asc: the order of wq_find_hi_prio, xq.c:190-217) and every
// candidate's rank among all candidates of the batch (k_rank's packed rank,
// rank << 6 | type).  A unit is a candidate of its own type only and its key
// holds its bucket position, so the keys are unique and both follow from one
// global order.  Instead of sorting each list (three radix digits) and then
// binary-searching every candidate in the 31 other lists (k_rank), the batch
// is binned once by a 16-bit digit of the key and ranked inside the bins:
//
//   k_kr_bits     OR / AND of every key: the bits the batch's keys vary in
//   k_kr_hist     digit = the top varying bits of the prio field, then the top
//                 varying bits of the position field (monotone in the key);
//                 global histogram of the 65,536 digits
//   k_kr_scan     exclusive scan of the bins, larger digits first; a bin larger
//                 than kr_bin_max (or more candidates than the buffers hold)
//                 fails the batch over: every later launch returns at once, the
//                 lists stay as they are and k_rank sorts and ranks them
//   k_kr_scatter  every key into its bin (any order inside the bin)
//   k_kr_rank     rank = bin start + keys of the bin greater than it; the
//                 candidate goes to that position of the order arrays and is
//                 counted under (rank / 1024, type)
//   k_kr_write    per chunk of 1024 ranks: a candidate's list position = its
//                 type's count in the earlier chunks + its earlier same-type
//                 peers in the chunk; ckey / cslot / crank written in list order
//
// Algorithmic traffic per candidate: ~8 B key read twice, 12 B binned, 13 B
// ordered, 16 B written back (plus the in-bin compares, L1/L2 hits).
#include "adlbq_impl.h"

#include <algorithm>

namespace adlbq {

constexpr int KR_BINS = 1 << 16, KR_CHUNK = 1024, KR_TY = 64;  // KR_TY: count row stride (T <= 64)

struct KrArgs {
    int T;
    const int *candoff;
    unsigned long long *ckey;
    int *cslot;
    unsigned int *crank;
    int *needsort;
    DevCounters *ctr;
    unsigned long long *bits;  // [2]: OR, AND of the keys (reset for the next batch by k_kr_write)
    int *flag;                 // [0]: this batch failed over to k_rank
    int *bins;                 // [KR_BINS] counts -> starts -> ends (zeroed by k_kr_write)
    int *ccnt;                 // [chunks][KR_TY] candidates per (rank chunk, type)
    unsigned long long *tkey, *okey;
    int *tidx, *oslot;
    unsigned char *otype;
    long long cap;  // candidates the buffers hold
    int bin_max;
};

// the digit's shape from the varying bits: dh top bits of the prio field's
// varying range, then dl top bits of the position field's
struct KrDigit {
    int shH, dh, shL, dl;
};

__device__ __forceinline__ KrDigit kr_shape(const unsigned long long *bits) {
    const unsigned long long v = bits[0] ^ bits[1];
    const unsigned int vh = (unsigned int)(v >> 32), vl = (unsigned int)v;
    const int nh = vh ? 32 - __clz(vh) : 0, nl = vl ? 32 - __clz(vl) : 0;
    const int dh = min(nh, 16), dl = min(nl, 16 - dh);
    return KrDigit{nh - dh, dh, nl - dl, dl};
}

__device__ __forceinline__ int kr_digit(unsigned long long k, const KrDigit &s) {
    const unsigned int H = (unsigned int)(k >> 32), L = (unsigned int)k;
    const unsigned int dH = (H >> s.shH) & ((1u << s.dh) - 1u), dL = (L >> s.shL) & ((1u << s.dl) - 1u);
    return (int)((dH << s.dl) | dL);
}

__global__ __launch_bounds__(256) void k_kr_bits(KrArgs a) {
    __shared__ unsigned long long so[4], sa[4];
    const int G = a.candoff[a.T];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (blockIdx.x == 0 && tid == 0) {
        a.flag[0] = G > a.cap ? 1 : 0;
        a.ctr->plan_g = G;  // sizes the next batch's buffers
        a.ctr->rank_fast = 0;  // k_kr_write sets it once the ranks are in
    }
    if (G > a.cap) return;
    const long long nc = ((long long)G + KR_CHUNK - 1) / KR_CHUNK * KR_TY;
    for (long long k = (long long)blockIdx.x * blockDim.x + tid; k < nc; k += (long long)gridDim.x * blockDim.x)
        a.ccnt[k] = 0;
    unsigned long long o = 0ull, n = ~0ull;
    for (int i = blockIdx.x * blockDim.x + tid; i < G; i += gridDim.x * blockDim.x) {
        const unsigned long long k = a.ckey[i];
        o |= k;
        n &= k;
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        o |= __shfl_xor(o, d, 64);
        n &= __shfl_xor(n, d, 64);
    }
    if (lane == 0) {
        so[w] = o;
        sa[w] = n;
    }
    __syncthreads();
    if (tid == 0) {
        for (int q = 1; q < 4; q++) {
            o |= so[q];
            n &= sa[q];
        }
        if (n != ~0ull || o != 0ull) {
            atomicOr(&a.bits[0], o);
            atomicAnd(&a.bits[1], n);
        }
    }
}

__global__ __launch_bounds__(256) void k_kr_hist(KrArgs a) {
    if (a.flag[0]) return;
    const int G = a.candoff[a.T];
    const KrDigit s = kr_shape(a.bits);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < G; i += gridDim.x * blockDim.x)
        atomicAdd(&a.bins[kr_digit(a.ckey[i], s)], 1);
}

// one workgroup: thread q owns the 64 bins [65536 - 64 (q + 1), 65536 - 64 q), larger digits first
__global__ __launch_bounds__(1024) void k_kr_scan(KrArgs a) {
    __shared__ int wsum[16], wmax[16];
    if (a.flag[0]) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int4 *b4 = reinterpret_cast<int4 *>(a.bins + KR_BINS - 64 * (tid + 1));
    int4 v[16];
#pragma unroll
    for (int q = 0; q < 16; q++) v[q] = b4[q];
    int sum = 0, mx = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        sum += v[q].x + v[q].y + v[q].z + v[q].w;
        mx = max(mx, max(max(v[q].x, v[q].y), max(v[q].z, v[q].w)));
    }
    int x = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    int m = mx;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if (lane == 63) wsum[w] = x;
    if (lane == 0) wmax[w] = m;
    __syncthreads();
    int run = x - sum;
    for (int q = 0; q < w; q++) run += wsum[q];
    bool big = false;
    for (int q = 0; q < 16; q++) big |= wmax[q] > a.bin_max;
    if (big) {  // every thread saw the same maxima: nobody writes starts
        if (tid == 0) a.flag[0] = 1;
        return;
    }
    // starts, from this thread's largest digit down
#pragma unroll
    for (int q = 15; q >= 0; q--) {
        int4 u = v[q];
        const int cw = u.w, cz = u.z, cy = u.y, cx = u.x;
        u.w = run;
        run += cw;
        u.z = run;
        run += cz;
        u.y = run;
        run += cy;
        u.x = run;
        run += cx;
        b4[q] = u;
    }
}

__global__ __launch_bounds__(256) void k_kr_scatter(KrArgs a) {
    if (a.flag[0]) return;
    const int G = a.candoff[a.T];
    const KrDigit s = kr_shape(a.bits);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < G; i += gridDim.x * blockDim.x) {
        const unsigned long long k = a.ckey[i];
        const int p = atomicAdd(&a.bins[kr_digit(k, s)], 1);
        a.tkey[p] = k;
        a.tidx[p] = i;
    }
}

__global__ __launch_bounds__(256) void k_kr_rank(KrArgs a) {
    __shared__ int soff[ADLBQ_MAX_TYPES + 1];
    if (a.flag[0]) return;
    const int T = a.T;
    for (int t = threadIdx.x; t <= T; t += blockDim.x) soff[t] = a.candoff[t];
    __syncthreads();
    const int G = soff[T];
    const KrDigit s = kr_shape(a.bits);
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < G; p += gridDim.x * blockDim.x) {
        const unsigned long long k = a.tkey[p];
        const int d = kr_digit(k, s);
        const int be = a.bins[d], bs = d == KR_BINS - 1 ? 0 : a.bins[d + 1];  // after the scatter: bin ends
        int r = bs;
        for (int q = bs; q < be; q++) r += a.tkey[q] > k ? 1 : 0;
        const int i = a.tidx[p];
        int lo = 0, hi = T - 1;  // the last list starting at or before i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (soff[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        a.okey[r] = k;
        a.oslot[r] = a.cslot[i];
        a.otype[r] = (unsigned char)lo;
        atomicAdd(&a.ccnt[(long long)(r / KR_CHUNK) * KR_TY + lo], 1);
    }
}

__global__ __launch_bounds__(KR_CHUNK) void k_kr_write(KrArgs a) {
    __shared__ int spre[16][KR_TY], wcnt[16][KR_TY], soff[ADLBQ_MAX_TYPES + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int T = a.T;
    // the next batch's histogram starts from zero bins and fresh OR / AND
    for (int k = blockIdx.x * blockDim.x + tid; k < KR_BINS; k += gridDim.x * blockDim.x) a.bins[k] = 0;
    const bool failed = a.flag[0] != 0;
    if (blockIdx.x == 0 && tid == 0) {
        a.bits[0] = 0ull;
        a.bits[1] = ~0ull;
        if (failed) a.ctr->kr_fail += 1;
        else a.ctr->rank_fast = 1;  // k_rank: the ranks are in, only its bookkeeping is left
    }
    if (failed) return;
    if (blockIdx.x == 0)
        for (int t = tid; t < T; t += blockDim.x)
            if (a.needsort[t] == 1) a.needsort[t] = 2;
    if (tid <= T) soff[tid] = a.candoff[tid];
    __syncthreads();
    const int G = soff[T], nch = (G + KR_CHUNK - 1) / KR_CHUNK;
    const unsigned long long lt = (1ull << lane) - 1ull;
    for (int c = blockIdx.x; c < nch; c += gridDim.x) {
        {  // per type: candidates of the earlier chunks (thread = type lane x 16 parts)
            int sum = 0;
            for (int q = w; q < c; q += 16) sum += a.ccnt[(long long)q * KR_TY + lane];
            spre[w][lane] = sum;
            wcnt[w][lane] = 0;
        }
        __syncthreads();
        const int r = c * KR_CHUNK + tid;
        const bool valid = r < G;
        const int t = valid ? (int)a.otype[r] : 0;
        unsigned long long pe = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 6; b++) {
            const unsigned long long bb = __ballot((t >> b) & 1);
            pe &= ((t >> b) & 1) ? bb : ~bb;
        }
        const int before = __popcll(pe & lt);
        if (valid && before == 0) wcnt[w][t] = __popcll(pe);
        __syncthreads();
        if (tid < KR_TY) {  // the chunk's start of type tid per wave
            int run = tid < T ? soff[tid] : 0;
            for (int q = 0; q < 16; q++) run += spre[q][tid];
            for (int q = 0; q < 16; q++) {
                const int x = wcnt[q][tid];
                wcnt[q][tid] = run;
                run += x;
            }
        }
        __syncthreads();
        if (valid) {
            const int pos = wcnt[w][t] + before;
            a.ckey[pos] = a.okey[r];
            a.cslot[pos] = a.oslot[r];
            a.crank[pos] = ((unsigned int)r << 6) | (unsigned int)t;
        }
        __syncthreads();  // spre / wcnt are reused by the next chunk
    }
}

// The six launches on the handle's stream.  Buffers are sized for the larger
// of the batch's demand bound and the newest landed batch's candidate count;
// a batch with more candidates than that fails over (and sizes the next).
int launch_keyrank(adlbq_server *h, int R) {
    const int T = h->T;
    hipStream_t s = h->stream;
    long long want = (long long)R * std::min(T, NREQ) + (long long)T * h->export_extra;
    int g_last = 0, lo_last = 0;
    if (plan_hint(h, &g_last, &lo_last)) want = std::max(want, (long long)g_last + g_last / 4 + 4096);
    want = std::max(1024ll, std::min(want, h->cap_cand));
    if (want > h->cap_kr) {
        AQ_HIP(hipStreamSynchronize(s));
        if (h->d_kr) AQ_HIP(hipFree(h->d_kr));
        const long long cap = std::min(std::max(want, 2 * h->cap_kr), std::max(h->cap_cand, 1024ll));
        const long long nch = (cap + KR_CHUNK - 1) / KR_CHUNK;
        const size_t bytes = sizeof(unsigned long long) * (2 * cap + 2) + sizeof(int) * (2 * cap + KR_BINS + 64) +
                             sizeof(int) * nch * KR_TY + (size_t)cap + 256;
        AQ_HIP(hipMalloc((void **)&h->d_kr, bytes));
        h->cap_kr = cap;
        AQ_HIP(hipMemsetAsync(h->d_kr, 0, bytes, s));
        unsigned long long *bits = reinterpret_cast<unsigned long long *>(h->d_kr);
        AQ_HIP(hipMemsetAsync(bits + 1, 0xff, sizeof(unsigned long long), s));  // AND starts at all ones
    }
    const long long cap = h->cap_kr, nch = (cap + KR_CHUNK - 1) / KR_CHUNK;
    char *p = h->d_kr;
    KrArgs a{};
    a.T = T;
    a.candoff = h->d_candoff;
    a.ckey = h->d_ckey;
    a.cslot = h->d_cslot;
    a.crank = h->d_crank;
    a.needsort = h->d_needsort;
    a.ctr = h->d_ctr;
    a.bits = reinterpret_cast<unsigned long long *>(p);
    a.tkey = a.bits + 2;
    a.okey = a.tkey + cap;
    a.bins = reinterpret_cast<int *>(a.okey + cap);
    a.flag = a.bins + KR_BINS;
    a.tidx = a.flag + 64;
    a.oslot = a.tidx + cap;
    a.ccnt = a.oslot + cap;
    a.otype = reinterpret_cast<unsigned char *>(a.ccnt + nch * KR_TY);
    a.cap = cap;
    a.bin_max = h->kr_bin_max;
    const int g256 = (int)std::min<long long>(2048, (want + 255) / 256);
    k_kr_bits<<<g256, 256, 0, s>>>(a);
    k_kr_hist<<<g256, 256, 0, s>>>(a);
    k_kr_scan<<<1, 1024, 0, s>>>(a);
    k_kr_scatter<<<g256, 256, 0, s>>>(a);
    k_kr_rank<<<g256, 256, 0, s>>>(a);
    k_kr_write<<<(int)std::max(64ll, std::min(nch, (want + KR_CHUNK - 1) / KR_CHUNK)), KR_CHUNK, 0, s>>>(a);
    AQ_HIP(hipGetLastError());
    h->n_keyrank++;
    return ADLBQ_OK;
}

}  // namespace adlbq
