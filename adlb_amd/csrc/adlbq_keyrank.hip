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
//   k_kr_hist     digit = the top 16 bits of (distance below the largest
//                 anchor, bucket position) -- monotone in the key, its ranges
//                 from the types' anchors and thresholds (no pass over the
//                 keys to find them); each candidate's place in its bin
//                 (atomic), per-group counts of 256 bins
//   k_kr_scan     256 workgroups: bin starts (better digits first); a bin
//                 larger than kr_bin_max, or more candidates than the buffers
//                 hold, fails the batch over: every later launch returns at
//                 once, the lists stay as they are and k_rank sorts and ranks
//   k_kr_scatter  every key to bin start + its place (no atomics)
//   k_kr_rank     rank = bin start + keys of the bin greater than it; the
//                 candidate goes to that position of the order arrays and is
//                 counted under (rank / 1024, type)
//   k_kr_write    per chunk of 1024 ranks: a candidate's list position = its
//                 type's count in the earlier chunks + its earlier same-type
//                 peers in the chunk; ckey / cslot / crank written in list
//                 order; bins, group counts and the other parity's chunk
//                 counts zeroed for the next batch
//
// Algorithmic traffic per candidate: the 8 B key read three times, 12 B
// binned, 13 B ordered, 16 B written back (plus the in-bin compares, L1/L2 hits).
#include "adlbq_impl.h"

#include <algorithm>
#include <climits>

namespace adlbq {

constexpr int KR_BINS = 1 << 16, KR_CHUNK = 1024, KR_TY = 64;  // KR_TY: count row stride (T <= 64)
constexpr int KR_COARSE = KR_BINS / 256;                        // 256 groups of 256 bins (k_kr_scan's workgroups)
constexpr int KR_RANK_PER = 256;                                // positions per k_kr_rank workgroup (one per thread)
constexpr int KR_SLACK = 256;                                   // ... and keys staged on either side

struct KrArgs {
    int T;
    const int *candoff, *candlen, *theta;
    const long long *anchor;
    int nbpos_bits;  // bits of an open-bucket position (pages << PAGE_SHIFT)
    unsigned long long *ckey;
    int *cslot;
    unsigned int *crank;
    int *needsort;
    DevCounters *ctr;
    int *flag;      // [0]: this batch failed over to k_rank
    int *bins;      // [KR_BINS] counts -> starts (zeroed by k_kr_write)
    int *coarse;    // [KR_COARSE] counts per group of 256 bins (zeroed by k_kr_write)
    int *tslot;     // [cap] each candidate's place inside its bin
    int *ccnt;      // [chunks][KR_TY] candidates per (rank chunk, type), this batch's parity
    int *ccnt_next; // the other parity: zeroed here for the next batch
    long long nccnt;
    unsigned long long *tkey, *okey;
    int *tidx, *oslot;
    unsigned char *otype;
    long long cap;  // candidates the buffers hold
    int bin_max;
};

// The digit: a candidate of type t has cut_t <= prio <= anchor_t (k_thresholds),
// so with A = the largest anchor and D = A - prio, (D, bucket position)
// ascending is the key order; the digit is the top 16 bits of D's and the
// position's bit ranges side by side (ascending digit = better key).
struct KrDigit {
    long long A;
    int nb, sh;  // position bits; right shift of (D << nb | position)
};

__device__ KrDigit kr_shape(const KrArgs &a) {
    __shared__ long long s_a, s_c;
    if (threadIdx.x < 64) {
        const int t = threadIdx.x;
        const bool on = t < a.T && a.candlen[t] > 0;
        const int th = on ? a.theta[t] : -1;
        const long long an = on ? a.anchor[t] : LLONG_MIN;
        long long cut = LLONG_MAX;
        if (on && th >= 0) cut = std::max(an - bin_hi(th), (long long)LOWEST + 1);
        else if (on) cut = (long long)LOWEST + 1;
        long long mx = an, mn = cut;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            mx = std::max(mx, (long long)__shfl_xor(mx, o, 64));
            mn = std::min(mn, (long long)__shfl_xor(mn, o, 64));
        }
        if (t == 0) {
            s_a = mx;
            s_c = mn;
        }
    }
    __syncthreads();
    const long long A = s_a, dmax = s_a > s_c ? s_a - s_c : 0;
    const int nd = dmax > 0 ? 64 - __clzll((unsigned long long)dmax) : 0;
    return KrDigit{A, a.nbpos_bits, max(0, nd + a.nbpos_bits - 16)};
}

__device__ __forceinline__ int kr_digit(unsigned long long k, const KrDigit &s) {
    const int prio = (int)((unsigned int)(k >> 32) ^ 0x80000000u);
    const unsigned int bpos = ~(unsigned int)k;
    const unsigned long long D = (unsigned long long)std::max(0ll, s.A - (long long)prio);
    const unsigned long long c = (D << s.nb) | bpos;
    return (int)min((unsigned long long)(KR_BINS - 1), c >> s.sh);
}

// digits, each candidate's place in its bin, per-group counts
__global__ __launch_bounds__(256) void k_kr_hist(KrArgs a) {
    __shared__ int lc[KR_COARSE];
    const int G = a.candoff[a.T];
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && tid == 0) {
        a.flag[0] = G > a.cap ? 1 : 0;
        a.ctr->plan_g = G;     // sizes the next batch's buffers
        a.ctr->rank_fast = 0;  // k_kr_write sets it once the ranks are in
        a.ctr->kr_maxbin = 0;
    }
    if (G > a.cap) return;
    const KrDigit s = kr_shape(a);
    lc[tid] = 0;
    __syncthreads();
    const int lane = tid & 63;
    const unsigned long long lt = (1ull << lane) - 1ull;
    // consecutive candidates of a list mostly share a digit: one atomic per distinct digit of a
    // wave (its lanes' places follow the leader's), as many LDS adds for the group counts
    for (int i0 = blockIdx.x * blockDim.x; i0 < G; i0 += gridDim.x * blockDim.x) {
        const int i = i0 + tid;
        const bool valid = i < G;
        const int d = valid ? kr_digit(a.ckey[i], s) : 0;
        unsigned long long pe = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const unsigned long long bb = __ballot((d >> b) & 1);
            pe &= ((d >> b) & 1) ? bb : ~bb;
        }
        const bool lead = valid && (pe & lt) == 0ull;
        int base = 0;
        if (lead) {
            const int n = __popcll(pe);
            base = atomicAdd(&a.bins[d], n);
            atomicAdd(&lc[d >> 8], n);
        }
        base = __shfl(base, valid ? __ffsll((long long)pe) - 1 : 0, 64);
        if (valid) a.tslot[i] = base + __popcll(pe & lt);
    }
    __syncthreads();
    if (lc[tid]) atomicAdd(&a.coarse[tid], lc[tid]);
}

// 256 workgroups: group g's bins get their starts (the groups before it, then a block scan)
__global__ __launch_bounds__(256) void k_kr_scan(KrArgs a) {
    __shared__ int wsum[4];
    if (a.flag[0]) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = blockIdx.x;
    int base = tid < g ? a.coarse[tid] : 0;
    const int c = a.bins[g * 256 + tid];
    if (c > a.bin_max) a.flag[0] = 2;  // every later launch returns at once; k_kr_write still cleans up
    int x = c, mx = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
        base += __shfl_xor(base, o, 64);
        mx = max(mx, __shfl_xor(mx, o, 64));
    }
    if (lane == 0 && mx > 0) atomicMax(&a.ctr->kr_maxbin, mx);
    __shared__ int bsum[4];
    if (lane == 63) wsum[w] = x;
    if (lane == 0) bsum[w] = base;
    __syncthreads();
    int st = x - c + bsum[0] + bsum[1] + bsum[2] + bsum[3];
    for (int q = 0; q < w; q++) st += wsum[q];
    a.bins[g * 256 + tid] = st;
}

__global__ __launch_bounds__(256) void k_kr_scatter(KrArgs a) {
    if (a.flag[0]) return;
    const int G = a.candoff[a.T];
    const KrDigit s = kr_shape(a);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < G; i += gridDim.x * blockDim.x) {
        const unsigned long long k = a.ckey[i];
        const int p = a.bins[kr_digit(k, s)] + a.tslot[i];
        a.tkey[p] = k;
        a.tidx[p] = i;
    }
}

// positions [KR_RANK_PER * b, +KR_RANK_PER): ranks land within a bin of them, so
// the (chunk, type) counts of chunks c0 - 1 .. c0 + 2 are gathered in LDS first
__global__ __launch_bounds__(256) void k_kr_rank(KrArgs a) {
    __shared__ int soff[ADLBQ_MAX_TYPES + 1], lc[4][KR_TY];
    __shared__ unsigned long long skey[KR_RANK_PER + 2 * KR_SLACK];
    if (a.flag[0]) return;
    const int T = a.T, tid = threadIdx.x;
    if (tid <= T) soff[tid] = a.candoff[tid];
    lc[tid >> 6][tid & 63] = 0;
    const KrDigit s = kr_shape(a);  // (synchronises)
    const int G = soff[T];
    const int c0 = (blockIdx.x * KR_RANK_PER) / KR_CHUNK - 1;
    for (int p0 = blockIdx.x * KR_RANK_PER; p0 < G; p0 += gridDim.x * KR_RANK_PER) {
        // the keys of positions [p0 - KR_SLACK, p0 + KR_RANK_PER + KR_SLACK) in LDS: the bins of
        // the block's positions, unless one reaches further
        const int l0 = p0 - KR_SLACK, l1 = min(G, p0 + KR_RANK_PER + KR_SLACK);
        __syncthreads();
        for (int q = max(0, l0) + tid; q < l1; q += 256) skey[q - l0] = a.tkey[q];
        __syncthreads();
        for (int p = p0 + tid; p < min(G, p0 + KR_RANK_PER); p += 256) {
            const unsigned long long k = skey[p - l0];
            const int d = kr_digit(k, s);
            const int bs = a.bins[d], be = d == KR_BINS - 1 ? G : a.bins[d + 1];
            int r = bs;
            if (bs >= l0 && be <= l1) {
#pragma unroll 4
                for (int q = bs; q < be; q++) r += skey[q - l0] > k ? 1 : 0;
            } else {
                for (int q = bs; q < be; q++) r += a.tkey[q] > k ? 1 : 0;
            }
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
            const int rc = r / KR_CHUNK - c0;
            if (p0 == blockIdx.x * KR_RANK_PER && rc >= 0 && rc < 4) atomicAdd(&lc[rc][lo], 1);
            else atomicAdd(&a.ccnt[(long long)(r / KR_CHUNK) * KR_TY + lo], 1);
        }
    }
    __syncthreads();
    const int q = tid >> 6, t = tid & 63, v = lc[q][t];
    if (v) atomicAdd(&a.ccnt[(long long)(c0 + q) * KR_TY + t], v);
}

__global__ __launch_bounds__(KR_CHUNK) void k_kr_write(KrArgs a) {
    __shared__ int spre[16][KR_TY], wcnt[16][KR_TY], soff[ADLBQ_MAX_TYPES + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int T = a.T;
    // the next batch starts from zero bins, group counts and (other parity) chunk counts
    const int gt = blockIdx.x * blockDim.x + tid, gs = gridDim.x * blockDim.x;
    for (int k = gt; k < KR_BINS; k += gs) a.bins[k] = 0;
    for (int k = gt; k < KR_COARSE; k += gs) a.coarse[k] = 0;
    for (long long k = gt; k < a.nccnt; k += gs) a.ccnt_next[k] = 0;
    const bool failed = a.flag[0] != 0;
    if (blockIdx.x == 0 && tid == 0) {
        if (failed) {
            a.ctr->kr_fail += 1;
            a.ctr->kr_why = a.flag[0];
        }
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
#pragma unroll 8
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

// The five launches on the handle's stream.  Buffers are sized for the larger
// of the batch's demand bound and the newest landed batch's candidate count;
// a batch with more candidates than that fails over (and sizes the next).
int launch_keyrank(adlbq_server *h, int R) {
    const int T = h->T;
    hipStream_t s = h->stream;
    const long long bound = (long long)R * std::min(T, NREQ) + (long long)T * h->export_extra;
    long long want = bound, grid_n = bound;
    int g_last = 0, lo_last = 0;
    if (plan_hint(h, &g_last, &lo_last)) {
        const long long g = (long long)g_last + g_last / 4 + 4096;
        want = std::max(want, g);
        grid_n = g;  // the grids follow the last batch's count (every loop is grid-strided)
    }
    want = std::max(1024ll, std::min(want, h->cap_cand));
    if (want > h->cap_kr) {
        AQ_HIP(hipStreamSynchronize(s));
        if (h->d_kr) AQ_HIP(hipFree(h->d_kr));
        const long long cap = std::min(std::max(want, 2 * h->cap_kr), std::max(h->cap_cand, 1024ll));
        const long long nch = (cap + KR_CHUNK - 1) / KR_CHUNK;
        const size_t bytes = sizeof(unsigned long long) * 2 * cap + sizeof(int) * (4 * cap + KR_BINS + KR_COARSE + 64) +
                             sizeof(int) * 2 * nch * KR_TY + (size_t)cap + 256;
        AQ_HIP(hipMalloc((void **)&h->d_kr, bytes));
        h->cap_kr = cap;
        AQ_HIP(hipMemsetAsync(h->d_kr, 0, bytes, s));
    }
    const long long cap = h->cap_kr, nch = (cap + KR_CHUNK - 1) / KR_CHUNK;
    char *p = h->d_kr;
    KrArgs a{};
    a.T = T;
    a.candoff = h->d_candoff;
    a.candlen = h->d_candlen;
    a.theta = h->d_theta;
    a.anchor = h->d_anchor;
    {
        const long long npos = std::max<long long>(1, (long long)h->open.pages.size() << PAGE_SHIFT);
        a.nbpos_bits = 64 - __builtin_clzll((unsigned long long)(npos - 1) | 1ull);
    }
    a.ckey = h->d_ckey;
    a.cslot = h->d_cslot;
    a.crank = h->d_crank;
    a.needsort = h->d_needsort;
    a.ctr = h->d_ctr;
    a.tkey = reinterpret_cast<unsigned long long *>(p);
    a.okey = a.tkey + cap;
    a.bins = reinterpret_cast<int *>(a.okey + cap);
    a.coarse = a.bins + KR_BINS;
    a.flag = a.coarse + KR_COARSE;
    a.tidx = a.flag + 64;
    a.oslot = a.tidx + cap;
    a.tslot = a.oslot + cap;
    int *cc = a.tslot + cap;
    h->kr_par ^= 1;
    a.ccnt = cc + (long long)h->kr_par * nch * KR_TY;
    a.ccnt_next = cc + (long long)(h->kr_par ^ 1) * nch * KR_TY;
    a.nccnt = nch * KR_TY;
    a.otype = reinterpret_cast<unsigned char *>(cc + 2 * nch * KR_TY);
    a.cap = cap;
    a.bin_max = h->kr_bin_max;
    const long long gn = std::min(grid_n, cap);
    const int g256 = (int)std::max(1ll, std::min<long long>(2048, (gn + 255) / 256));
    k_kr_hist<<<g256, 256, 0, s>>>(a);
    k_kr_scan<<<KR_COARSE, 256, 0, s>>>(a);
    k_kr_scatter<<<g256, 256, 0, s>>>(a);
    k_kr_rank<<<(int)std::max(1ll, (gn + KR_RANK_PER - 1) / KR_RANK_PER), 256, 0, s>>>(a);
    k_kr_write<<<(int)std::max(64ll, (gn + KR_CHUNK - 1) / KR_CHUNK), KR_CHUNK, 0, s>>>(a);
    AQ_HIP(hipGetLastError());
    h->n_keyrank++;
    return ADLBQ_OK;
}

}  // namespace adlbq
