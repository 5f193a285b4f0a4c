// adlbq_wide.hip -- the ordered choice of a Reserve batch for servers with
// more than ADLBQ_MAX_TYPES (64) work types, where the 64-bit type masks of the
// scan pipeline do not reach (get_type_idx, adlb.c:3476-3485).
//
// A correct, slower path: the available units (live, unpinned, prio above
// ADLB_LOWEST_PRIO) are sorted once per batch into runs keyed by (target rank
// or "untargeted", type index), each run in (prio desc, wqseqno asc) order --
// three stable LSD radix sorts (adlbq_rsx): by wqseqno, then by prio
// descending, then by run key.  The requests then go strictly in order through
// one workgroup: wq_find_pre_targeted_hi_prio (xq.c:219-247) is the best head
// over the request's runs of its own rank, wq_find_hi_prio (xq.c:190-217) the
// best head over its untargeted runs; the winner's run head advances.  Every
// unit is in exactly one run, so a taken unit is never seen again.  k_finalize
// then pins, replies and parks as on the scan path (tmatch = the chosen slot).
#include "adlbq_impl.h"
#include "adlbq_rsx.h"

#include <algorithm>
#include <climits>
#include <vector>

namespace adlbq {

constexpr int WREQ_INTS = 34;  // per request: nt, nu, 16 targeted runs (or lo, hi), 16 untargeted runs (or lo, hi)

// available units of the listed pages: (wqseqno, slot), in any order
__global__ __launch_bounds__(256) void k_wide_gather(const int2 *__restrict__ pages, const uint32_t *__restrict__ meta,
                                                     const int *__restrict__ prio, const int *__restrict__ seqa,
                                                     unsigned long long *__restrict__ key, int *__restrict__ val,
                                                     int *__restrict__ cnt) {
    const int2 pf = pages[blockIdx.x];
    const long long base = (long long)pf.x << PAGE_SHIFT;
    for (int o = threadIdx.x; o < PAGE; o += blockDim.x) {
        bool ok = false;
        long long s = base + o;
        if (o < pf.y) {
            const uint32_t m = meta[s];
            ok = (m & (M_LIVE | M_PINNED)) == M_LIVE && prio[s] > LOWEST;
        }
        const unsigned long long b = __ballot(ok);
        int p0 = 0;
        if ((threadIdx.x & 63) == 0 && b) p0 = atomicAdd(cnt, __popcll(b));
        p0 = __shfl(p0, 0, 64);
        if (ok) {
            const int pos = p0 + __popcll(b & ((1ull << (threadIdx.x & 63)) - 1ull));
            key[pos] = (unsigned int)seqa[s];
            val[pos] = (int)s;
        }
    }
}

// the next sort key of every entry: 1 = prio descending, 2 = run key (target rank or A, type index)
__global__ __launch_bounds__(256) void k_wide_key(int n, int stage, const int *__restrict__ val,
                                                  const int *__restrict__ prio, const uint32_t *__restrict__ meta,
                                                  const int4 *__restrict__ cold1, int A, int sh, int vw,
                                                  unsigned long long *__restrict__ key) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int s = val[i];
    if (stage == 1) {
        key[i] = (unsigned int)~((unsigned int)prio[s] ^ 0x80000000u);
    } else {
        const int tg = cold1[s].w;
        const unsigned int tk = tg < 0 ? (unsigned int)A : tg < A ? (unsigned int)tg : (unsigned int)A + 1u;
        key[i] = ((unsigned long long)tk << sh) | (unsigned long long)meta_type(meta[s], vw);
    }
}

// entry keys (larger = better) for the choice, run starts flagged
__global__ __launch_bounds__(256) void k_wide_ekey(int n, const int *__restrict__ val, const int *__restrict__ prio,
                                                   const int *__restrict__ seqa,
                                                   const unsigned long long *__restrict__ rk,
                                                   unsigned long long *__restrict__ ekey, int *__restrict__ flag) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int s = val[i];
    ekey[i] = make_key(prio[s], (unsigned int)seqa[s]);
    flag[i] = (i == 0 || rk[i] != rk[i - 1]) ? 1 : 0;
}

// one workgroup: the runs (key, start, head) in order, and rstart[nr] = n; cnt[1] = nr
__global__ __launch_bounds__(1024) void k_wide_runs(int n, const int *__restrict__ flag,
                                                    const unsigned long long *__restrict__ rk,
                                                    unsigned long long *__restrict__ rkey, int *__restrict__ rstart,
                                                    int *__restrict__ head, int *__restrict__ cnt) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        const int i = c0 + tid;
        const bool f = i < n && flag[i];
        const unsigned long long b = __ballot(f);
        if (lane == 0) wsum[w] = __popcll(b);
        __syncthreads();
        int pre = base, tot = 0;
        for (int q = 0; q < 16; q++) {
            pre += q < w ? wsum[q] : 0;
            tot += wsum[q];
        }
        if (f) {
            const int r = pre + __popcll(b & ((1ull << lane) - 1ull));
            rkey[r] = rk[i];
            rstart[r] = i;
            head[r] = i;
        }
        base += tot;
        __syncthreads();
    }
    if (tid == 0) {
        rstart[base] = n;
        cnt[1] = base;
    }
}

__device__ __forceinline__ int lower_bound_u64(const unsigned long long *a, int n, unsigned long long x) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// per request (one thread each): (rank, hang) for k_finalize, and the runs the
// choice looks at -- of its own rank (targeted) and of A (untargeted): one run
// per listed type, or the rank's whole range of runs for a -1 anywhere
__global__ __launch_bounds__(256) void k_wide_prep(const int *__restrict__ reqs, int R, const int *__restrict__ utypes,
                                                   int T, int A, const unsigned long long *__restrict__ rkey,
                                                   const int *__restrict__ cnt, int *__restrict__ wreq,
                                                   int2 *__restrict__ rh, int *__restrict__ tmatch,
                                                   int *__restrict__ umatch, int sh,
                                                   const int2 *__restrict__ utsorted, int nut) {
    __shared__ int s_ut[ADLBQ_MAX_TYPES_WIDE];
    if (!utsorted)
        for (int t = threadIdx.x; t < T; t += blockDim.x) s_ut[t] = utypes[t];
    __syncthreads();
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= R) return;
    const int nr = cnt[1];
    const int *q = reqs + (long long)ADLBQ_RESERVE_INTS * j;
    const int rank = q[0];
    rh[j] = make_int2(rank, q[1]);
    tmatch[j] = -1;
    umatch[j] = -1;
    int idx[NREQ], ni = 0;
    bool wild = false;
    for (int e = 0; e < NREQ; e++) {  // wants(): any entry -1 or equal to the unit's type (xq.c:199-207)
        const int v = q[2 + e];
        wild |= v == -1;
        if (v < 0) continue;
        if (utsorted) {  // more than 255 types: binary search in (value, first declared index) by value
            int lo = 0, hi = nut;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (utsorted[mid].x < v) lo = mid + 1;
                else hi = mid;
            }
            if (lo < nut && utsorted[lo].x == v) idx[ni++] = utsorted[lo].y;
            continue;
        }
        for (int t = 0; t < T; t++)
            if (s_ut[t] == v) {  // get_type_idx: the first declared match
                idx[ni++] = t;
                break;
            }
    }
    int *o = wreq + (long long)WREQ_INTS * j;
    for (int side = 0; side < 2; side++) {
        int *oo = o + (side ? 18 : 2);
        const bool valid = side ? true : (rank >= 0 && rank < A);
        const unsigned long long tk = side ? (unsigned long long)A : (unsigned long long)rank;
        int c = 0;
        if (!valid) {
            c = 0;
        } else if (wild) {
            oo[0] = lower_bound_u64(rkey, nr, tk << sh);
            oo[1] = lower_bound_u64(rkey, nr, (tk + 1ull) << sh);
            c = -1;
        } else {
            for (int e = 0; e < ni; e++) {
                const unsigned long long k = (tk << sh) | (unsigned long long)idx[e];
                const int r = lower_bound_u64(rkey, nr, k);
                if (r < nr && rkey[r] == k) oo[c++] = r;
            }
        }
        o[side] = c;
    }
}

// the requests strictly in order, one workgroup: thread i looks at the i-th
// run of the request's side (a wildcard: runs i, i + 256, ...), a block max of
// the heads' keys picks the unit
__global__ __launch_bounds__(256) void k_wide_choose(const int *__restrict__ wreq, int R, const int *__restrict__ rstart,
                                                     int *head, const unsigned long long *__restrict__ ekey,
                                                     const int *__restrict__ val, int *__restrict__ tmatch) {
    __shared__ int s_row[WREQ_INTS];
    __shared__ unsigned long long s_best[4];
    __shared__ int s_run[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int j = 0; j < R; j++) {
        if (tid < WREQ_INTS) s_row[tid] = wreq[(long long)WREQ_INTS * j + tid];
        __syncthreads();
        int chosen = -1;
        for (int side = 0; side < 2 && chosen < 0; side++) {
            const int c = s_row[side];
            const int *oo = s_row + (side ? 18 : 2);
            unsigned long long k = 0;  // the best head this thread sees (keys are unique, 0 = none)
            int kr = -1;
            auto look = [&](int r) {
                const int hd = __hip_atomic_load(head + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (hd < rstart[r + 1] && ekey[hd] > k) k = ekey[hd], kr = r;
            };
            if (c < 0) {  // a wildcard: every run of the side, 256 at a time (more than 255 types: more runs)
                for (int r = oo[0] + tid; r < oo[1]; r += 256) look(r);
            } else if (tid < c) {
                look(oo[tid]);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                const unsigned long long k2 = __shfl_xor(k, o, 64);
                const int r2 = __shfl_xor(kr, o, 64);
                if (k2 > k) k = k2, kr = r2;
            }
            if (lane == 0) {
                s_best[w] = k;
                s_run[w] = kr;
            }
            __syncthreads();
            unsigned long long bk = 0;
            int br = -1;
            for (int q = 0; q < 4; q++)
                if (s_best[q] > bk) bk = s_best[q], br = s_run[q];
            if (bk) {
                if (tid == 0) {
                    const int h = __hip_atomic_load(head + br, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    tmatch[j] = val[h];
                    __hip_atomic_store(head + br, h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                chosen = 1;
            }
            __syncthreads();
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
    }
}

static int wide_cap(adlbq_server *h, long long n, int R, int npg) {
    if (n > h->cap_wn) {
        void *ps[] = {h->d_wk0, h->d_wk1, h->d_wv0, h->d_wv1, h->d_wekey, h->d_wflag, h->d_wrkey, h->d_wrstart,
                      h->d_whead, h->d_wtmp};
        for (void *p : ps)
            if (p) AQ_HIP(hipFree(p));
        h->cap_wn = std::max(n, 2 * h->cap_wn);
        const long long c = h->cap_wn;
        AQ_HIP(hipMalloc((void **)&h->d_wk0, sizeof(unsigned long long) * c));
        AQ_HIP(hipMalloc((void **)&h->d_wk1, sizeof(unsigned long long) * c));
        AQ_HIP(hipMalloc((void **)&h->d_wv0, sizeof(int) * c));
        AQ_HIP(hipMalloc((void **)&h->d_wv1, sizeof(int) * c));
        AQ_HIP(hipMalloc((void **)&h->d_wekey, sizeof(unsigned long long) * c));
        AQ_HIP(hipMalloc((void **)&h->d_wflag, sizeof(int) * c));
        AQ_HIP(hipMalloc((void **)&h->d_wrkey, sizeof(unsigned long long) * (c + 1)));
        AQ_HIP(hipMalloc((void **)&h->d_wrstart, sizeof(int) * (c + 1)));
        AQ_HIP(hipMalloc((void **)&h->d_whead, sizeof(int) * (c + 1)));
        h->cap_wtmp = rsx_temp_bytes(c);
        AQ_HIP(hipMalloc((void **)&h->d_wtmp, h->cap_wtmp));
    }
    if (R > h->cap_wreq) {
        if (h->d_wreq) AQ_HIP(hipFree(h->d_wreq));
        h->cap_wreq = std::max(R, 2 * h->cap_wreq);
        AQ_HIP(hipMalloc((void **)&h->d_wreq, sizeof(int) * WREQ_INTS * (size_t)h->cap_wreq));
    }
    if (npg > h->cap_wpages) {
        if (h->d_wpages) AQ_HIP(hipFree(h->d_wpages));
        h->cap_wpages = std::max(npg, 2 * h->cap_wpages);
        AQ_HIP(hipMalloc((void **)&h->d_wpages, sizeof(int2) * (size_t)h->cap_wpages));
    }
    if (!h->d_wcnt) AQ_HIP(hipMalloc((void **)&h->d_wcnt, sizeof(int) * 2));
    return ADLBQ_OK;
}

// the batch's choices into tmatch (a slot or -1; umatch all -1) and (rank, hang) into d_rh
int wide_choose(adlbq_server *h, int R, const int *d_reqs) {
    hipStream_t s = h->stream;
    // every bucket's pages with their fills (the slow path synchronises: its buffers are reused)
    std::vector<int2> pg;
    auto add = [&](const Bucket &b) {
        for (size_t i = 0; i < b.pages.size(); i++)
            pg.push_back(make_int2(b.pages[i], i + 1 == b.pages.size() ? b.tail_fill : PAGE));
    };
    add(h->open);
    for (const Bucket &b : h->rankb) add(b);
    const long long nmax = (long long)pg.size() * PAGE;
    int rc;
    AQ_HIP(hipStreamSynchronize(s));
    if ((rc = wide_cap(h, std::max(nmax, 1ll), R, std::max((int)pg.size(), 1)))) return rc;
    if (!pg.empty()) AQ_HIP(hipMemcpy(h->d_wpages, pg.data(), sizeof(int2) * pg.size(), hipMemcpyHostToDevice));
    AQ_HIP(hipMemsetAsync(h->d_wcnt, 0, sizeof(int) * 2, s));
    AQ_HIP(hipMemsetAsync(h->d_needsort, 0, sizeof(int) * std::max(h->T, 1), s));  // k_finalize's tail reads it
    if (!pg.empty())
        k_wide_gather<<<(unsigned)pg.size(), 256, 0, s>>>(h->d_wpages, h->d_meta, h->d_prio, h->d_seq, h->d_wk0,
                                                          h->d_wv0, h->d_wcnt);
    int n = 0;
    AQ_HIP(hipMemcpyAsync(&h->h_result[0], h->d_wcnt, sizeof(int), hipMemcpyDeviceToHost, s));
    AQ_HIP(hipStreamSynchronize(s));
    n = h->h_result[0];
    // by wqseqno, then prio descending, then run key: each sort stable, so runs end up (prio desc, seqno asc)
    if ((rc = rsx_sort_pairs(h->d_wtmp, h->cap_wtmp, h->d_wk0, h->d_wk1, h->d_wv0, h->d_wv1, n, 0, 32, false, s)))
        return rc;
    const unsigned nb = (unsigned)std::max(1, (n + 255) / 256);
    // run key: (target rank, or A for untargeted, or A + 1) above the type index's sh bits
    const int vw = h->T > VW_TYPES ? 1 : 0;
    int sh = 8, tb = 1;
    while ((1ll << sh) < h->T) sh++;
    while ((1ll << tb) < (long long)h->A + 2) tb++;
    if (n > 0) k_wide_key<<<nb, 256, 0, s>>>(n, 1, h->d_wv1, h->d_prio, h->d_meta, h->d_cold1, h->A, sh, vw, h->d_wk0);
    if ((rc = rsx_sort_pairs(h->d_wtmp, h->cap_wtmp, h->d_wk0, h->d_wk1, h->d_wv1, h->d_wv0, n, 0, 32, false, s)))
        return rc;
    if (n > 0) k_wide_key<<<nb, 256, 0, s>>>(n, 2, h->d_wv0, h->d_prio, h->d_meta, h->d_cold1, h->A, sh, vw, h->d_wk0);
    if ((rc = rsx_sort_pairs(h->d_wtmp, h->cap_wtmp, h->d_wk0, h->d_wk1, h->d_wv0, h->d_wv1, n, 0, sh + tb, false, s)))
        return rc;
    if (n > 0)
        k_wide_ekey<<<nb, 256, 0, s>>>(n, h->d_wv1, h->d_prio, h->d_seq, h->d_wk1, h->d_wekey, h->d_wflag);
    k_wide_runs<<<1, 1024, 0, s>>>(n, h->d_wflag, h->d_wk1, h->d_wrkey, h->d_wrstart, h->d_whead, h->d_wcnt);
    k_wide_prep<<<(R + 255) / 256, 256, 0, s>>>(d_reqs, R, h->d_utypes, h->T, h->A, h->d_wrkey, h->d_wcnt, h->d_wreq,
                                                h->d_rh, h->d_tmatch, h->d_umatch, sh, vw ? h->d_utsorted : nullptr,
                                                h->n_utsorted);
    k_wide_choose<<<1, 256, 0, s>>>(h->d_wreq, R, h->d_wrstart, h->d_whead, h->d_wekey, h->d_wv1, h->d_tmatch);
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

}  // namespace adlbq
