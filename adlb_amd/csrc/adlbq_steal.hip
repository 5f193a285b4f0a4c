// adlbq_steal.hip -- the cross-shard steal round.
//
// The reference moves work between servers with SS_RFR / SS_RFR_RESP round
// trips: a server with a parked Reserve asks the donor its (stale) qmstat
// table names (find_cand_rank_with_worktype, adlb.c:3487-3534); the donor runs
// wq_find_pre_targeted_hi_prio / wq_find_hi_prio for the requesting rank and
// pins the unit (adlb.c:1802-1866); the requester answers the app and drops
// the rq entry (adlb.c:1868-1933).  Here one steal round settles every parked
// Reserve of every shard at once:
//
//   1. each shard exports, per work type, its k best available units
//      (adlbq_steal_export, a scan on the device) and its live rq entries
//      (adlbq_rq_export);
//   2. the exports are all-gathered (RCCL over xGMI, adlb_amd/shards.py);
//   3. every shard runs the same deterministic merge (adlbq_steal_merge,
//      host code below) -- the round-trips serialised in (shard, rqseqno)
//      order, each against the donors' current state;
//   4. donors pin what the merge granted (adlbq_grant_batch) and requesters
//      drop the settled rq entries (adlbq_rq_delete_batch).
//
// The merge restates, per parked Reserve in that order:
//   * donor choice (adlb.c:1280-1308 with 3487-3534): the first entry of the
//     type vector (up to the first value below -1) that has a donor; donor =
//     the other shard with the highest available prio of that type (wildcard
//     -1: of any type), strict > ADLB_LOWEST_PRIO, the lowest index on ties.
//     The table is fresh (every earlier steal of the round applied) and no
//     RFR is outstanding, so rfr_out never excludes a shard;
//   * the donor's unit (adlb.c:1816-1818): its best available unit over the
//     request's whole type set (wq_find_hi_prio semantics: -1 anywhere in the
//     16 entries = any type), prio desc then wqseqno asc.
// The merge sees only exported units: it stops at the first Reserve whose
// decision would need a unit below a shard's exported top k (that Reserve
// and every later one stay parked for the next round).  Units targeted at the
// requesting rank that sit on the donor (pre-targeted match, adlb.c:1816) and
// tq entries (adlb.c:3493-3498) exist only after puts that landed away from
// the target's home server (adlb.c:2767-2768, 2845-2852); the round does not
// model them.
#include "adlbq_impl.h"

#include <algorithm>
#include <chrono>
#include <climits>
#include <string>
#include <cstring>

using namespace adlbq;

namespace {

// donor side of SS_RFR: pin_rank = for_rank, pinned = (for_rank >= 0)
// (adlb.c:1820-1824) for units still live, unpinned and untargeted.
// found (optional) per pair; bad (optional) counts the pairs that were not.
__device__ __forceinline__ void grant_pair(int i, const int *__restrict__ pairs, int n,
                                           const long long *__restrict__ seq2slot, long long nseq, uint32_t *meta,
                                           int *pin, const int *__restrict__ seqa, const int4 *__restrict__ cold1,
                                           int *__restrict__ found, int *bad) {
    int ok = 0;
    if (i < n) {
        const int rank = pairs[2 * i], seq = pairs[2 * i + 1];
        const long long slot = (seq > 0 && seq < nseq) ? seq2slot[seq] : -1;
        if (slot >= 0) {
            const uint32_t m = meta[slot];
            if ((m & (M_LIVE | M_PINNED)) == M_LIVE && seqa[slot] == seq && cold1[slot].w < 0) {
                // the pin is claimed atomically: of two grants of one unit the first to land wins
                ok = rank < 0 || !(atomicOr(&meta[slot], M_PINNED) & M_PINNED);
                if (ok) pin[slot] = rank;
            }
        }
        if (found) found[i] = ok;
    }
    const unsigned long long b = __ballot(i < n && !ok);
    if (bad && (threadIdx.x & 63) == 0 && b) atomicAdd(bad, __popcll(b));
}

__global__ void k_grant(const int *__restrict__ pairs, int n, const long long *__restrict__ seq2slot,
                        long long nseq, uint32_t *meta, int *pin, const int *__restrict__ seqa,
                        const int4 *__restrict__ cold1, int *__restrict__ found, int *bad) {
    grant_pair(blockIdx.x * blockDim.x + threadIdx.x, pairs, n, seq2slot, nseq, meta, pin, seqa, cold1, found, bad);
}

__global__ void k_rfr_reset(int *rfr_to_rank, int A, int *rfr_out, int nworld, int *hdr = nullptr, int idx = 0) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < A) rfr_to_rank[i] = -1;
    if (i < nworld) rfr_out[i] = 0;
    if (hdr && i == 0) hdr[0] = idx;  // a steal group region's shard index
}

// rq_find_seqno + rq_delete for many rqseqnos (adlb.c:1883, 1933)
__global__ void k_rq_delete_batch(const int *__restrict__ rqseqnos, int n, int *rq_live,
                                  const int *__restrict__ rq_seq, const DevCounters *ctr, int *found, int *ndel,
                                  int *bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int hit = 0;
    if (i < n) {
        const int k = rq_slot_of(rq_seq, ctr->rq_n, rqseqnos[i]);
        if (k >= 0 && atomicExch(&rq_live[k], 0)) hit = 1;
        if (found) found[i] = hit;
    }
    const unsigned long long b = __ballot(hit), m = __ballot(i < n && !hit);
    if ((threadIdx.x & 63) == 0) {
        if (b) atomicAdd(ndel, __popcll(b));
        if (bad && m) atomicAdd(bad, __popcll(m));
    }
}

// rq->count bookkeeping and the new FIFO head (first live entry), 1024 slots per step
__global__ __launch_bounds__(1024) void k_rq_delete_fix(const int *rq_live, DevCounters *ctr, int *ndel) {
    __shared__ int s_first;
    const int head = ctr->rq_head, n = ctr->rq_n;
    if (threadIdx.x == 0) {
        ctr->rq_live -= *ndel;
        bytes_add(ctr, -BYTES_RQ * *ndel);  // rq_delete per settled Reserve (adlb.c:1933)
        *ndel = 0;
        s_first = n;
    }
    __syncthreads();
    for (int base = head; base < n; base += 1024) {
        const int k = base + threadIdx.x;
        if (k < n && rq_live[k]) atomicMin(&s_first, k);
        __syncthreads();
        const int f = s_first;
        __syncthreads();  // every thread has read it before the next step may lower it
        if (f < n) break;
    }
    if (threadIdx.x == 0) ctr->rq_head = s_first;
}

// k_rq_delete_batch + k_rq_delete_fix in one launch: the last workgroup to
// arrive (ticket) does the bookkeeping and finds the new FIFO head, reading
// rq_live at agent scope (the other workgroups' exchanges, not a stale line)
__device__ __forceinline__ void rq_delete_settle_blk(int bid, int nblk, const int *__restrict__ rqseqnos, int n,
                                                     int *rq_live, const int *__restrict__ rq_seq, DevCounters *ctr,
                                                     int *ndel, int *bad, int *ticket) {
    __shared__ int s_first;
    __shared__ bool s_last;
    const int i = bid * blockDim.x + threadIdx.x;
    int hit = 0;
    if (i < n) {
        const int k = rq_slot_of(rq_seq, ctr->rq_n, rqseqnos[i]);
        if (k >= 0 && atomicExch(&rq_live[k], 0)) hit = 1;
    }
    const unsigned long long b = __ballot(hit), m = __ballot(i < n && !hit);
    if ((threadIdx.x & 63) == 0) {
        if (b) atomicAdd(ndel, __popcll(b));
        if (m) atomicAdd(bad, __popcll(m));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        s_last = atomicAdd(ticket, 1) == nblk - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    const int head = ctr->rq_head, nn = ctr->rq_n;
    if (threadIdx.x == 0) {
        const int nd = __hip_atomic_load(ndel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ctr->rq_live -= nd;
        bytes_add(ctr, -BYTES_RQ * nd);  // rq_delete per settled Reserve (adlb.c:1933)
        *ndel = 0;
        *ticket = 0;
        s_first = nn;
    }
    __syncthreads();
    for (int base = head; base < nn; base += blockDim.x) {
        const int k = base + threadIdx.x;
        if (k < nn && __hip_atomic_load(rq_live + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(&s_first, k);
        __syncthreads();
        const int f = s_first;
        __syncthreads();  // every thread has read it before the next step may lower it
        if (f < nn) break;
    }
    if (threadIdx.x == 0) ctr->rq_head = s_first;
}

// k_rq_delete_batch + k_rq_delete_fix in one launch: the last workgroup to
// arrive (ticket) does the bookkeeping and finds the new FIFO head, reading
// rq_live at agent scope (the other workgroups' exchanges, not a stale line)
__global__ __launch_bounds__(256) void k_rq_delete_settle(const int *__restrict__ rqseqnos, int n, int *rq_live,
                                                          const int *__restrict__ rq_seq, DevCounters *ctr,
                                                          int *ndel, int *bad, int *ticket) {
    rq_delete_settle_blk(blockIdx.x, gridDim.x, rqseqnos, n, rq_live, rq_seq, ctr, ndel, bad, ticket);
}

// One group settle's grants and rq deletions for every local shard in one
// launch: blockIdx.y = shard, blocks [0, gb) of a row grant, the rest delete
// (the last of those to arrive fixes that shard's rq head).
struct ShardApply {
    const int *pairs, *dels;
    int ngrant, ndel;
    const long long *seq2slot;
    long long nseq;
    uint32_t *meta;
    int *pin;
    const int *seqa;
    const int4 *cold1;
    int *apply_bad;  // [bad grants, bad deletes, deleted, settle ticket]
    int *rq_live;
    const int *rq_seq;
    DevCounters *ctr;
};

__global__ __launch_bounds__(256) void k_group_apply(const ShardApply *__restrict__ tab, int gb) {
    const ShardApply a = tab[blockIdx.y];
    if ((int)blockIdx.x < gb) {
        if ((int)blockIdx.x * 256 < a.ngrant)
            grant_pair(blockIdx.x * 256 + threadIdx.x, a.pairs, a.ngrant, a.seq2slot, a.nseq, a.meta, a.pin, a.seqa,
                       a.cold1, nullptr, a.apply_bad);
        return;
    }
    if (a.ndel == 0) return;
    rq_delete_settle_blk((int)blockIdx.x - gb, (int)gridDim.x - gb, a.dels, a.ndel, a.rq_live, a.rq_seq, a.ctr,
                         a.apply_bad + 2, a.apply_bad + 1, a.apply_bad + 3);
}

// The grants' SS_UNRESERVE for every local shard in one launch (blockIdx.y = shard).
struct ShardUnres {
    const int *trip;
    int n;
    const long long *seq2slot;
    long long nseq;
    uint32_t *meta;
    int *pin;
    const int4 *rrec;
    long long *anchor;
};

__global__ __launch_bounds__(256) void k_group_unreserve(const ShardUnres *__restrict__ tab) {
    const ShardUnres a = tab[blockIdx.y];
    if ((int)blockIdx.x * 256 >= a.n) return;  // whole waves return together (raise_anchor)
    unreserve_triple(blockIdx.x * 256 + threadIdx.x, a.trip, a.n, a.seq2slot, a.nseq, a.meta, a.pin, a.rrec, a.anchor);
}

// The live rq entries in FIFO order, compacted: out[0] = count, then up to cap
// entries {rqseqno, world_rank, req_types[16]}.  One workgroup of 1024.
struct RfrReset {  // k_rfr_reset's work, done by k_rq_compact when it runs anyway (rfr_to_rank == nullptr: none)
    int *rfr_to_rank, A, *rfr_out, nworld, *hdr, idx;
};

__device__ __forceinline__ void rq_compact_body(const int *__restrict__ rq_live, const int *__restrict__ rq_rank,
                                                const int *__restrict__ rq_types, const int *__restrict__ rq_seq,
                                                const DevCounters *ctr, int cap, int *__restrict__ out,
                                                const RfrReset &rr) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (rr.rfr_to_rank) {
        for (int i = tid; i < rr.A || i < rr.nworld; i += blockDim.x) {
            if (i < rr.A) rr.rfr_to_rank[i] = -1;
            if (i < rr.nworld) rr.rfr_out[i] = 0;
        }
        if (rr.hdr && tid == 0) rr.hdr[0] = rr.idx;
    }
    const int head = ctr->rq_head, n = ctr->rq_n;
    int base = 0;
    for (int c0 = head; c0 < n; c0 += 1024) {
        const int k = c0 + tid;
        const bool live = k < n && rq_live[k];
        const unsigned long long b = __ballot(live);
        if (lane == 0) wsum[w] = __popcll(b);
        __syncthreads();
        int pre = base, tot = 0;
        for (int q = 0; q < 16; q++) {
            pre += q < w ? wsum[q] : 0;
            tot += wsum[q];
        }
        const int pos = pre + __popcll(b & lanemask_lt());
        if (live && pos < cap) {
            int *o = out + 1 + (long long)pos * 18;
            o[0] = rq_seq[k];
            o[1] = rq_rank[k];
            const int4 *src = reinterpret_cast<const int4 *>(rq_types + (long long)k * NREQ);
#pragma unroll
            for (int q = 0; q < NREQ / 4; q++) {
                const int4 v = src[q];
                o[2 + 4 * q] = v.x;
                o[3 + 4 * q] = v.y;
                o[4 + 4 * q] = v.z;
                o[5 + 4 * q] = v.w;
            }
        }
        base += tot;
        __syncthreads();
    }
    if (tid == 0) out[0] = base;
}

__global__ __launch_bounds__(1024) void k_rq_compact(const int *__restrict__ rq_live, const int *__restrict__ rq_rank,
                                                     const int *__restrict__ rq_types,
                                                     const int *__restrict__ rq_seq, const DevCounters *ctr,
                                                     int cap, int *__restrict__ out, RfrReset rr) {
    rq_compact_body(rq_live, rq_rank, rq_types, rq_seq, ctr, cap, out, rr);
}

// adlbq_steal_group_export: the shards' k_rq_compact as one launch, one workgroup per shard
struct RqCompactArgs {
    const int *rq_live, *rq_rank, *rq_types, *rq_seq;
    const DevCounters *ctr;
    int cap;
    int *out;
    RfrReset rr;
};
struct RqCompactGroup {
    RqCompactArgs a[EXPORT_GROUP];
};
__global__ __launch_bounds__(1024) void k_rq_compact_g(const RqCompactGroup g) {
    const RqCompactArgs &a = g.a[blockIdx.x];
    rq_compact_body(a.rq_live, a.rq_rank, a.rq_types, a.rq_seq, a.ctr, a.cap, a.out, a.rr);
}

// ---------------------------------------------------------------- merge (host)
// Max over a range of shards of one type's list heads, lowest shard on ties:
// an iterative segment tree of keys (prio, -shard).
struct HeadTree {
    int P = 1;
    std::vector<unsigned long long> v;
    static unsigned long long key(int prio, int s) {
        return ((unsigned long long)((unsigned int)prio ^ 0x80000000u) << 32) | (0xffffffffu - (unsigned int)s);
    }
    void init(int S) {
        while (P < S) P <<= 1;
        v.assign(2 * P, 0);
    }
    void set(int s, int prio) {
        int i = s + P;
        v[i] = key(prio, s);
        for (i >>= 1; i; i >>= 1) v[i] = std::max(v[2 * i], v[2 * i + 1]);
    }
    unsigned long long query(int l, int r) const {  // [l, r)
        unsigned long long m = 0;
        for (l += P, r += P; l < r; l >>= 1, r >>= 1) {
            if (l & 1) m = std::max(m, v[l++]);
            if (r & 1) m = std::max(m, v[--r]);
        }
        return m;
    }
    unsigned long long except(int i, int S) const { return std::max(query(0, i), query(i + 1, S)); }
};

inline int key_prio(unsigned long long k) { return (int)((unsigned int)(k >> 32) ^ 0x80000000u); }
inline int key_shard(unsigned long long k) { return (int)(0xffffffffu - (unsigned int)k); }

struct ShardView {
    const int *recs;          // [T][k][8]
    const int *nrec;          // [T]
    const long long *navail;  // [T]
};

}  // namespace

// the merge over S shards' exports, each given by a view (adlbq_steal_merge)
static int merge_views(int S, int T, const int *user_types, int k, const ShardView *vw, int nreq, const int *reqs19,
                       int *out3, int *n_decided) {
    for (int r = 0; r < nreq; r++) {
        const int *q = reqs19 + (size_t)r * 19;
        if (q[0] < 0 || q[0] >= S) return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: shard index out of range");
        if (r && (q[0] < q[-19] || (q[0] == q[-19] && q[1] <= q[-18])))
            return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: requests not in (shard, rqseqno) order");
    }
    for (int s = 0; s < S; s++)
        for (int t = 0; t < T; t++)
            if (!vw[s].nrec || vw[s].nrec[t] < 0 || vw[s].nrec[t] > k || vw[s].navail[t] < vw[s].nrec[t])
                return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: bad record counts (or a shard index without export)");
    auto tindex = [&](int v) {
        for (int t = 0; t < T; t++)
            if (user_types[t] == v) return t;
        return -1;
    };
    std::vector<int> head((size_t)S * T, 0), unk_cnt(T, 0);
    std::vector<char> unk((size_t)S * T, 0);
    std::vector<HeadTree> tree(T);
    auto rec = [&](int s, int t, int i) { return vw[s].recs + ((size_t)t * k + i) * 8; };
    // a list past its exported records is LOWEST when the shard had no more, else unknown
    auto refresh = [&](int s, int t) {
        const size_t st = (size_t)s * T + t;
        const bool more = head[st] < vw[s].nrec[t];
        const bool u = !more && vw[s].navail[t] > vw[s].nrec[t];
        if (u && !unk[st]) unk_cnt[t]++;
        unk[st] = u;
        tree[t].set(s, more ? rec(s, t, head[st])[0] : LOWEST);
    };
    for (int t = 0; t < T; t++) {
        tree[t].init(S);
        for (int s = 0; s < S; s++) refresh(s, t);
    }
    int r = 0;
    for (; r < nreq; r++) {
        const int *q = reqs19 + (size_t)r * 19;
        const int me = q[0];
        const int *types = q + 3;
        int *o = out3 + (size_t)r * 3;
        o[0] = o[1] = o[2] = -1;
        bool stop = false;
        int donor = -1;
        for (int e = 0; e < NREQ && donor < 0 && !stop; e++) {
            const int v = types[e];
            if (v < -1) break;
            unsigned long long best = 0;
            if (v == -1) {
                for (int t = 0; t < T && !stop; t++) {
                    stop = unk_cnt[t] - unk[(size_t)me * T + t] > 0;
                    best = std::max(best, tree[t].except(me, S));
                }
            } else {
                const int t = tindex(v);
                if (t < 0) continue;  // undeclared type: no donor (the reference reads out of bounds)
                stop = unk_cnt[t] - unk[(size_t)me * T + t] > 0;
                best = tree[t].except(me, S);
            }
            // ties between types of one shard keep the lower shard (key order)
            if (!stop && best && key_prio(best) > LOWEST) donor = key_shard(best);
        }
        if (stop) break;
        if (donor < 0) continue;
        // the donor's best unit over the request's whole type set
        unsigned long long set = 0;
        for (int e = 0; e < NREQ; e++) {
            const int v = types[e];
            if (v < -1) break;  // padding: the client fills every entry after the list's end with -2
            if (v == -1) set = T == 64 ? ~0ull : ((1ull << T) - 1);
            else {
                const int t = tindex(v);
                if (t >= 0) set |= 1ull << t;
            }
        }
        int bt = -1, bp = LOWEST, bs = INT_MAX;
        for (int t = 0; t < T && !stop; t++) {
            if (!((set >> t) & 1)) continue;
            const size_t st = (size_t)donor * T + t;
            if (unk[st]) stop = true;
            else if (head[st] < vw[donor].nrec[t]) {
                const int *x = rec(donor, t, head[st]);
                if (x[0] > bp || (x[0] == bp && x[1] < bs)) bt = t, bp = x[0], bs = x[1];
            }
        }
        if (stop) break;
        if (bt < 0) return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: donor without a unit (inconsistent records)");
        o[0] = donor;
        o[1] = bt;
        o[2] = head[(size_t)donor * T + bt]++;
        refresh(donor, bt);
    }
    *n_decided = r;
    for (int i = r; i < nreq; i++) out3[3 * i] = out3[3 * i + 1] = out3[3 * i + 2] = -1;
    return ADLBQ_OK;
}


// the grants (k_grant) and rq deletions of one shard from device-resident inputs,
// on the shard's stream (adlbq_steal_apply, and the group's one-copy settle)
static int steal_apply_launch(adlbq_server *h, int ngrant, const int *d_pairs, int ndel, const int *d_dels) {
    wq_changed(h);
    if (!h->d_apply_bad) {  // [bad grants, bad deletes, deleted, settle ticket]
        AQ_HIP(hipMalloc((void **)&h->d_apply_bad, sizeof(int) * 4));
        AQ_HIP(hipMemsetAsync(h->d_apply_bad, 0, sizeof(int) * 4, h->stream));
    }
    if (ngrant)
        k_grant<<<(ngrant + 255) / 256, 256, 0, h->stream>>>(d_pairs, ngrant, h->d_seq2slot, h->next_wqseqno,
                                                            h->d_meta, h->d_pin, h->d_seq, h->d_cold1, nullptr,
                                                            h->d_apply_bad);
    if (ndel) {
        k_rq_delete_settle<<<(ndel + 255) / 256, 256, 0, h->stream>>>(d_dels, ndel, h->d_rq_live, h->d_rq_seq,
                                                                     h->d_ctr,
                                                                     h->d_apply_bad + 2, h->d_apply_bad + 1,
                                                                     h->d_apply_bad + 3);
        h->ctr_stale = true;
    }
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

static int ensure_steal_buffers(adlbq_server *h, int k, int rqcap) {
    const int T = h->T;
    const long long n_out = (long long)T * k * 8 + T, n_rq = 1 + (long long)rqcap * 18;
    const long long n_host = n_out + 2ll * T + n_rq;
    if (n_out > h->cap_export || n_rq > h->cap_rqx || n_host > h->cap_hsteal) AQ_HIP(hipStreamSynchronize(h->stream));
    if (n_out > h->cap_export) {
        if (h->d_export) AQ_HIP(hipFree(h->d_export));
        AQ_HIP(hipMalloc((void **)&h->d_export, sizeof(int) * n_out));
        h->cap_export = n_out;
    }
    if (!h->d_navail) AQ_HIP(hipMalloc((void **)&h->d_navail, sizeof(long long) * std::max(T, 1)));
    if (n_rq > h->cap_rqx) {
        if (h->d_rqx) AQ_HIP(hipFree(h->d_rqx));
        const long long nc = std::max(n_rq, 2 * h->cap_rqx);
        AQ_HIP(hipMalloc((void **)&h->d_rqx, sizeof(int) * nc));
        h->cap_rqx = nc;
    }
    if (n_host > h->cap_hsteal) {
        if (h->h_steal) AQ_HIP(hipHostFree(h->h_steal));
        const long long nc = std::max(n_host, 2 * h->cap_hsteal);
        AQ_HIP(hipHostMalloc((void **)&h->h_steal, sizeof(int) * nc, hipHostMallocDefault));
        h->cap_hsteal = nc;
    }
    if (!h->steal_ev) AQ_HIP(hipEventCreateWithFlags(&h->steal_ev, hipEventDisableTiming));
    return ADLBQ_OK;
}

extern "C" {

int adlbq_steal_begin(adlbq_server *h, int k) {
    if (!h || k < 1) return fail(ADLBQ_ERR_ARG, "adlbq_steal_begin");
    hipSetDevice(h->device);
    const int T = h->T;
    // the round answers every SS_RFR the parks of this shard sent (resp[11]):
    // as each SS_RFR_RESP would (adlb.c:1877-1878), rfr_to_rank = -1 and
    // rfr_out = 0, so later parks and check_remote see no RFR outstanding
    // (k_rfr_reset, or inside k_rq_compact below; the export reads neither table)
    const RfrReset rr{h->d_rfr_to_rank, h->A, h->d_rfr_out, h->num_world, nullptr, 0};
    // every live rq entry fits: the landed-snapshot bound, else the whole capacity
    const long long up = rq_live_upper(h);
    const int rqcap = (int)std::max(0ll, std::min<long long>(up, h->rq_cap));
    int rc;
    if ((rc = ensure_steal_buffers(h, k, rqcap))) return rc;
    if (T && (rc = launch_export(h, k, h->d_export, h->d_navail))) return rc;
    if (h->rq_cap > 0) {
        k_rq_compact<<<1, 1024, 0, h->stream>>>(h->d_rq_live, h->d_rq_rank, h->d_rq_types, h->d_rq_seq, h->d_ctr, rqcap, h->d_rqx,
                                                rr);
    } else {
        k_rfr_reset<<<(std::max(std::max(h->A, h->num_world), 1) + 255) / 256, 256, 0, h->stream>>>(
            h->d_rfr_to_rank, h->A, h->d_rfr_out, h->num_world);
        AQ_HIP(hipMemsetAsync(h->d_rqx, 0, sizeof(int), h->stream));
    }
    AQ_HIP(hipGetLastError());
    const long long n_out = (long long)T * k * 8 + T;
    int *hs = h->h_steal;
    if (T) {
        AQ_HIP(hipMemcpyAsync(hs, h->d_export, sizeof(int) * n_out, hipMemcpyDeviceToHost, h->stream));
        AQ_HIP(hipMemcpyAsync(hs + n_out, h->d_navail, sizeof(long long) * T, hipMemcpyDeviceToHost, h->stream));
    }
    AQ_HIP(hipMemcpyAsync(hs + n_out + 2 * T, h->d_rqx, sizeof(int) * (1 + (size_t)rqcap * 18), hipMemcpyDeviceToHost,
                          h->stream));
    AQ_HIP(hipEventRecord(h->steal_ev, h->stream));
    h->steal_k = k;
    h->steal_rqcap = rqcap;
    return ADLBQ_OK;
}

int adlbq_steal_collect(adlbq_server *h, int *recs8, int *nrec, long long *navail, int cap, int *out18,
                        int *count) {
    if (!h || cap < 0 || (cap && !out18)) return fail(ADLBQ_ERR_ARG, "adlbq_steal_collect");
    if (h->steal_k < 0) return fail(ADLBQ_ERR_ARG, "adlbq_steal_collect: no adlbq_steal_begin in flight");
    hipSetDevice(h->device);
    AQ_HIP(hipEventSynchronize(h->steal_ev));
    const int T = h->T, k = h->steal_k;
    const long long n_out = (long long)T * k * 8 + T;
    const int *hs = h->h_steal;
    if (recs8) std::memcpy(recs8, hs, sizeof(int) * (size_t)T * k * 8);
    if (nrec) std::memcpy(nrec, hs + (size_t)T * k * 8, sizeof(int) * T);
    if (navail) std::memcpy(navail, hs + n_out, sizeof(long long) * T);
    const int *rq = hs + n_out + 2 * T;
    const int c = rq[0];
    if (c > h->steal_rqcap) return fail(ADLBQ_ERR_ARG, "adlbq_steal_collect: rq bound violated");
    if (out18) std::memcpy(out18, rq + 1, sizeof(int) * 18 * (size_t)std::min(c, cap));
    if (count) *count = c;
    h->steal_k = -1;
    return ADLBQ_OK;
}

int adlbq_steal_export(adlbq_server *h, int k, int *recs8, int *nrec, long long *navail) {
    if (!h || k < 1 || (h->T && (!nrec || !navail || !recs8))) return fail(ADLBQ_ERR_ARG, "adlbq_steal_export");
    int rc;
    if ((rc = adlbq_steal_begin(h, k))) return rc;
    return adlbq_steal_collect(h, recs8, nrec, navail, 0, nullptr, nullptr);
}

int adlbq_steal_apply(adlbq_server *h, int ngrant, const int *pairs2, int ndel, const int *rqseqnos) {
    if (h) wq_changed(h);
    if (!h || ngrant < 0 || ndel < 0 || (ngrant && !pairs2) || (ndel && !rqseqnos))
        return fail(ADLBQ_ERR_ARG, "adlbq_steal_apply");
    if (!ngrant && !ndel) return ADLBQ_OK;
    hipSetDevice(h->device);
    const long long need = 2ll * ngrant + ndel;
    if (h->apply_ev) AQ_HIP(hipEventSynchronize(h->apply_ev));  // the staging of the previous apply is free
    else AQ_HIP(hipEventCreateWithFlags(&h->apply_ev, hipEventDisableTiming));
    if (need > h->cap_happly) {
        if (h->h_apply) AQ_HIP(hipHostFree(h->h_apply));
        const long long nc = std::max(need, 2 * h->cap_happly);
        AQ_HIP(hipHostMalloc((void **)&h->h_apply, sizeof(int) * nc, hipHostMallocDefault));
        h->cap_happly = nc;
    }
    if (need > h->cap_dapply) {
        AQ_HIP(hipStreamSynchronize(h->stream));
        if (h->d_apply) AQ_HIP(hipFree(h->d_apply));
        const long long nc = std::max(need, 2 * h->cap_dapply);
        AQ_HIP(hipMalloc((void **)&h->d_apply, sizeof(int) * nc));
        h->cap_dapply = nc;
    }
    if (ngrant) std::memcpy(h->h_apply, pairs2, sizeof(int) * 2 * (size_t)ngrant);
    if (ndel) std::memcpy(h->h_apply + 2 * (size_t)ngrant, rqseqnos, sizeof(int) * (size_t)ndel);
    AQ_HIP(hipMemcpyAsync(h->d_apply, h->h_apply, sizeof(int) * need, hipMemcpyHostToDevice, h->stream));
    AQ_HIP(hipEventRecord(h->apply_ev, h->stream));
    return steal_apply_launch(h, ngrant, h->d_apply, ndel, h->d_apply + 2 * (size_t)ngrant);
}

int adlbq_steal_check(adlbq_server *h, int *bad_grants, int *bad_deletes) {
    if (!h || !bad_grants || !bad_deletes) return fail(ADLBQ_ERR_ARG, "adlbq_steal_check");
    hipSetDevice(h->device);
    *bad_grants = *bad_deletes = 0;
    if (!h->d_apply_bad) return ADLBQ_OK;
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_apply_bad, sizeof(int) * 2, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipMemsetAsync(h->d_apply_bad, 0, sizeof(int) * 2, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    *bad_grants = h->h_result[0];
    *bad_deletes = h->h_result[1];
    return ADLBQ_OK;
}

int adlbq_rq_export(adlbq_server *h, int cap, int *out18, int *count) {
    if (!h || cap < 0 || !count || (cap && !out18)) return fail(ADLBQ_ERR_ARG, "adlbq_rq_export");
    hipSetDevice(h->device);
    int rc;
    if ((rc = refresh_counters(h))) return rc;
    const int k0 = h->ctr.rq_head, n = h->ctr.rq_n - k0;
    *count = 0;
    if (n <= 0) return ADLBQ_OK;
    std::vector<int> live(n), rank(n), seq(n), types((size_t)n * NREQ);
    AQ_HIP(hipMemcpyAsync(live.data(), h->d_rq_live + k0, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipMemcpyAsync(seq.data(), h->d_rq_seq + k0, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipMemcpyAsync(rank.data(), h->d_rq_rank + k0, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipMemcpyAsync(types.data(), h->d_rq_types + (size_t)k0 * NREQ, sizeof(int) * types.size(),
                          hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    int c = 0;
    for (int i = 0; i < n; i++) {
        if (!live[i]) continue;
        if (c < cap) {
            int *o = out18 + (size_t)c * 18;
            o[0] = seq[i];  // rqseqno
            o[1] = rank[i];
            std::memcpy(o + 2, types.data() + (size_t)i * NREQ, sizeof(int) * NREQ);
        }
        c++;
    }
    *count = c;
    return ADLBQ_OK;
}

int adlbq_grant_batch(adlbq_server *h, int n, const int *pairs2, int *found) {
    if (h) wq_changed(h);
    if (!h || n < 0 || (n && (!pairs2 || !found))) return fail(ADLBQ_ERR_ARG, "adlbq_grant_batch");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    int *d = nullptr;
    AQ_HIP(hipMallocAsync((void **)&d, sizeof(int) * 3 * (size_t)n, h->stream));
    AQ_HIP(hipMemcpyAsync(d, pairs2, sizeof(int) * 2 * (size_t)n, hipMemcpyHostToDevice, h->stream));
    k_grant<<<(n + 255) / 256, 256, 0, h->stream>>>(d, n, h->d_seq2slot, h->next_wqseqno, h->d_meta, h->d_pin,
                                                   h->d_seq, h->d_cold1, d + 2 * (size_t)n, nullptr);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipMemcpyAsync(found, d + 2 * (size_t)n, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipFreeAsync(d, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    return ADLBQ_OK;
}

int adlbq_rq_delete_batch(adlbq_server *h, int n, const int *rqseqnos, int *found) {
    if (!h || n < 0 || (n && (!rqseqnos || !found))) return fail(ADLBQ_ERR_ARG, "adlbq_rq_delete_batch");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    int *d = nullptr;
    AQ_HIP(hipMallocAsync((void **)&d, sizeof(int) * (2 * (size_t)n + 1), h->stream));
    AQ_HIP(hipMemcpyAsync(d, rqseqnos, sizeof(int) * n, hipMemcpyHostToDevice, h->stream));
    AQ_HIP(hipMemsetAsync(d + 2 * (size_t)n, 0, sizeof(int), h->stream));
    k_rq_delete_batch<<<(n + 255) / 256, 256, 0, h->stream>>>(d, n, h->d_rq_live, h->d_rq_seq, h->d_ctr, d + n,
                                                              d + 2 * (size_t)n,
                                                              nullptr);
    k_rq_delete_fix<<<1, 1024, 0, h->stream>>>(h->d_rq_live, h->d_ctr, d + 2 * (size_t)n);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipMemcpyAsync(found, d + n, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipFreeAsync(d, h->stream));
    h->ctr_stale = true;
    return refresh_counters(h);
}

// ---------------------------------------------------------------- steal group
// The steal round for the shards one process holds, without a per-shard host
// round trip: every shard's export lands in one device blob (region per
// shard), the blobs of all processes are gathered by the caller (RCCL) or
// used as they are, one copy brings them to pinned host memory, the merge
// runs here, and each local shard gets its grants / deletions enqueued on its
// own stream (no synchronisation; adlbq_steal_group_check reads the counters).
}  // extern "C"

struct adlbq_steal_group {
    std::vector<adlbq_server *> sh;
    int n = 0, k = 0, T = 0, rqcap = 0;
    int group_launch = 1;       // the export's kernels as one launch for the shards (adlbq_steal_group_set_param)
    long long off_recs = 0, off_nrec = 0, off_nav = 0, off_rq = 0, blob = 0;
    int *d_own = nullptr;       // the local blob when the caller passes none
    int *d_last = nullptr;      // where the last export went
    int *h_all = nullptr;       // pinned copy of the gathered blobs
    // one process: the export written straight into mapped pinned memory (no copy before the merge)
    int *h_map = nullptr, *d_map = nullptr;
    long long cap_map = 0;
    bool last_mapped = false;
    int zero_copy = 1;          // ADLBQ_STEAL_ZERO_COPY=0: device blob + one copy (A/B runs)
    long long cap_h = 0;
    std::vector<hipEvent_t> ev;
    std::vector<int> reqs, out3, resp;  // merge scratch; resp [m][15] of the last settle
    std::vector<std::vector<int>> grants, dels;
    int *h_unr = nullptr, *d_unr = nullptr;  // SS_UNRESERVE staging of the grants
    long long cap_unr = 0;
    int *h_app = nullptr, *d_app = nullptr;  // every shard's grants + rq deletions, one copy per settle
    long long cap_app = 0;
    hipEvent_t app_ev = nullptr;
    hipEvent_t app_done_ev = nullptr;  // after k_group_apply: the other shards' streams wait for it
    hipEvent_t unr_ev = nullptr;  // the grants' SS_UNRESERVE staging copy (first shard's stream)
    std::vector<hipEvent_t> jev;  // join: the first shard's stream waits for every other shard's stream
    long long ns_copy = 0, ns_merge = 0, ns_apply = 0, nreq_last = 0;  // the last settle's host phases
};

extern "C" {

int adlbq_steal_group_create(adlbq_steal_group **out, adlbq_server **shards, int n, int k, int rqcap) {
    if (!out || !shards || n < 1 || k < 1 || rqcap < 0) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_create");
    for (int j = 0; j < n; j++)
        if (!shards[j] || shards[j]->T != shards[0]->T || shards[j]->device != shards[0]->device ||
            shards[j]->utypes != shards[0]->utypes || shards[j]->S != shards[0]->S)
            return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_create: shards differ in types, device or server count");
    auto *g = new adlbq_steal_group();
    g->sh.assign(shards, shards + n);
    for (int j = 0; j < n; j++) shards[j]->export_extra = std::max(shards[j]->export_extra, k);
    g->n = n, g->k = k, g->T = shards[0]->T, g->rqcap = rqcap;
    if (const char *e = std::getenv("ADLBQ_STEAL_GROUP_LAUNCH")) g->group_launch = std::atoi(e) != 0;  // A/B runs
    if (const char *e = std::getenv("ADLBQ_STEAL_ZERO_COPY")) g->zero_copy = std::atoi(e) != 0;
    const long long T = g->T;
    g->off_recs = 2;                                  // [0] shard index, [1] pad
    g->off_nrec = g->off_recs + T * k * 8;            // launch_export writes nrec right after the records
    g->off_nav = (g->off_nrec + T + 1) & ~1ll;        // 8-byte aligned long long navail[T]
    g->off_rq = g->off_nav + 2 * T;                   // count, then rqcap x 18
    g->blob = (g->off_rq + 1 + 18ll * rqcap + 63) & ~63ll;
    hipSetDevice(shards[0]->device);
    g->ev.resize((size_t)n);
    for (auto &e : g->ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            delete g;
            return fail(ADLBQ_ERR_HIP, "adlbq_steal_group_create: hipEventCreate");
        }
    *out = g;
    return ADLBQ_OK;
}

long long adlbq_steal_group_blob_ints(adlbq_steal_group *g) { return g ? g->blob * g->n : -1; }

int adlbq_steal_group_export(adlbq_steal_group *g, int *d_blob) {
    if (!g) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_export");
    hipSetDevice(g->sh[0]->device);
    g->last_mapped = false;
    if (!d_blob && g->zero_copy) {  // the merge reads the kernels' stores where they landed
        const long long need = g->blob * g->n;
        if (need > g->cap_map) {
            for (auto *h : g->sh) AQ_HIP(hipStreamSynchronize(h->stream));
            if (g->h_map) AQ_HIP(hipHostFree(g->h_map));
            g->h_map = g->d_map = nullptr;
            AQ_HIP(hipHostMalloc((void **)&g->h_map, sizeof(int) * need, hipHostMallocMapped));
            AQ_HIP(hipHostGetDevicePointer((void **)&g->d_map, g->h_map, 0));
            g->cap_map = need;
        }
        d_blob = g->d_map;
        g->last_mapped = true;
    } else if (!d_blob) {
        if (!g->d_own) AQ_HIP(hipMalloc((void **)&g->d_own, sizeof(int) * g->blob * g->n));
        d_blob = g->d_own;
    }
    g->d_last = d_blob;
    // shards whose last batch's lists serve the export and that have an rq: both kernels as one
    // launch each for all of them (grid.z / grid.x = shard), EXPORT_GROUP at a time
    std::vector<int> m;
    ExportAfterGroup eg{};
    RqCompactGroup rg{};
    int Tmax = 0, rc;
    auto flush = [&]() -> int {
        if (m.empty()) return ADLBQ_OK;
        int r2;
        if ((r2 = group_join(g->sh.data(), m))) return r2;
        hipStream_t ls = g->sh[(size_t)m[0]]->stream;
        if ((r2 = launch_export_after_group(eg, (int)m.size(), g->k, Tmax, ls))) return r2;
        k_rq_compact_g<<<(unsigned)m.size(), 1024, 0, ls>>>(rg);
        AQ_HIP(hipGetLastError());
        if ((r2 = group_release(g->sh.data(), m))) return r2;
        for (int j : m)
            if (g->sh[(size_t)j]->stream != g->sh[0]->stream) AQ_HIP(hipEventRecord(g->ev[(size_t)j], g->sh[(size_t)j]->stream));
        m.clear();
        Tmax = 0;
        return ADLBQ_OK;
    };
    for (int j = 0; j < g->n; j++) {
        adlbq_server *h = g->sh[(size_t)j];
        int *r = d_blob + (size_t)j * g->blob;
        // every SS_RFR of this shard's parks is answered by the round (adlb.c:1877-1878):
        // the reset rides in k_rq_compact (the export reads neither table)
        const RfrReset rr{h->d_rfr_to_rank, h->A, h->d_rfr_out, h->num_world, r, h->my_idx};
        long long *nav = reinterpret_cast<long long *>(r + g->off_nav);
        const size_t q = m.size();
        if (g->group_launch && g->T && h->rq_cap > 0 && g->rqcap > 0 &&
            export_after_args(h, g->k, r + g->off_recs, r + g->off_nrec, nav, &eg.a[q])) {
            rg.a[q] = RqCompactArgs{h->d_rq_live, h->d_rq_rank, h->d_rq_types, h->d_rq_seq, h->d_ctr, g->rqcap,
                                    r + g->off_rq, rr};
            Tmax = std::max(Tmax, h->T);
            m.push_back(j);
            if (m.size() == (size_t)EXPORT_GROUP && (rc = flush())) return rc;
            continue;
        }
        if (g->T && !launch_export_after(h, g->k, r + g->off_recs, r + g->off_nrec, nav) &&
            (rc = launch_export(h, g->k, r + g->off_recs, nav)))
            return rc;
        if (h->rq_cap > 0 && g->rqcap > 0) {
            k_rq_compact<<<1, 1024, 0, h->stream>>>(h->d_rq_live, h->d_rq_rank, h->d_rq_types, h->d_rq_seq, h->d_ctr, g->rqcap,
                                                    r + g->off_rq, rr);
        } else {
            k_rfr_reset<<<(std::max(std::max(h->A, h->num_world), 1) + 255) / 256, 256, 0, h->stream>>>(
                h->d_rfr_to_rank, h->A, h->d_rfr_out, h->num_world, r, h->my_idx);
            AQ_HIP(hipMemsetAsync(r + g->off_rq, 0, sizeof(int), h->stream));
        }
        AQ_HIP(hipGetLastError());
        if (h->stream != g->sh[0]->stream) AQ_HIP(hipEventRecord(g->ev[(size_t)j], h->stream));
    }
    return flush();
}

}  // extern "C"

static int group_host_cap(adlbq_steal_group *g, long long total) {
    if (total > g->cap_h) {
        if (g->h_all) AQ_HIP(hipHostFree(g->h_all));
        g->h_all = nullptr;
        AQ_HIP(hipHostMalloc((void **)&g->h_all, sizeof(int) * total, hipHostMallocDefault));
        g->cap_h = total;
    }
    return ADLBQ_OK;
}

static int group_settle_staged(adlbq_steal_group *g, const int *all, int nproc, int *n_decided, int *n_settled,
                               std::chrono::steady_clock::time_point t0, std::chrono::steady_clock::time_point t1);

extern "C" {

int adlbq_steal_group_settle(adlbq_steal_group *g, const int *d_all, int nproc, int *n_decided, int *n_settled) {
    if (!g || nproc < 1 || (nproc > 1 && !d_all)) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_settle");
    adlbq_server *h0 = g->sh[0];
    hipSetDevice(h0->device);
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    if (!d_all && nproc == 1 && g->last_mapped) {  // the export landed in mapped memory: no copy
        for (int j = 0; j < g->n; j++)
            if (g->sh[(size_t)j]->stream != h0->stream) AQ_HIP(hipStreamWaitEvent(h0->stream, g->ev[(size_t)j], 0));
        AQ_HIP(hipStreamSynchronize(h0->stream));
        return group_settle_staged(g, g->h_map, 1, n_decided, n_settled, t0, clk::now());
    }
    if (!d_all) d_all = g->d_last;
    if (!d_all) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_settle: no export");
    const long long total = g->blob * g->n * nproc;
    int rc;
    if ((rc = group_host_cap(g, total))) return rc;
    for (int j = 0; j < g->n; j++)  // shards on the first shard's stream are ordered already (no event)
        if (g->sh[(size_t)j]->stream != h0->stream) AQ_HIP(hipStreamWaitEvent(h0->stream, g->ev[(size_t)j], 0));
    AQ_HIP(hipMemcpyAsync(g->h_all, d_all, sizeof(int) * total, hipMemcpyDeviceToHost, h0->stream));
    AQ_HIP(hipStreamSynchronize(h0->stream));
    return group_settle_staged(g, g->h_all, nproc, n_decided, n_settled, t0, clk::now());
}

int adlbq_steal_group_export_host(adlbq_steal_group *g, int *h_blob) {
    if (!g || !h_blob) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_export_host");
    int rc;
    if ((rc = adlbq_steal_group_export(g, nullptr))) return rc;
    adlbq_server *h0 = g->sh[0];
    for (int j = 0; j < g->n; j++)  // shards on the first shard's stream are ordered already (no event)
        if (g->sh[(size_t)j]->stream != h0->stream) AQ_HIP(hipStreamWaitEvent(h0->stream, g->ev[(size_t)j], 0));
    if (g->last_mapped) {  // already in host memory
        AQ_HIP(hipStreamSynchronize(h0->stream));
        std::memcpy(h_blob, g->h_map, sizeof(int) * g->blob * g->n);
        return ADLBQ_OK;
    }
    AQ_HIP(hipMemcpyAsync(h_blob, g->d_last, sizeof(int) * g->blob * g->n, hipMemcpyDeviceToHost, h0->stream));
    AQ_HIP(hipStreamSynchronize(h0->stream));
    return ADLBQ_OK;
}

int adlbq_steal_group_settle_host(adlbq_steal_group *g, const int *h_all, int nproc, int *n_decided, int *n_settled) {
    if (!g || nproc < 1 || !h_all) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_settle_host");
    hipSetDevice(g->sh[0]->device);
    const long long total = g->blob * g->n * nproc;
    int rc;
    if ((rc = group_host_cap(g, total))) return rc;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    std::memcpy(g->h_all, h_all, sizeof(int) * total);
    return group_settle_staged(g, g->h_all, nproc, n_decided, n_settled, t0, clk::now());
}

}  // extern "C"

// A one-launch settle step (k_group_apply / k_group_unreserve) runs on the
// first shard's stream but writes every shard's queue: that stream first waits
// for the work already enqueued on every other shard's stream.
static int group_join_streams(adlbq_steal_group *g) {
    adlbq_server *h0 = g->sh[0];
    if (g->jev.size() != (size_t)g->n) {
        g->jev.assign((size_t)g->n, nullptr);
        for (auto &e : g->jev) AQ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    for (int j = 0; j < g->n; j++) {
        adlbq_server *h = g->sh[(size_t)j];
        if (h == h0 || h->stream == h0->stream) continue;
        AQ_HIP(hipEventRecord(g->jev[(size_t)j], h->stream));
        AQ_HIP(hipStreamWaitEvent(h0->stream, g->jev[(size_t)j], 0));
    }
    return ADLBQ_OK;
}

// The merge and the local side of it over all = [nproc][n][blob] (any region order).
static int group_settle_staged(adlbq_steal_group *g, const int *all, int nproc, int *n_decided, int *n_settled,
                               std::chrono::steady_clock::time_point t0, std::chrono::steady_clock::time_point t1) {
    using clk = std::chrono::steady_clock;
    adlbq_server *h0 = g->sh[0];
    const int S = h0->S, T = g->T, nreg = g->n * nproc;
    std::vector<ShardView> vw((size_t)S, ShardView{nullptr, nullptr, nullptr});
    std::vector<int> local_of((size_t)S, -1);
    for (int j = 0; j < g->n; j++) local_of[(size_t)g->sh[(size_t)j]->my_idx] = j;
    // (shard, rqseqno) order: each region's rq is in FIFO (rqseqno) order, so the
    // regions in shard order (regions may come in any order) give it directly
    std::vector<int> reg_of((size_t)S, -1);
    for (int r = 0; r < nreg; r++) {
        const int *b = all + (size_t)r * g->blob;
        const int idx = b[0];
        if (idx < 0 || idx >= S || reg_of[(size_t)idx] >= 0)
            return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_settle: bad or repeated shard index");
        reg_of[(size_t)idx] = r;
        vw[(size_t)idx] = ShardView{b + g->off_recs, b + g->off_nrec, reinterpret_cast<const long long *>(b + g->off_nav)};
    }
    g->reqs.clear();
    for (int idx = 0; idx < S; idx++) {
        if (reg_of[(size_t)idx] < 0) continue;
        const int *rq = all + (size_t)reg_of[(size_t)idx] * g->blob + g->off_rq;
        const int c = std::min(rq[0], g->rqcap);  // entries past rqcap wait for the next round
        const size_t o = g->reqs.size();
        g->reqs.resize(o + 19 * (size_t)c);
        int *dst = g->reqs.data() + o;
        for (int i = 0; i < c; i++, dst += 19) {
            dst[0] = idx;
            std::memcpy(dst + 1, rq + 1 + 18 * (size_t)i, sizeof(int) * 18);
        }
    }
    const int nreq = (int)(g->reqs.size() / 19);
    g->out3.assign(3 * (size_t)nreq, -1);
    int nd = 0, rc;
    if (nreq && (rc = merge_views(S, T, h0->utypes.data(), g->k, vw.data(), nreq, g->reqs.data(), g->out3.data(), &nd)))
        return rc;
    const auto t2 = clk::now();
    g->grants.assign((size_t)g->n, {});
    g->dels.assign((size_t)g->n, {});
    g->resp.clear();
    int won = 0;
    for (int i = 0; i < nd; i++) {
        const int d = g->out3[3 * (size_t)i];
        if (d < 0) continue;
        won++;
        const int *q = &g->reqs[19 * (size_t)i];
        const int *u = vw[(size_t)d].recs + ((size_t)g->out3[3 * (size_t)i + 1] * g->k + g->out3[3 * (size_t)i + 2]) * 8;
        if (local_of[(size_t)d] >= 0) {  // donor side: pin for the requesting rank (adlb.c:1820-1824)
            auto &gr = g->grants[(size_t)local_of[(size_t)d]];
            gr.push_back(q[2]);
            gr.push_back(u[1]);
        }
        const int lj = local_of[(size_t)q[0]];
        if (lj >= 0) {  // requester side: rq_delete + the reply to the app (adlb.c:1884-1933)
            g->dels[(size_t)lj].push_back(q[1]);
            const int r15[15] = {q[0], q[1], q[2], 1, u[2], u[0], u[3], u[4], u[1], h0->master + d, u[5], u[6], u[7],
                                 -1, -1};
            g->resp.insert(g->resp.end(), r15, r15 + 15);
        }
    }
    // every shard's grants and deletions staged together with a table of
    // per-shard arguments: one copy and one launch (k_group_apply) on the first
    // shard's stream, the other shards' streams ordered behind it
    long long tot = 0;
    int mg = 0, md = 0;
    for (int j = 0; j < g->n; j++) {
        tot += (long long)g->grants[(size_t)j].size() + (long long)g->dels[(size_t)j].size();
        mg = std::max(mg, (int)(g->grants[(size_t)j].size() / 2));
        md = std::max(md, (int)g->dels[(size_t)j].size());
    }
    if (tot > 0) {
        const long long toff = (tot + 1) & ~1ll;  // the table 8-byte aligned after the payload
        const long long need = toff + (long long)(sizeof(ShardApply) / sizeof(int)) * g->n;
        if (g->app_ev) AQ_HIP(hipEventSynchronize(g->app_ev));  // the previous settle's copy has left the staging
        else AQ_HIP(hipEventCreateWithFlags(&g->app_ev, hipEventDisableTiming));
        if (!g->app_done_ev) AQ_HIP(hipEventCreateWithFlags(&g->app_done_ev, hipEventDisableTiming));
        if (need > g->cap_app) {
            for (auto *h : g->sh) AQ_HIP(hipStreamSynchronize(h->stream));
            if (g->h_app) AQ_HIP(hipHostFree(g->h_app));
            if (g->d_app) AQ_HIP(hipFree(g->d_app));
            g->cap_app = std::max<long long>({need, 2 * g->cap_app, 1ll << 18});
            AQ_HIP(hipHostMalloc((void **)&g->h_app, sizeof(int) * g->cap_app, hipHostMallocDefault));
            AQ_HIP(hipMalloc((void **)&g->d_app, sizeof(int) * g->cap_app));
        }
        ShardApply *tab = reinterpret_cast<ShardApply *>(g->h_app + toff);
        long long off = 0;
        for (int j = 0; j < g->n; j++) {
            adlbq_server *h = g->sh[(size_t)j];
            const auto &gr = g->grants[(size_t)j];
            const auto &dl = g->dels[(size_t)j];
            if (!gr.empty()) std::memcpy(g->h_app + off, gr.data(), sizeof(int) * gr.size());
            if (!dl.empty()) std::memcpy(g->h_app + off + gr.size(), dl.data(), sizeof(int) * dl.size());
            if (!h->d_apply_bad) {  // [bad grants, bad deletes, deleted, settle ticket]
                AQ_HIP(hipMalloc((void **)&h->d_apply_bad, sizeof(int) * 4));
                AQ_HIP(hipMemset(h->d_apply_bad, 0, sizeof(int) * 4));
            }
            tab[j] = ShardApply{g->d_app + off, g->d_app + off + gr.size(), (int)(gr.size() / 2), (int)dl.size(),
                                h->d_seq2slot, h->next_wqseqno, h->d_meta, h->d_pin, h->d_seq, h->d_cold1,
                                h->d_apply_bad, h->d_rq_live, h->d_rq_seq, h->d_ctr};
            if (!gr.empty() || !dl.empty()) wq_changed(h);
            if (!dl.empty()) h->ctr_stale = true;
            off += (long long)gr.size() + (long long)dl.size();
        }
        if ((rc = group_join_streams(g))) return rc;
        AQ_HIP(hipMemcpyAsync(g->d_app, g->h_app, sizeof(int) * need, hipMemcpyHostToDevice, h0->stream));
        AQ_HIP(hipEventRecord(g->app_ev, h0->stream));
        const int gb = (mg + 255) / 256, db = (md + 255) / 256;
        k_group_apply<<<dim3(gb + db, g->n), 256, 0, h0->stream>>>(reinterpret_cast<const ShardApply *>(g->d_app + toff),
                                                                   gb);
        AQ_HIP(hipGetLastError());
        AQ_HIP(hipEventRecord(g->app_done_ev, h0->stream));
        for (int j = 0; j < g->n; j++)
            if (g->sh[(size_t)j]->stream != h0->stream)
                AQ_HIP(hipStreamWaitEvent(g->sh[(size_t)j]->stream, g->app_done_ev, 0));
    }
    const auto t3 = clk::now();
    g->ns_copy = std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    g->ns_merge = std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
    g->ns_apply = std::chrono::duration_cast<std::chrono::nanoseconds>(t3 - t2).count();
    g->nreq_last = nreq;
    if (n_decided) *n_decided = nd;
    if (n_settled) *n_settled = won;
    return ADLBQ_OK;
}

extern "C" {

int adlbq_steal_group_unreserve_grants(adlbq_steal_group *g) {
    if (!g) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_unreserve_grants");
    if (g->grants.size() != (size_t)g->n) return ADLBQ_OK;
    long long total = 0;
    for (const auto &gr : g->grants) total += (long long)(gr.size() / 2);
    if (!total) return ADLBQ_OK;
    hipSetDevice(g->sh[0]->device);
    // the staging is free: the previous round's copy (first shard's stream) completed
    // before this round's settle returned.  Every shard's triples and a table of
    // per-shard arguments in one copy, one launch on the first shard's stream
    adlbq_server *h0 = g->sh[0];
    const long long toff = (3 * total + 1) & ~1ll;
    const long long need = toff + (long long)(sizeof(ShardUnres) / sizeof(int)) * g->n;
    if (need > g->cap_unr) {
        for (auto *h : g->sh) AQ_HIP(hipStreamSynchronize(h->stream));
        if (g->h_unr) AQ_HIP(hipHostFree(g->h_unr));
        if (g->d_unr) AQ_HIP(hipFree(g->d_unr));
        g->cap_unr = std::max<long long>({need, 2 * g->cap_unr, 1ll << 18});
        AQ_HIP(hipHostMalloc((void **)&g->h_unr, sizeof(int) * g->cap_unr, hipHostMallocDefault));
        AQ_HIP(hipMalloc((void **)&g->d_unr, sizeof(int) * g->cap_unr));
    }
    ShardUnres *tab = reinterpret_cast<ShardUnres *>(g->h_unr + toff);
    long long off = 0;
    int mx = 0;
    for (int j = 0; j < g->n; j++) {
        adlbq_server *h = g->sh[(size_t)j];
        const auto &gr = g->grants[(size_t)j];
        const int m = (int)(gr.size() / 2);
        int *hb = g->h_unr + off;
        for (int i = 0; i < m; i++) hb[3 * i] = gr[2 * (size_t)i], hb[3 * i + 1] = gr[2 * (size_t)i + 1], hb[3 * i + 2] = -1;
        tab[j] = ShardUnres{g->d_unr + off, m, h->d_seq2slot, h->next_wqseqno, h->d_meta, h->d_pin, h->d_rrec,
                            h->d_anchor};
        if (m) wq_changed(h);
        mx = std::max(mx, m);
        off += 3ll * m;
    }
    if (!g->unr_ev) AQ_HIP(hipEventCreateWithFlags(&g->unr_ev, hipEventDisableTiming));
    int rc;
    if ((rc = group_join_streams(g))) return rc;
    AQ_HIP(hipMemcpyAsync(g->d_unr, g->h_unr, sizeof(int) * (size_t)need, hipMemcpyHostToDevice, h0->stream));
    k_group_unreserve<<<dim3((mx + 255) / 256, g->n), 256, 0, h0->stream>>>(
        reinterpret_cast<const ShardUnres *>(g->d_unr + toff));
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipEventRecord(g->unr_ev, h0->stream));
    for (int j = 0; j < g->n; j++)
        if (g->sh[(size_t)j]->stream != h0->stream) AQ_HIP(hipStreamWaitEvent(g->sh[(size_t)j]->stream, g->unr_ev, 0));
    return ADLBQ_OK;
}

long long adlbq_steal_group_stat(adlbq_steal_group *g, const char *name) {
    if (!g || !name) return -1;
    const std::string n(name);
    if (n == "copy_ns") return g->ns_copy;
    if (n == "merge_ns") return g->ns_merge;
    if (n == "apply_ns") return g->ns_apply;
    if (n == "requests") return g->nreq_last;
    return -1;
}

int adlbq_steal_group_responses(adlbq_steal_group *g, int cap, int *out15, int *count) {
    if (!g || !count || cap < 0 || (cap && !out15)) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_responses");
    const int m = (int)(g->resp.size() / 15);
    if (out15) std::memcpy(out15, g->resp.data(), sizeof(int) * 15 * (size_t)std::min(m, cap));
    *count = m;
    return ADLBQ_OK;
}

int adlbq_steal_group_grants(adlbq_steal_group *g, int cap, int *out3, int *count) {
    if (!g || !count || cap < 0 || (cap && !out3)) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_grants");
    int m = 0;
    for (int j = 0; j < g->n && g->grants.size() == (size_t)g->n; j++) {
        const auto &gr = g->grants[(size_t)j];
        for (size_t i = 0; i + 1 < gr.size(); i += 2, m++)
            if (m < cap) out3[3 * m] = j, out3[3 * m + 1] = gr[i], out3[3 * m + 2] = gr[i + 1];
    }
    *count = m;
    return ADLBQ_OK;
}

int adlbq_steal_group_check(adlbq_steal_group *g, int *bad_grants, int *bad_deletes) {
    if (!g || !bad_grants || !bad_deletes) return fail(ADLBQ_ERR_ARG, "adlbq_steal_group_check");
    *bad_grants = *bad_deletes = 0;
    for (auto *h : g->sh) {
        int a = 0, b = 0, rc;
        if ((rc = adlbq_steal_check(h, &a, &b))) return rc;
        *bad_grants += a;
        *bad_deletes += b;
    }
    return ADLBQ_OK;
}

int adlbq_steal_group_destroy(adlbq_steal_group *g) {
    if (!g) return ADLBQ_OK;
    hipSetDevice(g->sh[0]->device);
    for (auto *h : g->sh) hipStreamSynchronize(h->stream);
    for (auto &e : g->ev) hipEventDestroy(e);
    if (g->d_own) hipFree(g->d_own);
    if (g->h_all) hipHostFree(g->h_all);
    if (g->h_map) hipHostFree(g->h_map);
    if (g->h_unr) hipHostFree(g->h_unr);
    if (g->d_unr) hipFree(g->d_unr);
    if (g->h_app) hipHostFree(g->h_app);
    if (g->d_app) hipFree(g->d_app);
    if (g->app_ev) hipEventDestroy(g->app_ev);
    if (g->app_done_ev) hipEventDestroy(g->app_done_ev);
    if (g->unr_ev) hipEventDestroy(g->unr_ev);
    for (auto &e : g->jev) hipEventDestroy(e);
    delete g;
    return ADLBQ_OK;
}

int adlbq_steal_merge(int S, int T, const int *user_types, int k, const int *recs8, const int *nrec,
                      const long long *navail, int nreq, const int *reqs19, int *out3, int *n_decided) {
    if (S < 1 || T < 0 || T > ADLBQ_MAX_TYPES || k < 0 || nreq < 0 || !n_decided ||
        (T && (!user_types || !nrec || !navail || (k && !recs8))) || (nreq && (!reqs19 || !out3)))
        return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: bad argument");
    std::vector<ShardView> v((size_t)S);
    for (int s = 0; s < S; s++)
        v[(size_t)s] = ShardView{recs8 + (size_t)s * T * k * 8, nrec + (size_t)s * T, navail + (size_t)s * T};
    return merge_views(S, T, user_types, k, v.data(), nreq, reqs19, out3, n_decided);
}

}  // extern "C"
