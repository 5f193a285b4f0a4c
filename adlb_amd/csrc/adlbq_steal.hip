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
#include <climits>
#include <cstring>

using namespace adlbq;

namespace {

// donor side of SS_RFR: pin_rank = for_rank, pinned = (for_rank >= 0)
// (adlb.c:1820-1824) for units still live, unpinned and untargeted
__global__ void k_grant(const int *__restrict__ pairs, int n, const long long *__restrict__ seq2slot,
                        long long nseq, uint32_t *meta, int *pin, const int *__restrict__ seqa,
                        const int4 *__restrict__ cold1, int *__restrict__ found) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int rank = pairs[2 * i], seq = pairs[2 * i + 1];
    const long long slot = (seq > 0 && seq < nseq) ? seq2slot[seq] : -1;
    int ok = 0;
    if (slot >= 0) {
        const uint32_t m = meta[slot];
        if ((m & (M_LIVE | M_PINNED)) == M_LIVE && seqa[slot] == seq && cold1[slot].w < 0) {
            pin[slot] = rank;
            if (rank >= 0) meta[slot] = m | M_PINNED;
            ok = 1;
        }
    }
    found[i] = ok;
}

// rq_find_seqno + rq_delete for many rqseqnos (adlb.c:1883, 1933)
__global__ void k_rq_delete_batch(const int *__restrict__ rqseqnos, int n, int *rq_live, const DevCounters *ctr,
                                  int *found, int *ndel) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int hit = 0;
    if (i < n) {
        const int k = rqseqnos[i] - 1;
        if (k >= 0 && k < ctr->rq_n && atomicExch(&rq_live[k], 0)) hit = 1;
        found[i] = hit;
    }
    const unsigned long long b = __ballot(hit);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(ndel, __popcll(b));
}

__global__ void k_rq_delete_fix(int *rq_live, DevCounters *ctr, int *ndel) {
    ctr->rq_live -= *ndel;
    *ndel = 0;
    int head = ctr->rq_head;
    while (head < ctr->rq_n && !rq_live[head]) head++;
    ctr->rq_head = head;
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

}  // namespace

extern "C" {

int adlbq_rq_export(adlbq_server *h, int cap, int *out18, int *count) {
    if (!h || cap < 0 || !count || (cap && !out18)) return fail(ADLBQ_ERR_ARG, "adlbq_rq_export");
    hipSetDevice(h->device);
    int rc;
    if ((rc = refresh_counters(h))) return rc;
    const int k0 = h->ctr.rq_head, n = h->ctr.rq_n - k0;
    *count = 0;
    if (n <= 0) return ADLBQ_OK;
    std::vector<int> live(n), rank(n), types((size_t)n * NREQ);
    AQ_HIP(hipMemcpyAsync(live.data(), h->d_rq_live + k0, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipMemcpyAsync(rank.data(), h->d_rq_rank + k0, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipMemcpyAsync(types.data(), h->d_rq_types + (size_t)k0 * NREQ, sizeof(int) * types.size(),
                          hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    int c = 0;
    for (int i = 0; i < n; i++) {
        if (!live[i]) continue;
        if (c < cap) {
            int *o = out18 + (size_t)c * 18;
            o[0] = k0 + i + 1;  // rqseqno
            o[1] = rank[i];
            std::memcpy(o + 2, types.data() + (size_t)i * NREQ, sizeof(int) * NREQ);
        }
        c++;
    }
    *count = c;
    return ADLBQ_OK;
}

int adlbq_grant_batch(adlbq_server *h, int n, const int *pairs2, int *found) {
    if (!h || n < 0 || (n && (!pairs2 || !found))) return fail(ADLBQ_ERR_ARG, "adlbq_grant_batch");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    int *d = nullptr;
    AQ_HIP(hipMallocAsync((void **)&d, sizeof(int) * 3 * (size_t)n, h->stream));
    AQ_HIP(hipMemcpyAsync(d, pairs2, sizeof(int) * 2 * (size_t)n, hipMemcpyHostToDevice, h->stream));
    k_grant<<<(n + 255) / 256, 256, 0, h->stream>>>(d, n, h->d_seq2slot, h->next_wqseqno, h->d_meta, h->d_pin,
                                                   h->d_seq, h->d_cold1, d + 2 * (size_t)n);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipMemcpyAsync(found, d + 2 * (size_t)n, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipFreeAsync(d, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    h->qm_dirty = true;
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
    k_rq_delete_batch<<<(n + 255) / 256, 256, 0, h->stream>>>(d, n, h->d_rq_live, h->d_ctr, d + n, d + 2 * (size_t)n);
    k_rq_delete_fix<<<1, 1, 0, h->stream>>>(h->d_rq_live, h->d_ctr, d + 2 * (size_t)n);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipMemcpyAsync(found, d + n, sizeof(int) * n, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipFreeAsync(d, h->stream));
    h->ctr_stale = true;
    return refresh_counters(h);
}

int adlbq_steal_merge(int S, int T, const int *user_types, int k, const int *recs8, const int *nrec,
                      const long long *navail, int nreq, const int *reqs19, int *out3, int *n_decided) {
    if (S < 1 || T < 0 || T > ADLBQ_MAX_TYPES || k < 0 || nreq < 0 || !n_decided ||
        (T && (!user_types || !nrec || !navail || (k && !recs8))) || (nreq && (!reqs19 || !out3)))
        return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: bad argument");
    for (int r = 0; r < nreq; r++) {
        const int *q = reqs19 + (size_t)r * 19;
        if (q[0] < 0 || q[0] >= S) return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: shard index out of range");
        if (r && (q[0] < q[-19] || (q[0] == q[-19] && q[1] <= q[-18])))
            return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: requests not in (shard, rqseqno) order");
    }
    for (int i = 0; i < S * T; i++)
        if (nrec[i] < 0 || nrec[i] > k || navail[i] < nrec[i])
            return fail(ADLBQ_ERR_ARG, "adlbq_steal_merge: bad record counts");
    auto tindex = [&](int v) {
        for (int t = 0; t < T; t++)
            if (user_types[t] == v) return t;
        return -1;
    };
    std::vector<int> head((size_t)S * T, 0), unk_cnt(T, 0);
    std::vector<char> unk((size_t)S * T, 0);
    std::vector<HeadTree> tree(T);
    auto rec = [&](int s, int t, int i) { return recs8 + (((size_t)s * T + t) * k + i) * 8; };
    // a list past its exported records is LOWEST when the shard had no more, else unknown
    auto refresh = [&](int s, int t) {
        const size_t st = (size_t)s * T + t;
        const bool more = head[st] < nrec[st];
        const bool u = !more && navail[st] > nrec[st];
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
            else if (head[st] < nrec[st]) {
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

}  // extern "C"
