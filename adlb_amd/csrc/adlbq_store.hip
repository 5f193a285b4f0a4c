// adlbq_store.hip -- handle lifecycle, HBM unit store, Put / Get / Unreserve,
// qmstat row, info and donor-selection entry points of the C ABI (include/adlbq.h).
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>

#include "adlbq_donor.h"
#include "adlbq_impl.h"

using namespace adlbq;

static thread_local std::string g_err;

namespace adlbq {

int fail(int code, const char *msg) {
    g_err = msg;
    return code;
}

int hip_fail(hipError_t e, const char *where) {
    g_err = std::string(where) + ": " + hipGetErrorString(e);
    return ADLBQ_ERR_HIP;
}

template <typename T>
static int grow(T **p, long long old_n, long long new_n, hipStream_t s, int fill_byte = -1) {
    T *np = nullptr;
    AQ_HIP(hipMalloc((void **)&np, sizeof(T) * (size_t)new_n));
    if (*p && old_n > 0) AQ_HIP(hipMemcpyAsync(np, *p, sizeof(T) * (size_t)old_n, hipMemcpyDeviceToDevice, s));
    if (fill_byte >= 0 && new_n > old_n)
        AQ_HIP(hipMemsetAsync(np + old_n, fill_byte, sizeof(T) * (size_t)(new_n - old_n), s));
    if (*p) {
        AQ_HIP(hipStreamSynchronize(s));
        AQ_HIP(hipFree(*p));
    }
    *p = np;
    return ADLBQ_OK;
}

static int grow_pages(adlbq_server *h, int need) {
    if (need <= h->cap_pages) return ADLBQ_OK;
    int nc = std::max(need, h->cap_pages * 2);
    long long o = (long long)h->cap_pages * PAGE, n = (long long)nc * PAGE;
    int rc;
    if ((rc = grow(&h->d_prio, o, n, h->stream))) return rc;
    if ((rc = grow(&h->d_meta, o, n, h->stream, 0))) return rc;
    if ((rc = grow(&h->d_pin, o, n, h->stream, 0xff))) return rc;
    if ((rc = grow(&h->d_seq, o, n, h->stream))) return rc;
    if ((rc = grow(&h->d_cold0, o, n, h->stream))) return rc;
    if ((rc = grow(&h->d_cold1, o, n, h->stream))) return rc;
    if ((rc = grow(&h->d_rrec, 2 * o, 2 * n, h->stream))) return rc;
    h->cap_pages = nc;
    return ADLBQ_OK;
}

// Snapshot slot i has landed: k_finalize stores the slot's tag after writing
// the rest back (no event per batch: an event record stalls the queue for
// several microseconds behind the kernel before it).
static bool snap_landed(const adlbq_server *h, int i) {
    return h->snap_tag[i] != 0 && __atomic_load_n(&h->h_snap[i].snap_tag, __ATOMIC_ACQUIRE) == h->snap_tag[i];
}

// the newest reserve-batch snapshot that has landed in host memory, or -1; the
// tag checks run once per hint_stamp (one launch), older answers stay valid
static int newest_landed(adlbq_server *h) {
    if (h->landed_stamp == h->hint_stamp) return h->landed_idx;
    const int N = adlbq_server::NSNAP;
    int found = -1;
    for (int k = 1; k <= N && found < 0; k++) {
        const int i = (h->snap_next - k + N) % N;
        if (h->snap_at[i] && snap_landed(h, i)) found = i;
    }
    h->landed_idx = found;
    h->landed_stamp = h->hint_stamp;
    return found;
}

void tighten_rq_bound(adlbq_server *h, bool wait_oldest) {
    const int N = adlbq_server::NSNAP;
    if (wait_oldest) {  // backpressure: let the batches in flight land (every snapshot tag is then stored)
        hipStreamSynchronize(h->stream);
        h->hint_stamp++;
    }
    for (int k = 1; k <= N; k++) {
        const int i = (h->snap_next - k + N) % N;
        if (!h->snap_at[i]) continue;
        if (!snap_landed(h, i)) continue;
        const long long bound = (long long)h->h_snap[i].rq_n + (h->launched_reserves - h->snap_at[i]);
        if (bound < h->rq_n_upper) h->rq_n_upper = bound;
        return;
    }
}

// Wait (host spin on the mapped snapshot, no HIP call: the stream keeps its
// queued batches) until the oldest batch still in flight has landed its
// counter snapshot.  False when none is in flight, or after ~2 s (the caller
// then synchronises the stream).
static bool wait_oldest_snapshot(adlbq_server *h) {
    const int N = adlbq_server::NSNAP;
    for (int k = 0; k < N; k++) {
        const int i = (h->snap_next + k) % N;  // the ring from its oldest slot
        if (!h->snap_at[i] || h->snap_tag[i] == 0 || snap_landed(h, i)) continue;
        const auto t0 = std::chrono::steady_clock::now();
        while (!snap_landed(h, i)) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return false;
        }
        h->hint_stamp++;
        return true;
    }
    return false;
}

// Upper bound of the parked Reserves alive now, from the newest landed batch
// snapshot plus every Reserve launched after it (no synchronisation).
long long rq_live_upper(adlbq_server *h) {
    const int i = newest_landed(h);
    if (i < 0) return LLONG_MAX;  // nothing landed yet: assume a match is possible
    return (long long)h->h_snap[i].rq_live + (h->launched_reserves - h->snap_at[i]);
}

// Whether the newest landed reserve batch needed a multi-prio-bin sort.
bool rank_hint(adlbq_server *h) {  // the newest landed batch ranked its candidates in k_select_open
    const int i = newest_landed(h);
    return i >= 0 && h->h_snap[i].rank_fast != 0;
}

// the newest landed batch's candidate sort plan (G, lowest varying key bit), or false
bool plan_hint(adlbq_server *h, int *g, int *lo, int *phi) {
    const int i = newest_landed(h);
    if (i < 0) return false;
    *g = h->h_snap[i].plan_g;
    *lo = h->h_snap[i].plan_lo;
    if (phi) *phi = h->h_snap[i].plan_phi;
    return *g > 0;
}

// keyrank unless a landed batch failed it over lately (then 64 batches on the sort + k_rank path)
bool keyrank_hint(adlbq_server *h) {
    const int i = newest_landed(h);
    if (i >= 0 && h->h_snap[i].kr_fail > h->kr_fail_seen) {
        h->kr_fail_seen = h->h_snap[i].kr_fail;
        h->kr_skip_until = h->reserve_batches + 64;
    }
    return h->reserve_batches >= h->kr_skip_until;
}

bool sort_hint(adlbq_server *h) {
    const int i = newest_landed(h);
    // nothing landed yet (the first batches): sort whatever needs it through the
    // read-back path, never through k_rank's in-launch sort (milliseconds on long lists)
    return i < 0 || h->h_snap[i].needsort_last != 0;
}

constexpr long long RQ_GROW_MAX = 1ll << 24;  // rq entries a growth step reserves at most for batches in flight

// Stable in-place compaction of the live rq entries into slots [0, live), FIFO
// order kept (the reference frees each entry at rq_delete, xq.c:379; here the
// slots of dead entries are reclaimed in bulk before the rq would grow).
// Chunks of 1024 go in order and an entry only moves down; every entry of a
// chunk is read before any of the chunk is written, so nothing is overwritten
// before it is read.  rq_seq moves with its entry and stays ascending.
__global__ __launch_bounds__(1024) void k_rq_reclaim(int *rq_rank, int *rq_types, int *rq_live, int *rq_seq,
                                                     DevCounters *ctr) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int head = ctr->rq_head, n = ctr->rq_n;
    int base = 0;
    for (int c0 = head; c0 < n; c0 += 1024) {
        const int k = c0 + tid;
        const bool live = k < n && rq_live[k];
        int rk = 0, sq = 0;
        int4 ty[NREQ / 4];
        if (live) {
            rk = rq_rank[k];
            sq = rq_seq[k];
            const int4 *src = reinterpret_cast<const int4 *>(rq_types + (long long)k * NREQ);
#pragma unroll
            for (int q = 0; q < NREQ / 4; q++) ty[q] = src[q];
        }
        const unsigned long long b = __ballot(live);
        if (lane == 0) wsum[w] = __popcll(b);
        __syncthreads();  // also: the whole chunk has been read
        int pre = base, tot = 0;
        for (int q = 0; q < 16; q++) {
            pre += q < w ? wsum[q] : 0;
            tot += wsum[q];
        }
        if (live) {
            const int pos = pre + __popcll(b & lanemask_lt());
            rq_rank[pos] = rk;
            rq_seq[pos] = sq;
            rq_live[pos] = 1;
            int4 *dst = reinterpret_cast<int4 *>(rq_types + (long long)pos * NREQ);
#pragma unroll
            for (int q = 0; q < NREQ / 4; q++) dst[q] = ty[q];
        }
        base += tot;
        __syncthreads();
    }
    for (int k = base + tid; k < n; k += 1024) rq_live[k] = 0;
    if (tid == 0) {
        ctr->rq_n = base;
        ctr->rq_head = 0;
        ctr->rq_reclaims += 1;
    }
}

__global__ void k_set_rq_next(DevCounters *ctr, int v) { ctr->rq_next = v; }

// Parked Reserves come and go while the oldest stay: the live entries thin out
// over a long rq, and every Put batch's match stages the whole of it (from
// rq_head).  When the last landed counters show mostly dead slots, compact in
// the background (stream-ordered, nothing waits; the host's rq bounds stay
// upper bounds), at most once per RQ_COMPACT_EVERY calls, and before the rq fills (a
// full rq reclaims synchronously: config 3 did every fifth step).
constexpr int RQ_COMPACT_EVERY = 4;
void maybe_compact_rq(adlbq_server *h) {
    if (!h->d_rq_seq || h->rq_cap <= 0 || ++h->rq_compact_calls < RQ_COMPACT_EVERY) return;
    // the newest counters the host has: the synchronised copy, or -- while batches are in
    // flight (device-side entry points never synchronise) -- the newest landed batch snapshot
    const DevCounters *v = &h->ctr;
    if (h->ctr_stale) {
        const int i = newest_landed(h);
        if (i >= 0 && h->h_snap[i].rq_reclaims >= v->rq_reclaims) v = &h->h_snap[i];
    }
    // a compaction launched earlier that this view does not show yet: its effect is unknown, wait for it
    if (v->rq_reclaims < h->rq_reclaims_launched) return;
    const long long span = (long long)v->rq_n - v->rq_head;
    // mostly dead slots between head and tail, or the append index past half the slots: a steal round
    // deletes every Reserve it settles and the head follows, so the span stays short while rq_n still
    // climbs to the capacity check (which then reclaimed synchronously: config 3, every fifth step)
    const bool thin = span > 2ll * v->rq_live + 4096 || span * 2 > h->rq_cap;
    const bool high = 2ll * v->rq_n > h->rq_cap;
    if (!thin && !high) return;
    if (!high && span <= v->rq_live + 256) return;  // nothing much to reclaim
    h->rq_compact_calls = 0;
    h->rq_compactions++;
    h->rq_reclaims_launched++;
    k_rq_reclaim<<<1, 1024, 0, h->stream>>>(h->d_rq_rank, h->d_rq_types, h->d_rq_live, h->d_rq_seq, h->d_ctr);
}

int ensure_rq_capacity(adlbq_server *h, int extra) {
    if ((h->ctr_stale ? h->rq_next_upper : (long long)h->ctr.rq_next) + extra > INT_MAX) {
        int rc;
        if ((rc = refresh_counters(h))) return rc;
        if ((long long)h->ctr.rq_next + extra > INT_MAX)  // next_rqseqno is an int (adlb.c:1244)
            return fail(ADLBQ_ERR_NOMEM, "rq: rqseqnos would overflow an int");
    }
    long long need = (h->ctr_stale ? h->rq_n_upper : (long long)h->ctr.rq_n) + extra;
    if (need <= h->rq_cap) return ADLBQ_OK;
    if (h->ctr_stale) {
        // the bound is loose by the batches still in flight: use the newest
        // landed snapshot and, if that is not enough, wait for the oldest
        // tracked batch (the host then runs at most NSNAP batches ahead)
        tighten_rq_bound(h, false);
        need = h->rq_n_upper + extra;
        if (need <= h->rq_cap) return ADLBQ_OK;
        h->hacc["rq_waits"] += 1;
        {  // what the bound was made of (stats "hacc:rqw_*": the last wait)
            const int N = adlbq_server::NSNAP;
            int li = -1, nl = 0;
            for (int k = 1; k <= N; k++) {
                const int i = (h->snap_next - k + N) % N;
                if (!h->snap_at[i]) continue;
                if (snap_landed(h, i)) { if (li < 0) li = i; nl++; }
            }
            h->hacc["rqw_need"] = need;
            h->hacc["rqw_cap"] = h->rq_cap;
            h->hacc["rqw_landed"] = nl;
            h->hacc["rqw_snap_rq_n"] = li >= 0 ? h->h_snap[li].rq_n : -1;
            h->hacc["rqw_since"] = li >= 0 ? h->launched_reserves - h->snap_at[li] : -1;
            h->hacc["rqw_stale"] = h->ctr_stale ? 1 : 0;
        }
        // the oldest batches in flight first, one at a time (a stream synchronisation would
        // drain the queue and leave the GPU idle while the host issues the next batch)
        while (!h->rq_wait_sync && wait_oldest_snapshot(h)) {
            tighten_rq_bound(h, false);
            need = h->rq_n_upper + extra;
            if (need <= h->rq_cap) return ADLBQ_OK;
        }
        tighten_rq_bound(h, true);
        need = h->rq_n_upper + extra;
        if (need <= h->rq_cap) return ADLBQ_OK;
    }
    h->hacc["rq_reclaims"] += 1;
    if (h->rq_cap > 0 && h->d_rq_seq) {  // reclaim the slots of dead entries, then the exact count
        h->rq_reclaims_launched++;
        k_rq_reclaim<<<1, 1024, 0, h->stream>>>(h->d_rq_rank, h->d_rq_types, h->d_rq_live, h->d_rq_seq, h->d_ctr);
        AQ_HIP(hipGetLastError());
        int rc;
        if ((rc = refresh_counters(h))) return rc;  // synchronises
        need = (long long)h->ctr.rq_n + extra;
        // enough room left for the batches a host may run ahead: done; otherwise grow
        // now rather than wait and reclaim again at the next batches (config 3 did
        // both on half its shards every step)
        if (need + (long long)adlbq_server::NSNAP * extra <= h->rq_cap) return ADLBQ_OK;
    }
    // room for NSNAP batches of this size in flight at once (76 B per entry),
    // so that the wait above is the snapshot ring's, not a reallocation's
    long long nc = std::max<long long>(need, (long long)h->rq_cap * 2);
    nc = std::max<long long>(nc, std::min<long long>(need + (long long)(adlbq_server::NSNAP + 1) * extra, RQ_GROW_MAX));
    nc = std::max<long long>(nc, 1024);
    int rc;
    if ((rc = grow(&h->d_rq_rank, h->rq_cap, nc, h->stream))) return rc;
    if ((rc = grow(&h->d_rq_types, (long long)h->rq_cap * NREQ, nc * NREQ, h->stream))) return rc;
    if ((rc = grow(&h->d_rq_live, h->rq_cap, nc, h->stream, 0))) return rc;
    if ((rc = grow(&h->d_rq_req, h->rq_cap, nc, h->stream))) return rc;
    if ((rc = grow(&h->d_rq_seq, h->rq_cap, nc, h->stream))) return rc;
    h->rq_cap = (int)nc;
    return ADLBQ_OK;
}

static void apply_counters(adlbq_server *h);

// the counters into mapped host memory (one thread; visible once the stream is synchronised)
__global__ void k_ctr_out(const DevCounters *__restrict__ src, DevCounters *dst) { *dst = *src; }

// the counters land in mapped pinned memory (one-thread kernel): no staged copy
static int ensure_zctr(adlbq_server *h) {
    if (!h->h_zctr) {
        AQ_HIP(hipHostMalloc((void **)&h->h_zctr, sizeof(DevCounters), hipHostMallocMapped));
        AQ_HIP(hipHostGetDevicePointer((void **)&h->d_zctr, h->h_zctr, 0));
    }
    return ADLBQ_OK;
}

// mapped pinned staging of at least n ints for a synchronous entry point
int ensure_zc(adlbq_server *h, long long n) {
    if (n > h->cap_zc) {
        AQ_HIP(hipStreamSynchronize(h->stream));
        if (h->h_zc) AQ_HIP(hipHostFree(h->h_zc));
        h->cap_zc = std::max<long long>({n, 2 * h->cap_zc, 4096});
        AQ_HIP(hipHostMalloc((void **)&h->h_zc, sizeof(int) * h->cap_zc, hipHostMallocMapped));
        AQ_HIP(hipHostGetDevicePointer((void **)&h->d_zc, h->h_zc, 0));
    }
    return ADLBQ_OK;
}

int refresh_counters(adlbq_server *h) {
    int rc;
    if ((rc = ensure_zctr(h))) return rc;
    k_ctr_out<<<1, 1, 0, h->stream>>>(h->d_ctr, h->d_zctr);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipStreamSynchronize(h->stream));
    h->ctr = *h->h_zctr;
    apply_counters(h);
    return ADLBQ_OK;
}

static void apply_counters(adlbq_server *h);

// After a synchronous reserve batch: the counters its k_finalize copied into
// the newest snapshot slot (mapped memory, tagged last), no k_ctr_out launch.
// Spin (host, mapped memory) until the last launched batch's snapshot tag lands, then take its
// counters as sync_batch_counters does; false after ~2 s (the caller synchronises instead).
bool wait_last_snapshot(adlbq_server *h) {
    const int slot = (h->snap_next + adlbq_server::NSNAP - 1) % adlbq_server::NSNAP;
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(&h->h_snap[slot].snap_tag, __ATOMIC_ACQUIRE) != h->snap_tag[slot])
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return false;
    h->ctr = h->h_snap[slot];
    apply_counters(h);
    h->hint_stamp++;
    return true;
}

int sync_batch_counters(adlbq_server *h) {
    const int slot = (h->snap_next + adlbq_server::NSNAP - 1) % adlbq_server::NSNAP;
    AQ_HIP(hipStreamSynchronize(h->stream));
    if (__atomic_load_n(&h->h_snap[slot].snap_tag, __ATOMIC_ACQUIRE) != h->snap_tag[slot])
        return refresh_counters(h);
    h->ctr = h->h_snap[slot];
    apply_counters(h);
    return ADLBQ_OK;
}

// the host's view after h->ctr has been refreshed
static void apply_counters(adlbq_server *h) {
    h->ctr_stale = false;
    h->rq_n_upper = h->ctr.rq_n;
    h->rq_next_upper = h->ctr.rq_next;
    // units the device-side Get batches removed since the last look
    h->live_units -= h->ctr.got - h->got_seen;
    h->live_targeted -= h->ctr.got_targeted - h->got_t_seen;
    h->got_seen = h->ctr.got;
    h->got_t_seen = h->ctr.got_targeted;
}

template <typename T>
static int upload(T **dptr, int *cap, const std::vector<T> &v, hipStream_t s) {
    if ((int)v.size() > *cap) {
        if (*dptr) {
            AQ_HIP(hipStreamSynchronize(s));
            AQ_HIP(hipFree(*dptr));
        }
        int nc = std::max<int>((int)v.size(), 2 * *cap);
        nc = std::max(nc, 64);
        AQ_HIP(hipMalloc((void **)dptr, sizeof(T) * nc));
        *cap = nc;
    }
    if (!v.empty()) AQ_HIP(hipMemcpyAsync(*dptr, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, s));
    return ADLBQ_OK;
}

// ---------------------------------------------------------------- dead open pages
// Pages are append-only: a long-running server's open bucket keeps every page a
// Put ever filled, and each scan and table upload pays for the dead ones.  A
// full page (never the tail) with no LIVE unit stays dead -- units become LIVE
// only by a Put into the tail page -- so it can leave the bucket (the others
// keep their relative order, which is the bucket order) and be reused by
// later Puts.  k_page_dead flags them, one workgroup per page, into mapped
// host memory; the flags are applied by a later reserve call once the kernel's
// event has passed, never waited for.
__global__ __launch_bounds__(256) void k_page_dead(const int *__restrict__ pages, int n,
                                                   const uint32_t *__restrict__ meta, int *flags) {
    __shared__ int live;
    const int p = blockIdx.x;
    if (threadIdx.x == 0) live = 0;
    __syncthreads();
    const uint4 *M4 = reinterpret_cast<const uint4 *>(meta + ((long long)pages[p] << PAGE_SHIFT));
    uint32_t o = 0u;
    for (int i = threadIdx.x; i < PAGE / 4; i += 256) {
        const uint4 v = M4[i];
        o |= v.x | v.y | v.z | v.w;
    }
    if (o & M_LIVE) live = 1;  // every writer stores 1
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + p, live ? 0 : 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void recycle_apply(adlbq_server *h) {
    if (!h->pdead_pending || hipEventQuery(h->pdead_ev) != hipSuccess) return;
    h->pdead_pending = false;
    std::vector<int> &op = h->open.pages;
    const int n = std::min<int>(h->pdead_np, (int)op.size() - 1);  // pages that were full when flagged
    int w = 0, dropped = 0;
    for (int i = 0; i < (int)op.size(); i++) {
        if (i < n && __atomic_load_n(h->h_pdead + i, __ATOMIC_ACQUIRE) == 1) {
            h->free_pages.push_back(op[(size_t)i]);
            dropped++;
            continue;
        }
        op[(size_t)w++] = op[(size_t)i];
    }
    op.resize((size_t)w);
    if (dropped) {
        h->tables_dirty = true;
        h->batch_export_k = 0;  // the last batch's candidate lists hold bucket positions of the old list
        h->pages_recycled += dropped;
    }
}

int recycle_launch(adlbq_server *h) {
    const int np = (int)h->open.pages.size();
    if (!h->recycle_pages || h->pdead_pending || np < 4 || h->reserve_batches - h->pdead_last < 16) return ADLBQ_OK;
    const long long live_open = h->live_units - h->live_targeted;  // an upper bound (Gets land later)
    if (live_open * 2 >= (long long)(np - 1) * PAGE) return ADLBQ_OK;  // mostly live: nothing to drop
    if (np - 1 > h->cap_pdead) {
        if (h->h_pdead) AQ_HIP(hipHostFree(h->h_pdead));
        h->cap_pdead = std::max<long long>(np, 2 * h->cap_pdead);
        AQ_HIP(hipHostMalloc((void **)&h->h_pdead, sizeof(int) * h->cap_pdead, hipHostMallocDefault));
    }
    if (!h->pdead_ev) AQ_HIP(hipEventCreateWithFlags(&h->pdead_ev, hipEventDisableTiming));
    int *dflags = nullptr;
    AQ_HIP(hipHostGetDevicePointer((void **)&dflags, h->h_pdead, 0));
    k_page_dead<<<np - 1, 256, 0, h->stream>>>(h->d_open_pages, np - 1, h->d_meta, dflags);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipEventRecord(h->pdead_ev, h->stream));
    h->pdead_pending = true;
    h->pdead_np = np - 1;
    h->pdead_last = h->reserve_batches;
    return ADLBQ_OK;
}

int sync_tables(adlbq_server *h) {
    if (h->tables_dirty || h->pinfo_dirty) {
        // every page table in one pinned staging buffer and one copy: the open pages,
        // the rank buckets' pages (CSR) with their fills, bucket ranks, rank -> bucket,
        // every page with its fill (whole-store scans), per-page offset base and wide flag
        const std::vector<int> &op = h->open.pages;
        const size_t nb = h->bucket_ranks.size(), A = (size_t)std::max(h->A, 1), npg = h->page_base.size();
        size_t nrp = 0;
        for (size_t k = 0; k < nb; k++) nrp += h->rankb[k].pages.size();
        const size_t nall = op.size() + nrp;
        auto al = [](size_t n) { return (n + 15) & ~(size_t)15; };  // 64-B aligned sections
        const size_t o_open = 0, o_rp = o_open + al(op.size()), o_ps = o_rp + al(nrp), o_fill = o_ps + al(nb + 1),
                     o_br = o_fill + al(nb), o_r2b = o_br + al(nb), o_ap = o_r2b + al(A), o_af = o_ap + al(nall),
                     o_pb = o_af + al(nall), o_pw = o_pb + al(npg), total = o_pw + al(npg);
        const int sl = h->tab_slot;
        h->tab_slot ^= 1;
        const auto w0 = std::chrono::steady_clock::now();
        if (h->tab_ev[sl]) AQ_HIP(hipEventSynchronize(h->tab_ev[sl]));  // its last copy has left the buffer
        else AQ_HIP(hipEventCreateWithFlags(&h->tab_ev[sl], hipEventDisableTiming));
        h->hacc["tables_wait"] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
        if ((long long)total > h->cap_htab[sl]) {
            if (h->h_tab[sl]) AQ_HIP(hipHostFree(h->h_tab[sl]));
            h->cap_htab[sl] = std::max<long long>({(long long)total * 2, 2 * h->cap_htab[sl], 1ll << 16});
            AQ_HIP(hipHostMalloc((void **)&h->h_tab[sl], sizeof(int) * h->cap_htab[sl], hipHostMallocDefault));
        }
        if ((long long)total > h->cap_dtab) {
            AQ_HIP(hipStreamSynchronize(h->stream));  // kernels in flight read the old tables
            if (h->d_tab) AQ_HIP(hipFree(h->d_tab));
            h->cap_dtab = std::max((long long)total, 2 * h->cap_dtab);
            AQ_HIP(hipMalloc((void **)&h->d_tab, sizeof(int) * h->cap_dtab));
        }
        int *t = h->h_tab[sl];
        if (!op.empty()) std::memcpy(t + o_open, op.data(), sizeof(int) * op.size());
        size_t r = 0, q = 0;
        t[o_ps] = 0;
        for (size_t k = 0; k < nb; k++) {
            const Bucket &bk = h->rankb[k];
            if (!bk.pages.empty()) std::memcpy(t + o_rp + r, bk.pages.data(), sizeof(int) * bk.pages.size());
            r += bk.pages.size();
            t[o_ps + k + 1] = (int)r;
            t[o_fill + k] = bk.pages.empty() ? 0 : bk.tail_fill;
            t[o_br + k] = h->bucket_ranks[k];
        }
        for (size_t i = 0; i < A; i++) t[o_r2b + i] = -1;
        for (size_t k = 0; k < nb; k++)
            if (h->bucket_ranks[k] >= 0 && h->bucket_ranks[k] < h->A) t[o_r2b + h->bucket_ranks[k]] = (int)k;
        for (size_t i = 0; i < op.size(); i++, q++) {
            t[o_ap + q] = op[i];
            t[o_af + q] = i + 1 == op.size() ? h->open.tail_fill : PAGE;
        }
        for (size_t k = 0; k < nb; k++) {
            const Bucket &bk = h->rankb[k];
            for (size_t i = 0; i < bk.pages.size(); i++, q++) {
                t[o_ap + q] = bk.pages[i];
                t[o_af + q] = i + 1 == bk.pages.size() ? bk.tail_fill : PAGE;
            }
        }
        if (npg) {
            std::memcpy(t + o_pb, h->page_base.data(), sizeof(int) * npg);
            std::memcpy(t + o_pw, h->page_wide.data(), sizeof(int) * npg);
        }
        bool narrow = true;  // pass 1 skips the per-page wide flag when no open page is wide
        for (size_t i = 0; i < op.size() && narrow; i++) narrow = h->page_wide[(size_t)op[i]] == 0;
        h->open_all_narrow = narrow;
        AQ_HIP(hipMemcpyAsync(h->d_tab, t, sizeof(int) * total, hipMemcpyHostToDevice, h->stream));
        AQ_HIP(hipEventRecord(h->tab_ev[sl], h->stream));
        int *d = h->d_tab;
        h->d_open_pages = d + o_open;
        h->d_rank_pages = d + o_rp;
        h->d_rank_pstart = d + o_ps;
        h->d_rank_fill = d + o_fill;
        h->d_bucket_ranks = d + o_br;
        h->d_rank2b = d + o_r2b;
        h->d_all_pages = d + o_ap;
        h->d_all_fill = d + o_af;
        h->d_pbase = d + o_pb;
        h->d_pwide = d + o_pw;
        h->tables_dirty = false;
        h->pinfo_dirty = false;
    }
    int rc;
    if (h->qm_dirty) {
        if (h->S * h->T > 0)
            AQ_HIP(hipMemcpyAsync(h->d_qm_hi, h->qm_hi.data(), sizeof(int) * h->S * h->T,
                                  hipMemcpyHostToDevice, h->stream));
        AQ_HIP(hipMemcpyAsync(h->d_qm_qlen, h->qm_qlen.data(), sizeof(int) * h->S,
                              hipMemcpyHostToDevice, h->stream));
        h->qm_dirty = false;
    }
    if (h->tq_dirty) {
        if ((rc = upload(&h->d_tq, &h->cap_tq, h->tq, h->stream))) return rc;
        h->tq_dirty = false;
    }
    return ADLBQ_OK;
}

DonorCtx donor_ctx(adlbq_server *h) {
    DonorCtx c;
    c.qm_hi = h->d_qm_hi;
    c.qm_qlen = h->d_qm_qlen;
    c.tq = h->d_tq;
    c.utypes = h->d_utypes;
    c.rfr_out = h->d_rfr_out;
    c.rfr_to_rank = h->d_rfr_to_rank;
    c.S = h->S;
    c.T = h->T;
    c.n_tq = (int)(h->tq.size() / 4);
    c.master = h->master;
    c.my_world = h->my_world;
    c.A = h->A;
    c.num_world = h->num_world;
    return c;
}

static hipEvent_t pooled_event(adlbq_server *h) {
    hipEvent_t e = nullptr;
    if (!h->event_pool.empty()) {
        e = h->event_pool.back();
        h->event_pool.pop_back();
    } else {
        hipEventCreate(&e);
    }
    return e;
}

static bool stage_on(adlbq_server *h, const char *name) {
    // "profile_every" n: only every n-th reserve batch carries stage events (an
    // event record stalls the queue for microseconds behind the kernel before it)
    return h->profiling && (h->profile_only.empty() || h->profile_only == name) &&
           (h->profile_every <= 1 || h->reserve_batches % h->profile_every == 0);
}

void stage_begin(adlbq_server *h, const char *name, hipEvent_t *ev) {
    *ev = nullptr;
    if (!stage_on(h, name)) return;
    *ev = pooled_event(h);
    hipEventRecord(*ev, h->stream);
    h->stage_host_t0 = std::chrono::steady_clock::now();
}

void stage_end(adlbq_server *h, const char *name, hipEvent_t ev) {
    if (!ev) return;
    hipEvent_t e2 = pooled_event(h);
    hipEventRecord(e2, h->stream);
    auto &t = h->timers[name];
    t.pending.push_back({ev, e2});
    t.host_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                      h->stage_host_t0).count();
}

void host_stage_add(adlbq_server *h, const char *name, std::chrono::steady_clock::time_point t0) {
    if (!stage_on(h, name)) return;
    h->timers[name].host_ns +=
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace adlbq

// ============================================================================ kernels

struct PutRec {  // staged by the host per Put
    int slot, prio, meta, seq;
    int answer, len, home, clen;
    int csrv, cseq, utype, target;
};

__global__ void k_put_scatter(const PutRec *__restrict__ r, int n, int *prio, uint32_t *meta, int *pin,
                              int *seq, int4 *cold0, int4 *cold1, long long *seq2slot, long long *anchor,
                              int4 *rrec, DevCounters *ctr, long long add_bytes) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0 && add_bytes) bytes_add(ctr, add_bytes);  // the batch's puts, when no rq match interleaves
    const bool ok = i < n;
    PutRec u = r[ok ? i : 0];
    raise_anchor(anchor, ok ? (u.meta & M_TYPE) : 0, ok ? u.prio : INT_MIN);  // upper bounds of live prios
    if (!ok) return;
    prio[u.slot] = u.prio;
    meta[u.slot] = (uint32_t)u.meta;
    pin[u.slot] = -1;
    seq[u.slot] = u.seq;
    cold0[u.slot] = make_int4(u.answer, u.len, u.home, u.clen);
    cold1[u.slot] = make_int4(u.csrv, u.cseq, u.utype, u.target);
    rrec[2ll * u.slot] = make_int4(u.answer, u.len, u.seq, u.clen);
    rrec[2ll * u.slot + 1] = make_int4(u.csrv, u.cseq, u.utype, u.prio);
    seq2slot[u.seq] = u.slot;
}

// Put-side FIFO match, one wavefront, Puts strictly in order
// (rq_find_rank_queued_for_type, xq.c:388-405, at adlb.c:988-1042)
__global__ void k_put_match(const PutRec *__restrict__ r, int n, const int *__restrict__ rq_rank,
                            const int *__restrict__ rq_types, int *rq_live, const int *__restrict__ rq_seq,
                            DevCounters *ctr, uint32_t *meta, int *pin, int *out3, const int *gate) {
    if (gate && *gate == 0) return;  // k_put_match_blk handled the batch
    const int lane = threadIdx.x;
    int head = ctr->rq_head, nrq = ctr->rq_n, live = ctr->rq_live;
    for (int i = 0; i < n; i++) {
        PutRec u = r[i];
        if (lane == 0) bytes_add(ctr, BYTES_WQ + u.len);  // pmalloc + wq_node_create (adlb.c:933, 963)
        int found = -1;
        if (live > 0) {
            for (int base = head; base < nrq; base += 64) {
                int k = base + lane;
                bool hit = false;
                if (k < nrq && ld_agent(rq_live + k)) {
                    int rk = rq_rank[k];
                    if (u.target == -1 || u.target == rk) {
                        const int *tv = rq_types + (long long)k * NREQ;
#pragma unroll
                        for (int q = 0; q < NREQ; q++) {
                            int t = tv[q];
                            hit |= (u.utype == -1 || t == -1 || t == u.utype);
                        }
                    }
                }
                unsigned long long b = __ballot(hit);
                if (b) { found = base + __ffsll((long long)b) - 1; break; }
            }
        }
        if (lane == 0) {
            int *o = out3 + 3 * i;
            int o1 = -1, o2 = -1;
            if (found >= 0) {
                int rk = rq_rank[found];
                st_agent(rq_live + found, 0);
                o1 = rk;
                o2 = rq_seq[found];
                bytes_add(ctr, -BYTES_RQ);  // rq_delete (adlb.c:1040)
                pin[u.slot] = rk;
                if (rk >= 0) meta[u.slot] = (uint32_t)u.meta | M_PINNED;
            }
            o[0] = u.seq;  // every result word written once
            o[1] = o1;
            o[2] = o2;
        }
        if (found >= 0) {
            live--;
            if (found == head)
                while (head < nrq && !ld_agent(rq_live + head)) head++;
        }
        __builtin_amdgcn_s_waitcnt(0);
    }
    if (lane == 0) {
        ctr->rq_live = live;
        ctr->rq_head = head;
    }
}

// The same FIFO first-fit for a batch of Puts, one workgroup of 1024: the live
// rq entries (up to PM_CAP) are staged in LDS once as (rank, type-index mask);
// the Puts go in chunks of PM_CAP, PM_PER consecutive ones per thread.  A Put
// may take an entry when rank == target (targeted) and its type is in the
// entry's set or a -1 is anywhere in it (rq_find_rank_queued_for_type,
// xq.c:388-405).  Puts in order each taking the first such entry still free
// is a serial dictatorship with one preference order on each side (Puts rank
// entries by FIFO position, entries rank Puts by arrival), whose stable
// matching is unique: the entries in FIFO order each taking the first
// compatible Put still free give the same pairs.  So each chunk loops over
// whichever side is shorter, one block-wide minimum per step, and stops when
// no live entry is left (no step at all when nothing is parked).  Byte
// accounting keeps the sequential high-water mark: the peak is the largest
// running sum just after a Put's allocation (adlb.c:933, 963, 1040).  *over = 1
// when the live entries exceed PM_CAP (the caller then runs k_put_match).
constexpr int PM_CAP = 4096, PM_THREADS = 1024, PM_PER = PM_CAP / PM_THREADS, PM_WAVES = PM_THREADS / 64;
constexpr int PM_REG = 4;  // entries per lane of the register-resident match (<= 256 parked)
__global__ __launch_bounds__(PM_THREADS) void k_put_match_blk(const PutRec *__restrict__ r, int n,
                                                              const int *__restrict__ rq_rank,
                                                              const int *__restrict__ rq_types, int *rq_live,
                                                              const int *__restrict__ rq_seq,
                                                              DevCounters *ctr, uint32_t *meta, int *pin, int *out3,
                                                              const int *__restrict__ utypes, int T, int *over) {
    __shared__ int s_rank[PM_CAP], s_k[PM_CAP], s_res[PM_CAP];
    __shared__ int s_ml, s_rbig;
    // ranks with a parked entry (ranks below PM_RBITS; s_rbig: a larger one is parked): a targeted Put
    // whose rank has none skips the scan
    constexpr int PM_RBITS = 1 << 16;
    __shared__ unsigned int s_rbits[PM_RBITS / 32];
    __shared__ unsigned long long s_mask[PM_CAP];
    __shared__ int s_cnt[PM_WAVES], s_tot;
    __shared__ long long s_wsum[PM_WAVES], s_wpk[PM_WAVES];
    __shared__ int s_ut[ADLBQ_MAX_TYPES];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const int head = ctr->rq_head, nrq = ctr->rq_n;
    for (int t = tid; t < T; t += PM_THREADS) s_ut[t] = utypes[t];
    for (int q = tid; q < PM_RBITS / 32; q += PM_THREADS) s_rbits[q] = 0u;
    if (tid == 0) s_tot = 0, s_rbig = 0;
    __syncthreads();
    // T <= 8: the user types in registers, a type equal to an earlier one never matching (get_type_idx
    // returns the first declared match): a slot's lookup is eight compares instead of a walk over LDS
    int ur[8];
    bool uok[8];
#pragma unroll
    for (int t = 0; t < 8; t++) ur[t] = s_ut[t < T ? t : 0];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        uok[t] = t < T;
#pragma unroll
        for (int t2 = 0; t2 < t; t2++) uok[t] = uok[t] && ur[t2] != ur[t];
    }
    // stage the live entries in FIFO order (compaction in chunks of 1024)
    for (int c0 = head; c0 < nrq; c0 += PM_THREADS) {
        const int k = c0 + tid;
        const bool live = k < nrq && ld_agent(rq_live + k);
        const unsigned long long b = __ballot(live);
        if (lane == 0) s_cnt[w] = __popcll(b);
        __syncthreads();
        int pre = s_tot;
        for (int q = 0; q < w; q++) pre += s_cnt[q];
        const int pos = pre + __popcll(b & lanemask_lt());
        if (live && pos < PM_CAP) {
            // the entry's 16 types in four vector loads, all in flight before the lookups (a load per
            // type inside the lookup loop waited for each in turn)
            const int4 *tv4 = reinterpret_cast<const int4 *>(rq_types + (long long)k * NREQ);
            int tv[NREQ];
#pragma unroll
            for (int q = 0; q < NREQ / 4; q++) {
                const int4 x = tv4[q];
                tv[4 * q] = x.x, tv[4 * q + 1] = x.y, tv[4 * q + 2] = x.z, tv[4 * q + 3] = x.w;
            }
            unsigned long long m = 0;
            bool wild = false;
            if (T <= 8) {
#pragma unroll
                for (int q = 0; q < NREQ; q++) {
                    const int v = tv[q];
                    wild |= v == -1;
#pragma unroll
                    for (int t = 0; t < 8; t++) m |= (uok[t] && v == ur[t]) ? (1ull << t) : 0ull;
                }
            } else {
#pragma unroll
                for (int q = 0; q < NREQ; q++) {
                    const int v = tv[q];
                    wild |= v == -1;
                    for (int t = 0; t < T; t++)
                        if (s_ut[t] == v) {  // get_type_idx: first declared match
                            m |= 1ull << t;
                            break;
                        }
                }
            }
            const int rk = rq_rank[k];
            s_rank[pos] = rk;
            s_mask[pos] = wild ? ~0ull : m;
            s_k[pos] = k;
            if (rk >= 0 && rk < PM_RBITS) atomicOr(&s_rbits[rk >> 5], 1u << (rk & 31));
            else s_rbig = 1;
        }
        __syncthreads();
        if (tid == 0) {
            int tot = s_tot;
            for (int q = 0; q < PM_WAVES; q++) tot += s_cnt[q];
            s_tot = tot;
        }
        __syncthreads();
    }
    const int m = s_tot;
    const unsigned long long t_staged = __builtin_amdgcn_s_memrealtime();
    if (m > PM_CAP) {  // too many parked Reserves for the staging: the caller falls back
        if (tid == 0) *over = 1;
        return;
    }
    auto s_mlive_sync = [&](int v, int wv) {  // wave 0's count of live entries, to every thread
        if (wv == 0 && lane == 0) s_ml = v;
        __syncthreads();
        const int x = s_ml;
        __syncthreads();
        return x;
    };
    int mlive = m, nmatch = 0;
    long long run = 0, peak = LLONG_MIN;  // running byte delta before the chunk; peak over the batch
    for (int c0 = 0; c0 < n; c0 += PM_CAP) {
        const int nc = min(PM_CAP, n - c0);
        PutRec u[PM_PER];
        int res[PM_PER];
        unsigned long long bit[PM_PER];
#pragma unroll
        for (int q = 0; q < PM_PER; q++) {
            const int i = tid * PM_PER + q;
            res[q] = -1;
            if (i < nc) u[q] = r[c0 + i];
            bit[q] = i < nc ? 1ull << (u[q].meta & (int)M_TYPE) : 0ull;
        }
        if (mlive > 0) {
            // One wave takes the Puts in order (adlb.c:1020-1040 per Put): each takes the first free
            // compatible entry in FIFO order, found 64 entries per step (s_rank[e] == INT_MIN: taken).
            // Lane t keeps a lower bound for type t: the entries before it holding type t are all
            // taken, so an untargeted Put of type t starts there and moves it past its match.
            if (w == 0 && m <= PM_REG * 64) {
                // at most 256 entries: lane l holds entries l, l + 64, ... in registers and a bit per
                // entry still free; a Put is PM_REG ballots without a branch (the short-circuit test
                // and the early exit per ballot had made each Put a chain of exec-mask branches)
                int erk[PM_REG];
                unsigned long long emk[PM_REG];
                unsigned int fr = 0u;  // bit q: entry q * 64 + lane exists and is free
#pragma unroll
                for (int q = 0; q < PM_REG; q++) {
                    const int e = q * 64 + lane;
                    erk[q] = e < m ? s_rank[e] : INT_MIN;
                    emk[q] = e < m ? s_mask[e] : 0ull;
                    fr |= (e < m && erk[q] != INT_MIN ? 1u : 0u) << q;  // INT_MIN: taken by an earlier chunk
                }
                int pty = 0, ptg = -1, res_l = -1;  // lane l: Put i0 + l's type, target, result
                int i = 0;
                for (; i < nc && mlive > 0; i++) {
                    if ((i & 63) == 0) {  // unconditional loads (clamped), masked after
                        const int il = i + lane, ilc = il < nc ? il : nc - 1;
                        const int mt = r[c0 + ilc].meta, tt = r[c0 + ilc].target;
                        unsigned int in = il < nc ? 1u : 0u;
                        asm volatile("" : "+v"(in));
                        pty = in ? (mt & (int)M_TYPE) : 0;
                        ptg = in ? tt : -1;
                        res_l = -1;
                    }
                    const int t = __builtin_amdgcn_readlane(pty, i & 63);
                    const int tg = __builtin_amdgcn_readlane(ptg, i & 63);
                    unsigned int cand = 0u;
#pragma unroll
                    for (int q = 0; q < PM_REG; q++)
                        cand |= ((unsigned int)(emk[q] >> t) & (unsigned int)((tg == -1) | (tg == erk[q]))) << q;
                    cand &= fr;
                    int found = -1;
#pragma unroll
                    for (int q = PM_REG - 1; q >= 0; q--) {  // the first entry in FIFO order: lowest q, then lane
                        const unsigned long long hb = __ballot((cand >> q) & 1u);
                        found = hb ? q * 64 + __ffsll((long long)hb) - 1 : found;
                    }
                    fr &= ~((found >= 0 && lane == (found & 63)) ? (1u << (found >> 6)) : 0u);
                    mlive -= found >= 0 ? 1 : 0;
                    if ((i & 63) == lane) res_l = found;
                    if ((i & 63) == 63 || i == nc - 1 || mlive == 0) {  // this block of 64 Puts' results
                        const int il = (i & ~63) + lane;
                        if (il <= i) s_res[il] = res_l;
                    }
                }
                for (int il = i + lane; il < nc; il += 64) s_res[il] = -1;  // every entry taken
#pragma unroll
                for (int q = 0; q < PM_REG; q++) {  // the taken entries, for the later chunks
                    const int e = q * 64 + lane;
                    if (e < m && !((fr >> q) & 1u)) s_rank[e] = INT_MIN;
                }
            } else if (w == 0) {
                int tptr = 0;
                int pty = 0, ptg = -1;  // lane l: Put c0 + i0 + l's type and target (64 Puts per load)
                for (int i = 0; i < nc; i++) {
                    if ((i & 63) == 0) {  // unconditional loads (clamped), masked after
                        const int il = i + lane, ilc = il < nc ? il : nc - 1;
                        const int mt = r[c0 + ilc].meta, tt = r[c0 + ilc].target;
                        unsigned int in = il < nc ? 1u : 0u;
                        asm volatile("" : "+v"(in));
                        pty = in ? (mt & (int)M_TYPE) : 0;
                        ptg = in ? tt : -1;
                    }
                    int found = -1;
                    if (mlive > 0) {
                        const int t = __builtin_amdgcn_readlane(pty, i & 63);
                        const int tg = __builtin_amdgcn_readlane(ptg, i & 63);
                        const unsigned long long pb = 1ull << t;
                        const int e0 = __builtin_amdgcn_readlane(tptr, t);
                        // a targeted Put whose rank has no parked entry: no scan
                        const bool none = tg >= 0 && !s_rbig && (tg >= PM_RBITS || !((s_rbits[tg >> 5] >> (tg & 31)) & 1u));
                        for (int base = none ? m : e0; base < m; base += 64) {
                            // both LDS reads unconditional (a clamped entry) and the test without
                            // short-circuits: no exec-mask branch inside the step
                            const int e = base + lane, ec = e < m ? e : m - 1;
                            const int rk = s_rank[ec];
                            const unsigned long long mk = s_mask[ec];
                            const bool hit = (e < m) & (rk != INT_MIN) & ((mk & pb) != 0ull) & ((tg == -1) | (tg == rk));
                            const unsigned long long hb = __ballot(hit);
                            if (hb) {
                                found = base + __ffsll((long long)hb) - 1;
                                break;
                            }
                        }
                        if (found >= 0) {
                            if (lane == 0) s_rank[found] = INT_MIN;
                            mlive--;
                        }
                        if (tg == -1 && lane == t) tptr = found >= 0 ? found + 1 : m;
                        __builtin_amdgcn_wave_barrier();  // one wave's LDS operations stay in order
                    }
                    if (lane == 0) s_res[i] = found;
                }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < PM_PER; q++) {
                const int i = tid * PM_PER + q;
                if (i < nc) res[q] = s_res[i];
            }
            mlive = s_mlive_sync(mlive, w);
            if (tid == 0 && c0 == 0) {  // diagnostic sums (first chunk)
                atomicAdd((unsigned long long *)&ctr->diag[5], (unsigned long long)m);
                atomicAdd((unsigned long long *)&ctr->diag[6], t_staged - t_start);
                atomicAdd((unsigned long long *)&ctr->diag[7], __builtin_amdgcn_s_memrealtime() - t_staged);
            }
        }
        // results, pins, and the byte deltas of this thread's Puts in order
        long long acc = 0, pk = LLONG_MIN;
#pragma unroll
        for (int q = 0; q < PM_PER; q++) {
            const int i = tid * PM_PER + q;
            if (i >= nc) break;
            int *o = out3 + 3ll * (c0 + i);
            const long long wb = BYTES_WQ + u[q].len;  // pmalloc + wq_node_create
            pk = max(pk, acc + wb);
            acc += wb;
            const int e = res[q];
            int o1 = -1, o2 = -1;
            if (e >= 0) {
                const int k = s_k[e], rk = rq_rank[k];
                rq_live[k] = 0;
                o1 = rk;
                o2 = rq_seq[k];
                pin[u[q].slot] = rk;
                if (rk >= 0) meta[u[q].slot] = (uint32_t)u[q].meta | M_PINNED;
                acc -= BYTES_RQ;  // rq_delete (adlb.c:1040)
                nmatch++;
            }
            // every result word written once (a reader of mapped memory may poll them)
            o[0] = u[q].seq;
            o[1] = o1;
            o[2] = o2;
        }
        // block exclusive scan of acc in Put order, the peak, the chunk total
        long long x = acc;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const long long y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        long long px = pk == LLONG_MIN ? LLONG_MIN : pk + (x - acc);  // peak within the wave's prefix
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) px = max(px, __shfl_xor(px, o, 64));
        if (lane == 63) s_wsum[w] = x;
        if (lane == 0) s_wpk[w] = px;
        __syncthreads();
        long long wpre = 0, tot = 0, cpk = LLONG_MIN;
        for (int q = 0; q < PM_WAVES; q++) {
            if (s_wpk[q] != LLONG_MIN) cpk = max(cpk, tot + s_wpk[q]);
            tot += s_wsum[q];
        }
        (void)wpre;
        if (cpk != LLONG_MIN) peak = max(peak, run + cpk);
        run += tot;
        __syncthreads();
    }
    // matches of every thread
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nmatch += __shfl_xor(nmatch, o, 64);
    if (lane == 0) s_cnt[w] = nmatch;
    __syncthreads();
    if (tid == 0) {
        int tm = 0;
        for (int q = 0; q < PM_WAVES; q++) tm += s_cnt[q];
        const long long b0 = ctr->bytes;
        if (peak != LLONG_MIN && b0 + peak > ctr->bytes_hwm) ctr->bytes_hwm = b0 + peak;
        ctr->bytes = b0 + run;
        ctr->rq_live -= tm;
        // new FIFO head: the first staged entry still live (entries before the first staged one are dead)
        int nh = nrq;
        for (int j = 0; j < m; j++)
            if (s_rank[j] != INT_MIN) {
                nh = s_k[j];
                break;
            }
        ctr->rq_head = m ? nh : head;
    }
}

// the results of a Put batch that cannot match a parked Reserve: {wqseqno, -1, -1}
__global__ void k_put_out(const PutRec *__restrict__ r, int n, int *out3) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        out3[3 * i] = r[i].seq;
        out3[3 * i + 1] = -1;
        out3[3 * i + 2] = -1;
    }
}

__global__ void k_get(int slot, int rank, int seq, const int *prio, uint32_t *meta, const int *pin,
                      const int *seqa, const int4 *cold0, const int4 *cold1, int *res, DevCounters *ctr) {
    uint32_t m = meta[slot];
    res[0] = -1;
    res[1] = res[2] = res[3] = res[4] = 0;
    res[5] = -1;
    if ((m & M_LIVE) && pin[slot] == rank && seqa[slot] == seq) {
        int4 c0 = cold0[slot], c1 = cold1[slot];
        res[0] = 1;
        res[1] = c0.y;
        res[2] = c1.z;
        res[3] = prio[slot];
        res[4] = c0.x;
        res[5] = c1.w;
        meta[slot] = 0;
        bytes_add(ctr, -(BYTES_WQ + c0.y));  // wq_delete frees the record, node and payload (xq.c:160-174)
    }
}

__global__ void k_unreserve(int slot, int rank, int seq, int newpin, uint32_t *meta, int *pin,
                            const int *seqa, int *res, const int *prio, long long *anchor) {
    uint32_t m = meta[slot];
    res[0] = 0;
    if ((m & M_LIVE) && pin[slot] == rank && seqa[slot] == seq) {
        pin[slot] = newpin;
        meta[slot] = m & ~M_PINNED;
        atomicMax(&anchor[m & M_TYPE], (long long)prio[slot]);
        res[0] = 1;
    }
}

__global__ void k_unreserve_batch(const int *__restrict__ trip, int n, const long long *__restrict__ seq2slot,
                                  long long nseq, uint32_t *meta, int *pin, const int4 *__restrict__ rrec,
                                  long long *anchor) {
    unreserve_triple(blockIdx.x * blockDim.x + threadIdx.x, trip, n, seq2slot, nseq, meta, pin, rrec, anchor);
}

// FA_GET_RESERVED for a batch of (rank, wqseqno) pairs (adlb.c:1347-1381:
// wq_find_pinned_for_rank, then wq_delete).  Sequentially a unit can be got
// once: of several valid Gets of one wqseqno in a batch the lowest index wins
// (claimed with atomicMin in k_get_claim), the others find it gone.
__global__ void k_get_claim(const int *__restrict__ pairs, int n, const long long *__restrict__ seq2slot,
                            long long nseq, const uint32_t *__restrict__ meta, const int *__restrict__ pin,
                            const int *__restrict__ seqa, int *claim) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int rank = pairs[2 * i], seq = pairs[2 * i + 1];
    const long long slot = (seq > 0 && seq < nseq) ? seq2slot[seq] : -1;
    if (slot < 0) return;
    if ((meta[slot] & M_LIVE) && pin[slot] == rank && seqa[slot] == seq) atomicMin(&claim[seq], i);
}

__global__ void k_get_apply(const int *__restrict__ pairs, int n, long long *seq2slot, long long nseq,
                            uint32_t *meta, const int *__restrict__ prio, const int4 *__restrict__ cold0,
                            const int4 *__restrict__ cold1, int *claim, int *out5, DevCounters *ctr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int ok = 0, tgt = 0;
    long long freed = 0;
    if (i < n) {
        const int seq = pairs[2 * i + 1];
        int o[5] = {-1, 0, 0, 0, 0};
        if (seq > 0 && seq < nseq && claim[seq] == i) {
            const long long slot = seq2slot[seq];
            const int4 c0 = cold0[slot], c1 = cold1[slot];
            o[0] = 1;
            o[1] = c0.y;
            o[2] = c1.z;
            o[3] = prio[slot];
            o[4] = c0.x;
            meta[slot] = 0;
            seq2slot[seq] = -1;
            claim[seq] = INT_MAX;  // for the next batch
            ok = 1;
            tgt = c1.w >= 0;
            freed = BYTES_WQ + c0.y;
        }
#pragma unroll
        for (int k = 0; k < 5; k++) out5[5 * i + k] = o[k];
    }
    // wave totals: removed units, targeted ones, freed bytes (deletions only lower the count: no mark)
    const unsigned long long b = __ballot(ok), bt = __ballot(tgt);
    for (int o = 32; o > 0; o >>= 1) freed += __shfl_xor(freed, o, 64);
    if ((threadIdx.x & 63) == 0 && b) {
        atomicAdd((unsigned long long *)&ctr->got, (unsigned long long)__popcll(b));
        if (bt) atomicAdd((unsigned long long *)&ctr->got_targeted, (unsigned long long)__popcll(bt));
        atomicAdd((unsigned long long *)&ctr->bytes, (unsigned long long)(-freed));
    }
}

// A Get batch of at most 256 in one launch (the synchronous entry's few dozen
// Gets): claim, barrier, apply, then the counters into mapped memory -- the
// work of k_get_claim, k_get_apply and k_ctr_out without two launch boundaries.
__global__ __launch_bounds__(256) void k_get_small(const int *__restrict__ pairs, int n, long long *seq2slot,
                                                   long long nseq, uint32_t *meta, const int *__restrict__ pin,
                                                   const int *__restrict__ seqa, const int *__restrict__ prio,
                                                   const int4 *__restrict__ cold0, const int4 *__restrict__ cold1,
                                                   int *claim, int *out5, DevCounters *ctr, DevCounters *zctr) {
    const int i = threadIdx.x;
    int seq = 0;
    long long slot = -1;
    if (i < n) {
        const int rank = pairs[2 * i];
        seq = pairs[2 * i + 1];
        slot = (seq > 0 && seq < nseq) ? seq2slot[seq] : -1;
        if (slot >= 0 && (meta[slot] & M_LIVE) && pin[slot] == rank && seqa[slot] == seq) atomicMin(&claim[seq], i);
    }
    __syncthreads();
    int ok = 0, tgt = 0;
    long long freed = 0;
    if (i < n) {
        int o[5] = {-1, 0, 0, 0, 0};
        if (slot >= 0 && __hip_atomic_load(claim + seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == i) {
            const int4 c0 = cold0[slot], c1 = cold1[slot];
            o[0] = 1;
            o[1] = c0.y;
            o[2] = c1.z;
            o[3] = prio[slot];
            o[4] = c0.x;
            meta[slot] = 0;
            seq2slot[seq] = -1;
            claim[seq] = INT_MAX;  // for the next batch
            ok = 1;
            tgt = c1.w >= 0;
            freed = BYTES_WQ + c0.y;
        }
#pragma unroll
        for (int k = 0; k < 5; k++) out5[5 * i + k] = o[k];
    }
    const unsigned long long b = __ballot(ok), bt = __ballot(tgt);
    for (int o = 32; o > 0; o >>= 1) freed += __shfl_xor(freed, o, 64);
    if ((threadIdx.x & 63) == 0 && b) {
        atomicAdd((unsigned long long *)&ctr->got, (unsigned long long)__popcll(b));
        if (bt) atomicAdd((unsigned long long *)&ctr->got_targeted, (unsigned long long)__popcll(bt));
        atomicAdd((unsigned long long *)&ctr->bytes, (unsigned long long)(-freed));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // every field after the block's atomics (L2 reads), into mapped host memory
    const int *src = reinterpret_cast<const int *>(ctr);
    int *dst = reinterpret_cast<int *>(zctr);
    for (int k = threadIdx.x; k < (int)(sizeof(DevCounters) / 4); k += blockDim.x)
        dst[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// FA_INFO_NUM_WORK_UNITS (adlb.c:2466-2496) in one pass over every page:
// max prio of the type (strict >, from LOWEST), units at that max, units of
// the type.  Blocks publish partials; the last to arrive combines them.
__global__ __launch_bounds__(256) void k_info_fused(const int *__restrict__ pages, const int *__restrict__ fills,
                                                    int npages, const int *__restrict__ prio,
                                                    const uint32_t *__restrict__ meta, int tidx, int vw, int *part,
                                                    int *res) {
    __shared__ int smx[4], scm[4], scn[4];
    __shared__ bool s_last;
    int mx = LOWEST, cm = 0, cn = 0;
    for (int p = blockIdx.x; p < npages; p += gridDim.x) {
        const long long base = (long long)pages[p] << PAGE_SHIFT;
        for (int o = threadIdx.x; o < fills[p]; o += blockDim.x) {
            const uint32_t m = meta[base + o];
            if ((m & M_LIVE) && meta_type(m, vw) == tidx) {
                const int pr = prio[base + o];
                cn++;
                if (pr > mx) {
                    mx = pr;
                    cm = 1;
                } else if (pr == mx) {
                    cm++;
                }
            }
        }
    }
    // combine (max, count at max, count) over the block
    for (int o = 32; o > 0; o >>= 1) {
        const int m2 = __shfl_xor(mx, o, 64), c2 = __shfl_xor(cm, o, 64), n2 = __shfl_xor(cn, o, 64);
        cm = m2 > mx ? c2 : m2 == mx ? cm + c2 : cm;
        mx = max(mx, m2);
        cn += n2;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        smx[w] = mx;
        scm[w] = cm;
        scn[w] = cn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int q = 1; q < 4; q++) {
            cm = smx[q] > mx ? scm[q] : smx[q] == mx ? cm + scm[q] : cm;
            mx = max(mx, smx[q]);
            cn += scn[q];
        }
        __hip_atomic_store(part + 3 * blockIdx.x, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part + 3 * blockIdx.x + 1, cm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part + 3 * blockIdx.x + 2, cn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = atomicAdd(part + 3 * gridDim.x, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last || threadIdx.x != 0) return;
    mx = LOWEST;
    cm = cn = 0;
    for (int b = 0; b < (int)gridDim.x; b++) {
        const int m2 = __hip_atomic_load(part + 3 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int c2 = __hip_atomic_load(part + 3 * b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cm = m2 > mx ? c2 : m2 == mx ? cm + c2 : cm;
        mx = max(mx, m2);
        cn += __hip_atomic_load(part + 3 * b + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    part[3 * gridDim.x] = 0;  // for the next call
    res[0] = mx;
    res[1] = cm;
    res[2] = cn;
}


// SS_UNRESERVE of every unit a reserve batch handed out, read straight from the
// batch's requests and TA_RESERVE_RESP records (rc 1 = matched, [5] = wqseqno;
// the new pin is -1, i.e. the unit is available again).  The slot comes from
// the last batch's record of what it gave request i (mslot, read with the
// response: one dependent load level fewer), checked against the unit's
// wqseqno; responses of another batch fall back to the wqseqno -> slot map.
// The anchor is raised by a fire-and-forget atomic max per type of the wave
// (a stale read could only add a harmless one: no load of it first).

__global__ void k_unreserve_resp(const int *__restrict__ reqs, const int *__restrict__ resp, int n,
                                 const long long *__restrict__ seq2slot, long long nseq, uint32_t *meta, int *pin,
                                 const int4 *__restrict__ rrec, long long *anchor, const int2 *__restrict__ mslot,
                                 int ntypes, const int2 *__restrict__ rh, int trusted) {
    unreserve_resp_body(reqs, resp, n, seq2slot, nseq, meta, pin, rrec, anchor, mslot, ntypes, blockIdx.x, rh,
                        trusted != 0);
}

// The last batch's compacted (rank, hang) rows when the unreserve is of that batch's own requests
// (k_finalize read the same rows), else none (the ranks come from the request records).
static const int2 *unres_rh(const adlbq_server *h, const int *d_reqs18, int n) {
    return (h->d_rh && d_reqs18 == h->last_reqs && n == h->last_R) ? h->d_rh : nullptr;
}
// ... and nothing has changed the queue since that batch launched (read before this call's wq_changed):
// k_unreserve_resp's exact path from the batch's (slot, wqseqno) records alone
static int unres_trusted(const adlbq_server *h, const int *d_reqs18, int n) {
    return (unres_rh(h, d_reqs18, n) != nullptr && h->d_mslot && n <= h->cap_req && h->unres_trust &&
            h->mslot_epoch == h->mut_epoch) ? 1 : 0;
}

// adlbq_unreserve_resp_group_device: up to UNRES_GROUP shards per launch, blockIdx.y = shard, the
// arguments in the kernel's own argument block (no table upload)
constexpr int UNRES_GROUP = 16;
struct UnresArgs {
    const int *reqs, *resp;
    int n;
    const long long *seq2slot;
    long long nseq;
    uint32_t *meta;
    int *pin;
    const int4 *rrec;
    long long *anchor;
    const int2 *mslot;
    int ntypes;
    const int2 *rh;
    int trusted;
};
struct UnresGroup {
    UnresArgs a[UNRES_GROUP];
};
__global__ __launch_bounds__(256) void k_unreserve_resp_g(const UnresGroup g) {
    const UnresArgs &a = g.a[blockIdx.y];
    if ((int)blockIdx.x * 256 >= a.n) return;  // whole workgroups return together
    unreserve_resp_body(a.reqs, a.resp, a.n, a.seq2slot, a.nseq, a.meta, a.pin, a.rrec, a.anchor, a.mslot, a.ntypes,
                        blockIdx.x, a.rh, a.trusted != 0);
}

// Several handles' work as one launch on the first handle's stream (hs[m[0]]):
// that stream first waits for what every member's stream already holds, and
// every member's stream then waits for the launch (events kept by the first).
namespace adlbq {
int group_join(adlbq_server *const *hs, const std::vector<int> &m) {
    adlbq_server *L = hs[m[0]];
    if (L->gjoin.size() < m.size()) {
        const size_t old = L->gjoin.size();
        L->gjoin.resize(m.size(), nullptr);
        for (size_t j = old; j < m.size(); j++) AQ_HIP(hipEventCreateWithFlags(&L->gjoin[j], hipEventDisableTiming));
    }
    for (size_t j = 1; j < m.size(); j++) {
        adlbq_server *h = hs[m[j]];
        if (h->stream == L->stream) continue;
        AQ_HIP(hipEventRecord(L->gjoin[j], h->stream));
        AQ_HIP(hipStreamWaitEvent(L->stream, L->gjoin[j], 0));
    }
    return ADLBQ_OK;
}

int group_release(adlbq_server *const *hs, const std::vector<int> &m) {
    adlbq_server *L = hs[m[0]];
    AQ_HIP(hipEventRecord(L->gjoin[0], L->stream));
    for (size_t j = 1; j < m.size(); j++) {
        adlbq_server *h = hs[m[j]];
        if (h->stream != L->stream) AQ_HIP(hipStreamWaitEvent(h->stream, L->gjoin[0], 0));
    }
    return ADLBQ_OK;
}
}  // namespace adlbq

// update_local_state over the open bucket: count of live unpinned units and per
// type max prio (strictly above ADLB_LOWEST_PRIO, else LOWEST)
__global__ void k_qmrow(const int *__restrict__ pages, int npages, int tail_fill, const int *__restrict__ prio,
                        const uint32_t *__restrict__ meta, int T, int *res /* [0]=qlen, [1+t]=max */) {
    __shared__ int smax[ADLBQ_MAX_TYPES_WIDE];
    __shared__ int scnt;
    const int vw = T > VW_TYPES;  // more than 255 types: the maxima go straight to res (global atomics)
    if (!vw)
        for (int t = threadIdx.x; t < T; t += blockDim.x) smax[t] = LOWEST;
    if (threadIdx.x == 0) scnt = 0;
    __syncthreads();
    int cnt = 0;
    long long total = (long long)npages * PAGE;
    for (long long L = (long long)blockIdx.x * blockDim.x + threadIdx.x; L < total;
         L += (long long)gridDim.x * blockDim.x) {
        int p = (int)(L >> PAGE_SHIFT), off = (int)(L & (PAGE - 1));
        if (p == npages - 1 && off >= tail_fill) continue;
        long long s = ((long long)pages[p] << PAGE_SHIFT) + off;
        uint32_t m = meta[s];
        if ((m & (M_LIVE | M_PINNED)) == M_LIVE) {
            cnt++;
            int pr = prio[s];
            if (pr > LOWEST) {
                if (vw) atomicMax(&res[1 + meta_type(m, 1)], pr);
                else atomicMax(&smax[m & M_TYPE], pr);
            }
        }
    }
    atomicAdd(&scnt, cnt);
    __syncthreads();
    if (!vw)
        for (int t = threadIdx.x; t < T; t += blockDim.x)
            if (smax[t] > LOWEST) atomicMax(&res[1 + t], smax[t]);
    if (threadIdx.x == 0) atomicAdd(&res[0], scnt);
}

// whole-store scan helper (wq_find_unpinned)
__global__ void k_first_unpinned(const int *__restrict__ pages, const int *__restrict__ fills, int npages,
                                 const uint32_t *__restrict__ meta, const int *__restrict__ seqa, int *res) {
    int p = blockIdx.x;
    if (p >= npages) return;
    long long base = (long long)pages[p] << PAGE_SHIFT;
    int best = INT_MAX;
    for (int o = threadIdx.x; o < fills[p]; o += blockDim.x) {
        uint32_t m = meta[base + o];
        if ((m & (M_LIVE | M_PINNED)) == M_LIVE) {
            int s = seqa[base + o];
            best = s < best ? s : best;
        }
    }
    if (best != INT_MAX) atomicMin(res, best);
}

// check_remote_work_for_queued_apps, one wavefront over rq in FIFO order
__global__ void k_checkrem(DonorCtx c, const int *__restrict__ rq_rank, const int *__restrict__ rq_types,
                           const int *rq_live, const int *__restrict__ rq_seq, const DevCounters *ctr, int cap,
                           int *out3, int *count) {
    int k0 = ctr->rq_head, nrq = ctr->rq_n, n = 0;
    for (int k = k0; k < nrq; k++) {
        if (!ld_agent(rq_live + k)) continue;
        int rank = rq_rank[k];
        if (rank >= 0 && rank < c.A && ld_agent(c.rfr_to_rank + rank) >= 0) continue;
        int cand = rfr_select(c, rank, rq_types + (long long)k * NREQ);
        if (cand >= 0) {
            if (threadIdx.x == 0 && n < cap) {
                out3[3 * n] = rq_seq[k];
                out3[3 * n + 1] = rank;
                out3[3 * n + 2] = cand;
            }
            n++;
        }
    }
    if (threadIdx.x == 0) *count = n;
}

__global__ void k_rq_delete(int rqseqno, const int *__restrict__ rq_seq, int *rq_live, DevCounters *ctr, int *res) {
    res[0] = 0;
    const int k = rq_slot_of(rq_seq, ctr->rq_n, rqseqno);
    if (k >= 0 && rq_live[k]) {
        rq_live[k] = 0;
        ctr->rq_live--;
        bytes_add(ctr, -BYTES_RQ);
        res[0] = 1;
        int head = ctr->rq_head;
        while (head < ctr->rq_n && !rq_live[head]) head++;
        ctr->rq_head = head;
    }
}

// SS_RFR_RESP failure's retry for the original Reserve (adlb.c:2007-2041): if
// rqseqno is still parked, its first type with a donor gets a new SS_RFR
__global__ void k_rfr_retry(DonorCtx c, const int *__restrict__ rq_rank, const int *__restrict__ rq_types,
                            const int *rq_live, const int *__restrict__ rq_seq, const DevCounters *ctr, int rqseqno,
                            int *out2) {
    int found = 0, cand = -1;
    const int k = rq_slot_of(rq_seq, ctr->rq_n, rqseqno);
    if (k >= 0 && ld_agent(rq_live + k)) {
        found = 1;
        cand = rfr_select(c, rq_rank[k], rq_types + (long long)k * NREQ);
    }
    if (threadIdx.x == 0) {
        out2[0] = found;
        out2[1] = cand;
    }
}

// ---- memory-pressure push (adlb.c:2109-2362): single-unit control operations
// a unit accepted by SS_PUSH_QUERY is held for the server (pinned to it) until SS_PUSH_HDR
__global__ void k_push_hold(int slot, int pin_rank, uint32_t *meta, int *pin) {
    meta[slot] |= M_PINNED;
    pin[slot] = pin_rank;
}

// SS_PUSH_QUERY_RESP at the pusher: the unit leaves if still live and unpinned (adlb.c:2179-2222)
__global__ void k_push_take(int slot, int seq, const int *prio, uint32_t *meta, const int *seqa,
                            const int4 *cold0, const int4 *cold1, int *res, DevCounters *ctr) {
    const uint32_t m = meta[slot];
    res[0] = 0;
    if ((m & (M_LIVE | M_PINNED)) == M_LIVE && seqa[slot] == seq) {
        const int4 c0 = cold0[slot], c1 = cold1[slot];  // {answer, len, home, clen}, {csrv, cseq, utype, target}
        res[0] = 1;
        res[1] = c1.z;
        res[2] = prio[slot];
        res[3] = c0.y;
        res[4] = c0.x;
        res[5] = c1.w;
        res[6] = c0.z;
        res[7] = c0.w;
        res[8] = c1.x;
        res[9] = c1.y;
        meta[slot] = 0;
        bytes_add(ctr, -(BYTES_WQ + c0.y));  // wq_delete (the payload leaves with the Isend, adlb.c:2221)
    }
}

// SS_PUSH_HDR at the pushee (adlb.c:2232-2340): unpin, then the put-side FIFO
// match of k_put_match for this one unit (rq_find_rank_queued_for_type,
// xq.c:388-405); one wavefront
__global__ void k_push_commit(int slot, int seq, const int *prio, uint32_t *meta, int *pin, const int *seqa,
                              const int4 *cold1, const int *__restrict__ rq_rank, const int *__restrict__ rq_types,
                              int *rq_live, const int *__restrict__ rq_seq, DevCounters *ctr, long long *anchor,
                              int *res) {
    const int lane = threadIdx.x;
    const uint32_t m = meta[slot];
    if (!((m & M_LIVE) && seqa[slot] == seq)) {
        if (lane == 0) res[0] = 0, res[1] = -1, res[2] = -1;
        return;
    }
    const int4 c1 = cold1[slot];
    const int utype = c1.z, target = c1.w;
    const int head = ctr->rq_head, nrq = ctr->rq_n;
    int found = -1;
    if (ctr->rq_live > 0) {
        for (int base = head; base < nrq; base += 64) {
            const int k = base + lane;
            bool hit = false;
            if (k < nrq && ld_agent(rq_live + k)) {
                const int rk = rq_rank[k];
                if (target == -1 || target == rk) {
                    const int *tv = rq_types + (long long)k * NREQ;
#pragma unroll
                    for (int q = 0; q < NREQ; q++) hit |= (tv[q] == -1 || tv[q] == utype);
                }
            }
            const unsigned long long b = __ballot(hit);
            if (b) {
                found = base + __ffsll((long long)b) - 1;
                break;
            }
        }
    }
    if (lane == 0) {
        res[0] = 1;
        res[1] = -1;
        res[2] = -1;
        pin[slot] = -1;
        meta[slot] = m & ~M_PINNED;
        if (found >= 0) {
            const int rk = rq_rank[found];
            st_agent(rq_live + found, 0);
            res[1] = rk;
            res[2] = rq_seq[found];
            bytes_add(ctr, -BYTES_RQ);  // rq_delete (adlb.c:2338)
            pin[slot] = rk;
            if (rk >= 0) meta[slot] = m | M_PINNED;
            ctr->rq_live -= 1;
        } else {
            atomicMax(&anchor[m & M_TYPE], (long long)prio[slot]);  // available: the anchor bounds it
        }
    }
    if (found >= 0 && found == head) {  // advance the FIFO head past dead entries
        if (lane == 0) {
            int hd = head;
            while (hd < nrq && !ld_agent(rq_live + hd)) hd++;
            ctr->rq_head = hd;
        }
    }
}

// SS_PUSH_DEL at the pushee (adlb.c:2353-2360): the held unit is dropped
__global__ void k_push_discard(int slot, int seq, uint32_t *meta, const int *seqa, const int4 *cold0,
                               const int4 *cold1, int *res, DevCounters *ctr) {
    const uint32_t m = meta[slot];
    res[0] = 0;
    if ((m & M_LIVE) && seqa[slot] == seq) {
        const int4 c0 = cold0[slot];
        res[0] = 1;
        res[1] = cold1[slot].w;
        meta[slot] = 0;
        bytes_add(ctr, -(BYTES_WQ + c0.y));  // wq_delete frees node, record and the payload buffer
    }
}

__global__ void k_set_int(int *p, int v) { *p = v; }

__global__ void k_add_bytes(DevCounters *ctr, long long d) { bytes_add(ctr, d); }

// ============================================================================ C ABI

static bool ok_handle(adlbq_server *h) { return h != nullptr; }

extern "C" {

const char *adlbq_last_error(void) { return g_err.c_str(); }
const char *adlbq_version(void) { return "adlbq 0.1 (gfx950)"; }

int adlbq_create(adlbq_server **out, int ntypes, const int *user_types, int num_app_ranks, int num_servers,
                 int my_server_idx, long long max_units, int device) {
    if (!out || ntypes < 0 || (ntypes && !user_types) || num_app_ranks < 0 || num_servers < 1 ||
        my_server_idx < 0 || my_server_idx >= num_servers)
        return fail(ADLBQ_ERR_ARG, "adlbq_create: bad argument");
    if (ntypes > ADLBQ_MAX_TYPES_VWIDE)
        return fail(ADLBQ_ERR_UNSUPPORTED, "adlbq_create: more than 2^22 work types");
    if (ntypes > ADLBQ_MAX_TYPES && num_app_ranks >= (1 << 24) - 2)
        return fail(ADLBQ_ERR_UNSUPPORTED, "adlbq_create: more than 64 types with 2^24 or more app ranks");
    auto *h = new adlbq_server();
    hipError_t e;
    if (device < 0) {  // one GPU per server shard, round robin over the visible devices
        int ndev = 0;
        if ((e = hipGetDeviceCount(&ndev)) != hipSuccess || ndev < 1) {
            delete h;
            return hip_fail(e == hipSuccess ? hipErrorNoDevice : e, "hipGetDeviceCount");
        }
        device = my_server_idx % ndev;
    }
    h->device = device;
    e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete h;
        return hip_fail(e, "hipSetDevice");
    }
    if ((e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking)) != hipSuccess) {
        delete h;
        return hip_fail(e, "hipStreamCreate");
    }
    h->stream = h->own_stream;
    h->T = ntypes;
    h->utypes.assign(user_types, user_types + ntypes);
    for (int i = 0; i < ntypes; i++)
        if (!h->tindex.count(user_types[i])) h->tindex[user_types[i]] = i;  // get_type_idx: first match
    h->A = num_app_ranks;
    h->S = num_servers;
    h->my_idx = my_server_idx;
    h->master = num_app_ranks;                    // adlb.c:256
    h->my_world = num_app_ranks + my_server_idx;
    h->num_world = num_app_ranks + num_servers;
    h->qm_hi.assign((size_t)num_servers * std::max(ntypes, 1), LOWEST);  // adlb.c:301-316
    h->qm_qlen.assign(num_servers, 0);
    h->qm_bytes.assign(num_servers, 0.0);
    h->seq2slot.assign(1, -1);
    int rc;
    auto cleanup = [&](int code) { adlbq_destroy(h); return code; };
    int T1 = std::max(ntypes, 1);
    AQ_HIP(hipMalloc((void **)&h->d_anchor, sizeof(long long) * T1));
    AQ_HIP(hipMalloc((void **)&h->d_anchor_next, sizeof(long long) * T1));
    AQ_HIP(hipMalloc((void **)&h->d_gcut, sizeof(long long) * T1));
    AQ_HIP(hipMalloc((void **)&h->d_gcut_next, sizeof(long long) * T1));
    {  // anchors start below every prio; the device keeps them (puts / unreserves raise, batches lower)
        std::vector<long long> lo(T1, (long long)INT_MIN), none(T1, LLONG_MIN);
        AQ_HIP(hipMemcpy(h->d_anchor, lo.data(), sizeof(long long) * T1, hipMemcpyHostToDevice));
        AQ_HIP(hipMemcpy(h->d_anchor_next, none.data(), sizeof(long long) * T1, hipMemcpyHostToDevice));
        AQ_HIP(hipMemcpy(h->d_gcut_next, none.data(), sizeof(long long) * T1, hipMemcpyHostToDevice));
        std::vector<long long> noguess(T1, LLONG_MAX);
        AQ_HIP(hipMemcpy(h->d_gcut, noguess.data(), sizeof(long long) * T1, hipMemcpyHostToDevice));
    }
    AQ_HIP(hipMalloc((void **)&h->d_utypes, sizeof(int) * T1));
    if (ntypes) AQ_HIP(hipMemcpy(h->d_utypes, user_types, sizeof(int) * ntypes, hipMemcpyHostToDevice));
    AQ_HIP(hipMalloc((void **)&h->d_qm_hi, sizeof(int) * num_servers * T1));
    AQ_HIP(hipMalloc((void **)&h->d_qm_qlen, sizeof(int) * num_servers));
    AQ_HIP(hipMalloc((void **)&h->d_rfr_out, sizeof(int) * std::max(h->num_world, 1)));
    AQ_HIP(hipMemsetAsync(h->d_rfr_out, 0, sizeof(int) * std::max(h->num_world, 1), h->stream));  // SURVEY hard part 4
    AQ_HIP(hipMalloc((void **)&h->d_rfr_to_rank, sizeof(int) * std::max(num_app_ranks, 1)));
    AQ_HIP(hipMemsetAsync(h->d_rfr_to_rank, 0xff, sizeof(int) * std::max(num_app_ranks, 1), h->stream));
    AQ_HIP(hipMalloc((void **)&h->d_ctr, sizeof(DevCounters)));
    AQ_HIP(hipMemsetAsync(h->d_ctr, 0, sizeof(DevCounters), h->stream));
    AQ_HIP(hipHostMalloc((void **)&h->h_snap, sizeof(DevCounters) * adlbq_server::NSNAP, hipHostMallocMapped));
    memset(h->h_snap, 0, sizeof(DevCounters) * adlbq_server::NSNAP);
    AQ_HIP(hipHostGetDevicePointer((void **)&h->d_snap, h->h_snap, 0));
    AQ_HIP(hipMalloc((void **)&h->d_dem, sizeof(int) * T1));
    AQ_HIP(hipMemsetAsync(h->d_dem, 0, sizeof(int) * T1, h->stream));  // k_finalize re-zeroes it after every batch
    AQ_HIP(hipMalloc((void **)&h->d_theta, sizeof(int) * T1));
    AQ_HIP(hipMalloc((void **)&h->d_need, sizeof(int) * T1));
    AQ_HIP(hipMalloc((void **)&h->d_candoff, sizeof(int) * (T1 + 1)));
    AQ_HIP(hipMalloc((void **)&h->d_candlen, sizeof(int) * T1));
    AQ_HIP(hipMalloc((void **)&h->d_needsort, sizeof(int) * T1));
    AQ_HIP(hipMalloc((void **)&h->d_binoff, sizeof(int) * T1 * NB));
    AQ_HIP(hipMalloc((void **)&h->d_coltot, sizeof(unsigned int) * T1 * NB));
    AQ_HIP(hipMalloc((void **)&h->d_type_cnt, sizeof(int) * T1));
    AQ_HIP(hipMemsetAsync(h->d_type_cnt, 0, sizeof(int) * T1, h->stream));
    AQ_HIP(hipMalloc((void **)&h->d_rank_sync, sizeof(int) * (ADLBQ_MAX_TYPES + 6)));
    AQ_HIP(hipMemsetAsync(h->d_rank_sync, 0, sizeof(int) * (ADLBQ_MAX_TYPES + 6), h->stream));
    AQ_HIP(hipMalloc((void **)&h->d_result, sizeof(int) * (std::max(ntypes, ADLBQ_MAX_TYPES_WIDE) + 16)));
    AQ_HIP(hipHostMalloc((void **)&h->h_result, sizeof(int) * (std::max(ntypes, ADLBQ_MAX_TYPES_WIDE) + 16)));
    if (ntypes > VW_TYPES) {  // the wide path's (value, first declared index) table, sorted by value
        std::vector<std::pair<int, int>> vs;
        for (int i = 0; i < ntypes; i++) vs.emplace_back(user_types[i], i);
        std::stable_sort(vs.begin(), vs.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        std::vector<int2> tab;
        for (size_t i = 0; i < vs.size(); i++)
            if (i == 0 || vs[i].first != vs[i - 1].first) tab.push_back(make_int2(vs[i].first, vs[i].second));
        h->n_utsorted = (int)tab.size();
        AQ_HIP(hipMalloc((void **)&h->d_utsorted, sizeof(int2) * tab.size()));
        AQ_HIP(hipMemcpy(h->d_utsorted, tab.data(), sizeof(int2) * tab.size(), hipMemcpyHostToDevice));
    }
    long long pages = std::max<long long>(16, (max_units + PAGE - 1) / PAGE + 16);
    if ((rc = grow_pages(h, (int)std::min<long long>(pages, INT_MAX / PAGE)))) return cleanup(rc);
    if ((rc = ensure_rq_capacity(h, 1024))) return cleanup(rc);
    AQ_HIP(hipStreamSynchronize(h->stream));
    *out = h;
    return ADLBQ_OK;
}

int adlbq_destroy(adlbq_server *h) {
    if (!h) return ADLBQ_OK;
    hipSetDevice(h->device);
    if (h->own_stream) hipStreamSynchronize(h->own_stream);
    void *ptrs[] = {h->d_tab, h->d_prio, h->d_meta, h->d_pin, h->d_seq, h->d_cold0, h->d_cold1, h->d_rrec,
                    h->d_tcnt, h->d_tlist, h->d_seq2slot, h->d_anchor, h->d_anchor_next, h->d_gcut, h->d_gcut_next, h->d_spec, h->d_specn, h->d_utypes, h->d_rq_rank, h->d_rq_types,
                    h->d_rq_live, h->d_rq_req, h->d_rq_seq, h->d_ctr, h->d_qm_hi, h->d_qm_qlen, h->d_rfr_out, h->d_rfr_to_rank, h->d_tq,
                    h->d_mask, h->d_tmatch, h->d_umatch, h->d_reqbuf, h->d_respbuf, h->d_dem, h->d_theta,
                    h->d_need, h->d_candoff, h->d_candlen, h->d_needsort, h->d_binoff, h->d_coltot, h->d_type_cnt, h->d_rank_sync, h->d_gh, h->d_csum,
                    h->d_ckey, h->d_ckey2, h->d_cslot, h->d_cslot2, h->d_crank, h->d_result,
                    h->d_kst, h->d_putrec, h->d_putout, h->d_seg_cnt, h->d_chS, h->d_chD, h->d_chLP, h->d_chGT, h->d_chGO, h->d_chclean, h->d_cht, h->d_chcnt, h->d_chE, h->d_chflag, h->d_stamps, h->d_export,
                    h->d_navail, h->d_rqx, h->d_apply, h->d_apply_bad, h->d_pmask, h->d_lv, h->d_rtype, h->d_pm_over,
                    h->d_tkeys, h->d_tkeys2, h->d_tvals, h->d_tvals2, h->d_tstart, h->d_tend, h->d_tsort,
                    h->d_ssort, h->d_kb, h->d_getclaim, h->d_getbuf, h->d_info, h->d_crem,
                    h->d_ckey3, h->d_cslot3, h->d_plan, h->d_rs, h->d_rs_cnt, h->d_rs_acc,
                    h->d_dkeys, h->d_dkeys2, h->d_dvals, h->d_dvals2, h->d_dstart, h->d_dend,
                    h->d_mslot, h->d_rh, h->d_wk0, h->d_wk1, h->d_wekey, h->d_wv0, h->d_wv1,
                    h->d_wflag, h->d_wrstart, h->d_whead, h->d_wrkey, h->d_wreq, h->d_wcnt, h->d_wpages, h->d_wtmp, h->d_kr,
                    h->d_onepart, h->d_utsorted, h->d_jpref};
    for (void *p : ptrs)
        if (p) hipFree(p);
    if (h->h_result) hipHostFree(h->h_result);
    if (h->h_snap) hipHostFree(h->h_snap);
    if (h->h_zc) hipHostFree(h->h_zc);
    if (h->h_zctr) hipHostFree(h->h_zctr);
    for (int q = 0; q < 2; q++) {
        if (h->h_tab[q]) hipHostFree(h->h_tab[q]);
        if (h->tab_ev[q]) hipEventDestroy(h->tab_ev[q]);
    }
    if (h->h_steal) hipHostFree(h->h_steal);
    if (h->h_apply) hipHostFree(h->h_apply);
    if (h->h_crem) hipHostFree(h->h_crem);
    if (h->h_pdead) hipHostFree(h->h_pdead);
    if (h->pdead_ev) hipEventDestroy(h->pdead_ev);
    for (int q = 0; q < 2; q++)
        if (h->h_putrec[q]) hipHostFree(h->h_putrec[q]);
    if (h->d_tnewk) hipFree(h->d_tnewk);
    if (h->d_tnewv) hipFree(h->d_tnewv);
    for (int q = 0; q < 2; q++)
        if (h->put_ev[q]) hipEventDestroy(h->put_ev[q]);
    for (int q = 0; q < 2; q++) {
        if (h->gtab_ev[q]) hipEventDestroy(h->gtab_ev[q]);
        if (h->h_gtab[q]) hipHostFree(h->h_gtab[q]);
    }
    if (h->d_gtab) hipFree(h->d_gtab);
    for (hipEvent_t e : h->gjoin)
        if (e) hipEventDestroy(e);
    for (int q = 0; q < 2; q++) {
        if (h->tnew_ev[q]) hipEventDestroy(h->tnew_ev[q]);
        if (h->h_tnewk[q]) hipHostFree(h->h_tnewk[q]);
        if (h->h_tnewv[q]) hipHostFree(h->h_tnewv[q]);
    }
    if (h->steal_ev) hipEventDestroy(h->steal_ev);
    if (h->apply_ev) hipEventDestroy(h->apply_ev);
    for (auto &kv : h->timers)
        for (auto &pe : kv.second.pending) {
            hipEventDestroy(pe.first);
            hipEventDestroy(pe.second);
        }
    for (hipEvent_t e : h->event_pool) hipEventDestroy(e);
    if (h->own_stream) hipStreamDestroy(h->own_stream);
    delete h;
    return ADLBQ_OK;
}

// the put path's type lookup (get_type_idx, adlb.c:3476-3485): a dense table over
// the declared types' value range when it is small, the map otherwise
static inline int type_index(adlbq_server *h, int v) {
    if (h->tindex.empty()) return -1;
    if (h->tindex_dense.empty() && h->tindex.size() <= 4096) {
        int lo = INT_MAX, hi = INT_MIN;
        for (const auto &kv : h->tindex) lo = std::min(lo, kv.first), hi = std::max(hi, kv.first);
        if ((long long)hi - lo < (1 << 20)) {
            h->tindex_lo = lo;
            h->tindex_dense.assign((size_t)((long long)hi - lo + 1), -1);
            for (const auto &kv : h->tindex) h->tindex_dense[(size_t)(kv.first - lo)] = kv.second;
        }
    }
    if (!h->tindex_dense.empty()) {
        const long long d = (long long)v - h->tindex_lo;
        return (d >= 0 && d < (long long)h->tindex_dense.size()) ? h->tindex_dense[(size_t)d] : -1;
    }
    auto it = h->tindex.find(v);
    return it == h->tindex.end() ? -1 : it->second;
}

static int rank_bucket(adlbq_server *h, int target) {
    if (target < h->A && h->rank_index_dense.size() == (size_t)h->A && h->rank_index_dense[(size_t)target] >= 0)
        return h->rank_index_dense[(size_t)target];
    auto it = h->rank_index.find(target);
    if (it != h->rank_index.end()) return it->second;
    int k = (int)h->bucket_ranks.size();
    h->bucket_ranks.push_back(target);
    h->rankb.emplace_back();
    h->rank_index[target] = k;
    if (target < h->A) {
        if (h->rank_index_dense.size() != (size_t)h->A) h->rank_index_dense.assign((size_t)h->A, -1);
        h->rank_index_dense[(size_t)target] = k;
    }
    return k;
}

// out3: host results (synchronises when a parked Reserve may match); d_out3:
// device results, nothing waits (adlbq_put_batch_device)
// hold_rank >= 0: one unit held for that server (adlbq_push_accept): pinned, no rq match
static int put_impl(adlbq_server *h, int n, const int *units9, int *out3, int *d_out3, int hold_rank = -1) {
    if (h) wq_changed(h);
    if (n == 0) return ADLBQ_OK;
    hipSetDevice(h->device);
    maybe_compact_rq(h);
    for (int i = 0; i < n; i++)
        if (type_index(h, units9[9 * i]) < 0) return fail(ADLBQ_ERR_TYPE, "adlbq_put_batch: undeclared work type");
    int rc;
    // records are staged in pinned memory, two buffers used in turn: the copy out of
    // this one (two batches ago) must have completed; so must the device record buffer's readers
    const int sb = h->put_slot;
    h->put_slot ^= 1;
    if (h->put_ev[sb]) AQ_HIP(hipEventSynchronize(h->put_ev[sb]));
    else AQ_HIP(hipEventCreateWithFlags(&h->put_ev[sb], hipEventDisableTiming));
    if (n > h->cap_put) {
        AQ_HIP(hipStreamSynchronize(h->stream));
        if (h->d_putrec) AQ_HIP(hipFree(h->d_putrec));
        if (h->d_putout) AQ_HIP(hipFree(h->d_putout));
        for (int q = 0; q < 2; q++)
            if (h->h_putrec[q]) AQ_HIP(hipHostFree(h->h_putrec[q]));
        h->cap_put = std::max({n, 2 * h->cap_put, 1 << 14});
        AQ_HIP(hipMalloc((void **)&h->d_putrec, sizeof(PutRec) * 2 * (size_t)h->cap_put));
        AQ_HIP(hipMalloc((void **)&h->d_putout, sizeof(int) * 3 * (size_t)h->cap_put));
        for (int q = 0; q < 2; q++)
            AQ_HIP(hipHostMalloc((void **)&h->h_putrec[q], sizeof(PutRec) * (size_t)h->cap_put, hipHostMallocDefault));
    }
    PutRec *rec = reinterpret_cast<PutRec *>(h->h_putrec[sb]);
    for (int i = 0; i < n; i++) {
        const int *u = units9 + 9 * i;
        int tgt = u[3];
        Bucket *b;
        int bk = -1;
        if (tgt < 0) {
            b = &h->open;
        } else {
            bk = rank_bucket(h, tgt);
            b = &h->rankb[bk];
        }
        if (b->pages.empty() || b->tail_fill == PAGE) {
            // the page's packed-offset base: its first prio less half the range
            const int pbase = (int)std::max((long long)u[1] - M_OFF_RANGE / 2, (long long)INT_MIN);
            if (!h->free_pages.empty()) {  // a recycled dead page (every slot is written before it is read)
                const int pg = h->free_pages.back();
                h->free_pages.pop_back();
                b->pages.push_back(pg);
                h->page_base[(size_t)pg] = pbase;
                h->page_wide[(size_t)pg] = 0;
            } else {
                if (h->n_pages == h->cap_pages && (rc = grow_pages(h, h->n_pages + 1))) return rc;
                b->pages.push_back(h->n_pages++);
                h->page_base.push_back(pbase);
                h->page_wide.push_back(0);
            }
            b->tail_fill = 0;
            h->pinfo_dirty = true;
        }
        h->tables_dirty = true;
        long long slot = ((long long)b->pages.back() << PAGE_SHIFT) + b->tail_fill++;
        int seq = h->next_wqseqno++;
        const int ti = type_index(h, u[0]);
        PutRec &r = rec[i];
        r.slot = (int)slot;
        r.prio = u[1];
        const bool vw = h->T > VW_TYPES;  // the offset field holds the type index's high bits
        r.meta = (int)meta_of_type(ti, vw) | (int)M_LIVE;
        {
            const int pg = b->pages.back();
            const long long off = (long long)u[1] - h->page_base[pg];
            if (!vw && off >= 0 && off < M_OFF_RANGE) r.meta |= (int)((unsigned int)off << M_OFF_SHIFT);
            else if (!h->page_wide[pg]) {
                h->page_wide[pg] = 1;
                h->pinfo_dirty = true;
            }
        }
        r.seq = seq;
        r.answer = u[2];
        r.len = u[4];
        r.home = u[5];
        r.clen = u[6];
        r.csrv = u[7];
        r.cseq = u[8];
        r.utype = u[0];
        r.target = tgt;
        if ((long long)h->seq2slot.size() <= seq) h->seq2slot.resize((size_t)seq * 2 + 16, -1);
        h->seq2slot[seq] = slot;
        h->live_units++;
        if (tgt >= 0) {
            h->live_targeted++;
            h->tindex_dirty = true;
            // the unit's targeted-index entry (k_tindex_keys' key): merged in at the next build
            const unsigned int inv = ~((unsigned int)u[1] ^ 0x80000000u);
            h->tnew_keys.push_back(((unsigned long long)bk << 38) | ((unsigned long long)ti << 32) | inv);
            h->tnew_vals.push_back((int)((b->pages.size() - 1) * PAGE + (b->tail_fill - 1)));
        }
        if (h->live_units > h->max_count) h->max_count = h->live_units;
    }
    if ((long long)h->next_wqseqno > h->cap_seq) {
        long long nc = std::max<long long>(h->next_wqseqno + 1024, h->cap_seq * 2);
        if ((rc = grow(&h->d_seq2slot, h->cap_seq, nc, h->stream, 0xff))) return rc;
        h->cap_seq = nc;
    }
    // only a possible rq match synchronises
    PutRec *d_rec = reinterpret_cast<PutRec *>(h->d_putrec) + (size_t)sb * h->cap_put;
    AQ_HIP(hipMemcpyAsync(d_rec, rec, sizeof(PutRec) * n, hipMemcpyHostToDevice, h->stream));
    // a parked Reserve can only exist if the last known count, plus every
    // Reserve launched since, is positive
    bool may_match = hold_rank < 0 &&
                     (h->put_always_match || (h->ctr_stale ? (rq_live_upper(h) > 0) : (h->ctr.rq_live > 0)));
    long long add_bytes = 0;  // bytes of the batch's units (k_put_match adds them one Put at a time)
    if (!may_match)
        for (int i = 0; i < n; i++) add_bytes += BYTES_WQ + rec[i].len;
    k_put_scatter<<<(n + 255) / 256, 256, 0, h->stream>>>(d_rec, n, h->d_prio, h->d_meta, h->d_pin, h->d_seq,
                                                          h->d_cold0, h->d_cold1, h->d_seq2slot, h->d_anchor,
                                                          h->d_rrec, h->d_ctr, add_bytes);
    if (hold_rank >= 0) k_push_hold<<<1, 1, 0, h->stream>>>(rec[0].slot, hold_rank, h->d_meta, h->d_pin);
    if (may_match) {
        // one workgroup over the staged rq; too many parked Reserves: the one-wave scan of the whole rq
        if (!h->d_pm_over) AQ_HIP(hipMalloc((void **)&h->d_pm_over, sizeof(int)));
        const bool blk = h->put_match_block && h->T <= ADLBQ_MAX_TYPES;  // its type sets are 64-bit masks
        AQ_HIP(hipMemsetAsync(h->d_pm_over, blk ? 0 : 1, sizeof(int), h->stream));
        if (blk)
            k_put_match_blk<<<1, PM_THREADS, 0, h->stream>>>(d_rec, n, h->d_rq_rank, h->d_rq_types, h->d_rq_live,
                                                         h->d_rq_seq, h->d_ctr, h->d_meta, h->d_pin,
                                                         d_out3 ? d_out3 : h->d_putout, h->d_utypes, h->T,
                                                         h->d_pm_over);
        k_put_match<<<1, 64, 0, h->stream>>>(d_rec, n, h->d_rq_rank, h->d_rq_types, h->d_rq_live, h->d_rq_seq, h->d_ctr,
                                             h->d_meta, h->d_pin, d_out3 ? d_out3 : h->d_putout, h->d_pm_over);
        AQ_HIP(hipGetLastError());
        AQ_HIP(hipEventRecord(h->put_ev[sb], h->stream));
        if (d_out3) {
            h->ctr_stale = true;
            return ADLBQ_OK;
        }
        AQ_HIP(hipMemcpyAsync(out3, h->d_putout, sizeof(int) * 3 * n, hipMemcpyDeviceToHost, h->stream));
        if ((rc = refresh_counters(h))) return rc;
    } else if (d_out3) {
        k_put_out<<<(n + 255) / 256, 256, 0, h->stream>>>(d_rec, n, d_out3);
        AQ_HIP(hipGetLastError());
        AQ_HIP(hipEventRecord(h->put_ev[sb], h->stream));
    } else {
        for (int i = 0; i < n; i++) {
            out3[3 * i] = rec[i].seq;
            out3[3 * i + 1] = -1;
            out3[3 * i + 2] = -1;
        }
        AQ_HIP(hipGetLastError());
        AQ_HIP(hipEventRecord(h->put_ev[sb], h->stream));
    }
    return ADLBQ_OK;
}

int adlbq_put_batch(adlbq_server *h, int n, const int *units9, int *out3) {
    if (!ok_handle(h) || n < 0 || (n && (!units9 || !out3))) return fail(ADLBQ_ERR_ARG, "adlbq_put_batch");
    return put_impl(h, n, units9, out3, nullptr);
}

int adlbq_put_batch_device(adlbq_server *h, int n, const int *units9, int *d_out3) {
    if (!ok_handle(h) || n < 0 || (n && (!units9 || !d_out3))) return fail(ADLBQ_ERR_ARG, "adlbq_put_batch_device");
    return put_impl(h, n, units9, nullptr, d_out3);
}

static int find_slot(adlbq_server *h, int seq, long long *slot) {
    if (seq <= 0 || seq >= (long long)h->seq2slot.size() || seq >= h->next_wqseqno) return 0;
    *slot = h->seq2slot[seq];
    return *slot >= 0;
}

int adlbq_get_reserved(adlbq_server *h, int rank, int wqseqno, int *out5) {
    if (h) wq_changed(h);
    if (!ok_handle(h) || !out5) return fail(ADLBQ_ERR_ARG, "adlbq_get_reserved");
    hipSetDevice(h->device);
    long long slot;
    out5[0] = -1;
    out5[1] = out5[2] = out5[3] = out5[4] = 0;
    if (!find_slot(h, wqseqno, &slot)) return ADLBQ_OK;
    int rc;
    if ((rc = ensure_zc(h, 6))) return rc;
    k_get<<<1, 1, 0, h->stream>>>((int)slot, rank, wqseqno, h->d_prio, h->d_meta, h->d_pin, h->d_seq, h->d_cold0,
                                  h->d_cold1, h->d_zc, h->d_ctr);  // the record straight into mapped memory
    AQ_HIP(hipStreamSynchronize(h->stream));
    memcpy(out5, h->h_zc, sizeof(int) * 5);
    if (out5[0] == 1) {
        h->seq2slot[wqseqno] = -1;
        h->live_units--;
        if (h->h_zc[5] >= 0) h->live_targeted--;
        // keep the device map consistent for batch unreserves
        AQ_HIP(hipMemsetAsync(h->d_seq2slot + wqseqno, 0xff, sizeof(long long), h->stream));
    }
    return ADLBQ_OK;
}

static int launch_get_batch(adlbq_server *h, int n, const int *d_pairs, int *d_out5) {
    if (h) wq_changed(h);
    if ((long long)h->next_wqseqno > h->cap_getclaim) {
        AQ_HIP(hipStreamSynchronize(h->stream));
        if (h->d_getclaim) AQ_HIP(hipFree(h->d_getclaim));
        h->cap_getclaim = std::max<long long>(h->cap_seq, h->next_wqseqno);
        AQ_HIP(hipMalloc((void **)&h->d_getclaim, sizeof(int) * h->cap_getclaim));
        AQ_HIP(hipMemsetAsync(h->d_getclaim, 0x7f, sizeof(int) * h->cap_getclaim, h->stream));  // "none"
    }
    const int g = (n + 255) / 256;
    k_get_claim<<<g, 256, 0, h->stream>>>(d_pairs, n, h->d_seq2slot, h->next_wqseqno, h->d_meta, h->d_pin, h->d_seq,
                                         h->d_getclaim);
    k_get_apply<<<g, 256, 0, h->stream>>>(d_pairs, n, h->d_seq2slot, h->next_wqseqno, h->d_meta, h->d_prio,
                                         h->d_cold0, h->d_cold1, h->d_getclaim, d_out5, h->d_ctr);
    AQ_HIP(hipGetLastError());
    h->ctr_stale = true;
    return ADLBQ_OK;
}

int adlbq_get_reserved_batch_device(adlbq_server *h, int n, const int *d_pairs2, int *d_out5) {
    if (!ok_handle(h) || n < 0 || (n && (!d_pairs2 || !d_out5)))
        return fail(ADLBQ_ERR_ARG, "adlbq_get_reserved_batch_device");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    return launch_get_batch(h, n, d_pairs2, d_out5);
}

int adlbq_get_reserved_batch(adlbq_server *h, int n, const int *pairs2, int *out5) {
    if (!ok_handle(h) || n < 0 || (n && (!pairs2 || !out5))) return fail(ADLBQ_ERR_ARG, "adlbq_get_reserved_batch");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    int rc0;
    // zero-copy: the pairs, the records and the counters go through mapped pinned
    // memory (no copies to stage for a few dozen Gets; the call is synchronous, so
    // the staging is free again when it returns)
    if ((rc0 = ensure_zc(h, (long long)n * 7)) || (rc0 = ensure_zctr(h))) return rc0;
    std::memcpy(h->h_zc, pairs2, sizeof(int) * 2 * (size_t)n);
    int rc;
    if (n <= 256 && (long long)h->next_wqseqno <= h->cap_getclaim) {  // one launch
        wq_changed(h);
        k_get_small<<<1, 256, 0, h->stream>>>(h->d_zc, n, h->d_seq2slot, h->next_wqseqno, h->d_meta,
                                              h->d_pin, h->d_seq, h->d_prio, h->d_cold0, h->d_cold1, h->d_getclaim,
                                              h->d_zc + 2 * (size_t)n, h->d_ctr, h->d_zctr);
        h->ctr_stale = true;
    } else {
        if ((rc = launch_get_batch(h, n, h->d_zc, h->d_zc + 2 * (size_t)n))) return rc;
        k_ctr_out<<<1, 1, 0, h->stream>>>(h->d_ctr, h->d_zctr);
    }
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipStreamSynchronize(h->stream));
    std::memcpy(out5, h->h_zc + 2 * (size_t)n, sizeof(int) * 5 * (size_t)n);
    h->ctr = *h->h_zctr;
    apply_counters(h);  // folds the removed units into the host counts
    for (int i = 0; i < n; i++)
        if (out5[5 * i] == 1) {
            const int seq = pairs2[2 * i + 1];
            if (seq > 0 && seq < (long long)h->seq2slot.size()) h->seq2slot[seq] = -1;
        }
    return ADLBQ_OK;
}

int adlbq_unreserve(adlbq_server *h, int rank, int wqseqno, int new_pin_rank, int *found) {
    if (h) wq_changed(h);
    if (!ok_handle(h) || !found) return fail(ADLBQ_ERR_ARG, "adlbq_unreserve");
    hipSetDevice(h->device);
    long long slot;
    *found = 0;
    if (!find_slot(h, wqseqno, &slot)) return ADLBQ_OK;
    int rc;
    if ((rc = ensure_zc(h, 1))) return rc;
    k_unreserve<<<1, 1, 0, h->stream>>>((int)slot, rank, wqseqno, new_pin_rank, h->d_meta, h->d_pin, h->d_seq,
                                        h->d_zc, h->d_prio, h->d_anchor);  // found straight into mapped memory
    AQ_HIP(hipStreamSynchronize(h->stream));
    *found = h->h_zc[0];
    return ADLBQ_OK;
}

}  // extern "C"
namespace adlbq {
int launch_unreserve_resp(adlbq_server *h, int n, const int *d_reqs18, const int *d_resp12, int trusted) {
    if (trusted) h->unres_trusted_calls++;
    k_unreserve_resp<<<(n + 255) / 256, 256, 0, h->stream>>>(d_reqs18, d_resp12, n, h->d_seq2slot, h->next_wqseqno,
                                                             h->d_meta, h->d_pin, h->d_rrec, h->d_anchor,
                                                             (h->d_mslot && n <= h->cap_req) ? h->d_mslot : nullptr,
                                                             std::min(h->T, 64), unres_rh(h, d_reqs18, n), trusted);
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}
}  // namespace adlbq
extern "C" {

int adlbq_unreserve_resp_device(adlbq_server *h, int n, const int *d_reqs18, const int *d_resp12) {
    const int trusted = (h && ok_handle(h) && n > 0) ? unres_trusted(h, d_reqs18, n) : 0;
    if (h) wq_changed(h);
    if (!ok_handle(h) || n < 0 || (n && (!d_reqs18 || !d_resp12)))
        return fail(ADLBQ_ERR_ARG, "adlbq_unreserve_resp_device");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    return launch_unreserve_resp(h, n, d_reqs18, d_resp12, trusted);
}

int adlbq_unreserve_resp_group_device(adlbq_server *const *hs, int n, const int *const *d_reqs18,
                                      const int *const *d_resp12, const int *counts) {
    if (n < 0 || (n && (!hs || !d_reqs18 || !d_resp12 || !counts)))
        return fail(ADLBQ_ERR_ARG, "adlbq_unreserve_resp_group_device");
    std::vector<int> m, trust(n > 0 ? n : 0);
    for (int i = 0; i < n; i++) {
        if (!ok_handle(hs[i]) || counts[i] < 0 || (counts[i] && (!d_reqs18[i] || !d_resp12[i])) ||
            hs[i]->device != hs[0]->device)
            return fail(ADLBQ_ERR_ARG, "adlbq_unreserve_resp_group_device: bad handle, count or pointer, or mixed devices");
        for (int j = 0; j < i; j++)
            if (hs[j] == hs[i]) return fail(ADLBQ_ERR_ARG, "adlbq_unreserve_resp_group_device: a handle appears twice");
        trust[i] = counts[i] > 0 ? unres_trusted(hs[i], d_reqs18[i], counts[i]) : 0;
        wq_changed(hs[i]);
        if (counts[i] > 0) m.push_back(i);
    }
    if (m.empty()) return ADLBQ_OK;
    hipSetDevice(hs[0]->device);
    int rc;
    for (size_t c0 = 0; c0 < m.size(); c0 += UNRES_GROUP) {  // UNRES_GROUP shards per launch (kernel arguments)
        const std::vector<int> mm(m.begin() + c0, m.begin() + std::min(m.size(), c0 + UNRES_GROUP));
        UnresGroup g{};
        int nb = 0;
        for (size_t j = 0; j < mm.size(); j++) {
            adlbq_server *h = hs[mm[j]];
            const int c = counts[mm[j]];
            g.a[j] = UnresArgs{d_reqs18[mm[j]], d_resp12[mm[j]], c, h->d_seq2slot, h->next_wqseqno, h->d_meta, h->d_pin,
                               h->d_rrec, h->d_anchor, (h->d_mslot && c <= h->cap_req) ? h->d_mslot : nullptr,
                               std::min(h->T, 64), unres_rh(h, d_reqs18[mm[j]], c), trust[mm[j]]};
            nb = std::max(nb, (c + 255) / 256);
        }
        adlbq_server *L = hs[mm[0]];
        if ((rc = group_join(hs, mm))) return rc;
        k_unreserve_resp_g<<<dim3(nb, (unsigned)mm.size()), 256, 0, L->stream>>>(g);
        AQ_HIP(hipGetLastError());
        if ((rc = group_release(hs, mm))) return rc;
    }
    return ADLBQ_OK;
}

int adlbq_unreserve_batch_device(adlbq_server *h, int n, const int *d_triples) {
    if (h) wq_changed(h);
    if (!ok_handle(h) || n < 0) return fail(ADLBQ_ERR_ARG, "adlbq_unreserve_batch_device");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    k_unreserve_batch<<<(n + 255) / 256, 256, 0, h->stream>>>(d_triples, n, h->d_seq2slot, h->next_wqseqno,
                                                              h->d_meta, h->d_pin, h->d_rrec, h->d_anchor);
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

int adlbq_qmstat_row(adlbq_server *h, int *qlen, int *type_hi_prio) {
    if (!ok_handle(h) || !qlen || (h->T && !type_hi_prio)) return fail(ADLBQ_ERR_ARG, "adlbq_qmstat_row");
    hipSetDevice(h->device);
    int rc;
    if ((rc = sync_tables(h))) return rc;
    std::vector<int> init(1 + h->T, LOWEST);
    init[0] = 0;
    AQ_HIP(hipMemcpyAsync(h->d_result, init.data(), sizeof(int) * (1 + h->T), hipMemcpyHostToDevice, h->stream));
    int np = (int)h->open.pages.size();
    if (np) {
        int blocks = std::min(2048, np * (PAGE / 256));
        k_qmrow<<<blocks, 256, 0, h->stream>>>(h->d_open_pages, np, h->open.tail_fill, h->d_prio, h->d_meta, h->T,
                                               h->d_result);
    }
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int) * (1 + h->T), hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    *qlen = h->h_result[0];
    for (int t = 0; t < h->T; t++) type_hi_prio[t] = h->h_result[1 + t];
    // this server's own qmstat row (adlb.c:3586-3591), nbytes_used included
    h->ctr_stale = true;
    if ((rc = refresh_counters(h))) return rc;
    h->qm_bytes[h->my_idx] = (double)h->ctr.bytes;
    h->qm_qlen[h->my_idx] = *qlen;
    for (int t = 0; t < h->T; t++) h->qm_hi[(size_t)h->my_idx * h->T + t] = type_hi_prio[t];
    h->qm_dirty = true;
    return ADLBQ_OK;
}

int adlbq_set_qmstat_row(adlbq_server *h, int server_idx, int qlen, double nbytes_used, const int *type_hi_prio) {
    if (!ok_handle(h) || server_idx < 0 || server_idx >= h->S || (h->T && !type_hi_prio))
        return fail(ADLBQ_ERR_ARG, "adlbq_set_qmstat_row");
    if (server_idx == h->my_idx) return ADLBQ_OK;  // the local row survives the unpack (adlb.c:1724-1728)
    h->qm_qlen[server_idx] = qlen;
    h->qm_bytes[server_idx] = nbytes_used;
    for (int t = 0; t < h->T; t++) h->qm_hi[(size_t)server_idx * h->T + t] = type_hi_prio[t];
    h->qm_dirty = true;
    return ADLBQ_OK;
}

int adlbq_set_qmstat_nbytes(adlbq_server *h, int server_idx, double nbytes_used) {
    if (!ok_handle(h) || server_idx < 0 || server_idx >= h->S) return fail(ADLBQ_ERR_ARG, "adlbq_set_qmstat_nbytes");
    h->qm_bytes[server_idx] = nbytes_used;
    h->qm_dirty = true;
    return ADLBQ_OK;
}

int adlbq_check_remote(adlbq_server *h, int cap, int *out3, int *count) {
    if (!ok_handle(h) || cap < 0 || !count || (cap && !out3)) return fail(ADLBQ_ERR_ARG, "adlbq_check_remote");
    hipSetDevice(h->device);
    int rc;
    if ((rc = sync_tables(h))) return rc;
    if (h->ctr_stale && (rc = refresh_counters(h))) return rc;
    const int nrq = h->ctr.rq_n;
    const int capd = std::max(1, std::min(cap, nrq));
    // persistent device buffer and pinned staging (no allocation, one synchronisation)
    if (3ll * capd + 1 > h->cap_crem) {
        if (h->d_crem) AQ_HIP(hipFree(h->d_crem));
        if (h->h_crem) AQ_HIP(hipHostFree(h->h_crem));
        h->cap_crem = std::max(3ll * capd + 1, 2 * h->cap_crem);
        AQ_HIP(hipMalloc((void **)&h->d_crem, sizeof(int) * h->cap_crem));
        AQ_HIP(hipHostMalloc((void **)&h->h_crem, sizeof(int) * h->cap_crem, hipHostMallocDefault));
    }
    k_checkrem<<<1, 64, 0, h->stream>>>(donor_ctx(h), h->d_rq_rank, h->d_rq_types, h->d_rq_live, h->d_rq_seq, h->d_ctr, capd,
                                        h->d_crem + 1, h->d_crem);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipMemcpyAsync(h->h_crem, h->d_crem, sizeof(int) * (3 * (size_t)capd + 1), hipMemcpyDeviceToHost,
                          h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    const int kk = std::min(h->h_crem[0], cap);
    if (kk) memcpy(out3, h->h_crem + 1, sizeof(int) * 3 * (size_t)kk);
    *count = kk;
    return ADLBQ_OK;
}

int adlbq_rfr_done(adlbq_server *h, int from_server_rank, int for_rank) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_rfr_done");
    hipSetDevice(h->device);
    if (for_rank >= 0 && for_rank < h->A) k_set_int<<<1, 1, 0, h->stream>>>(h->d_rfr_to_rank + for_rank, -1);
    if (from_server_rank >= 0 && from_server_rank < h->num_world)
        k_set_int<<<1, 1, 0, h->stream>>>(h->d_rfr_out + from_server_rank, 0);
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

// adlbq_rfr_done for up to RFR_BATCH pairs, in order, by one thread
constexpr int RFR_BATCH = 32;
struct RfrPairs {
    int n;
    int v[2 * RFR_BATCH];
};
__global__ void k_rfr_done_batch(RfrPairs p, int *rfr_to_rank, int A, int *rfr_out, int nworld) {
    for (int k = 0; k < p.n; k++) {
        const int srv = p.v[2 * k], rank = p.v[2 * k + 1];
        if (rank >= 0 && rank < A) rfr_to_rank[rank] = -1;
        if (srv >= 0 && srv < nworld) rfr_out[srv] = 0;
    }
}

int adlbq_rfr_done_batch(adlbq_server *h, int n, const int *pairs) {
    if (!ok_handle(h) || n < 0 || (n && !pairs)) return fail(ADLBQ_ERR_ARG, "adlbq_rfr_done_batch");
    hipSetDevice(h->device);
    for (int k0 = 0; k0 < n; k0 += RFR_BATCH) {
        RfrPairs p{};
        p.n = std::min(RFR_BATCH, n - k0);
        memcpy(p.v, pairs + 2 * k0, sizeof(int) * 2 * p.n);
        k_rfr_done_batch<<<1, 1, 0, h->stream>>>(p, h->d_rfr_to_rank, h->A, h->d_rfr_out, h->num_world);
    }
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

int adlbq_tq_add(adlbq_server *h, int app_rank, int work_type, int server_rank) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_tq_add");
    for (size_t i = 0; i + 3 < h->tq.size(); i += 4)
        if (h->tq[i] == app_rank && h->tq[i + 1] == work_type && h->tq[i + 2] == server_rank) {
            h->tq[i + 3]++;
            h->tq_dirty = true;
            return ADLBQ_OK;
        }
    h->tq.insert(h->tq.end(), {app_rank, work_type, server_rank, 1});
    h->tq_dirty = true;
    hipSetDevice(h->device);
    k_add_bytes<<<1, 1, 0, h->stream>>>(h->d_ctr, BYTES_TQ);  // tq_node_create (adlb.c:1176)
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

int adlbq_tq_dec(adlbq_server *h, int app_rank, int work_type, int server_rank) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_tq_dec");
    for (size_t i = 0; i + 3 < h->tq.size(); i += 4)
        if (h->tq[i] == app_rank && h->tq[i + 1] == work_type && h->tq[i + 2] == server_rank) {
            if (--h->tq[i + 3] <= 0) {  // tq_delete (adlb.c:1942-1945, 2081-2083)
                h->tq.erase(h->tq.begin() + (long)i, h->tq.begin() + (long)i + 4);
                hipSetDevice(h->device);
                k_add_bytes<<<1, 1, 0, h->stream>>>(h->d_ctr, -BYTES_TQ);
                AQ_HIP(hipGetLastError());
            }
            h->tq_dirty = true;
            return ADLBQ_OK;
        }
    return ADLBQ_OK;
}

int adlbq_rfr_failed(adlbq_server *h, int donor_rank, int for_rank, const int *types16) {
    if (!ok_handle(h) || !types16) return fail(ADLBQ_ERR_ARG, "adlbq_rfr_failed");
    const int idx = donor_rank - h->master;
    if (idx < 0 || idx >= h->S) return fail(ADLBQ_ERR_ARG, "adlbq_rfr_failed: donor is not a server rank");
    // a wildcard first entry stands for every declared type (adlb.c:1973-1978)
    std::vector<int> list;
    if (types16[0] < 0) list.assign(h->utypes.begin(), h->utypes.end());
    else
        for (int i = 0; i < NREQ && types16[i] >= 0; i++) list.push_back(types16[i]);
    for (int v : list) {
        int t = -1;
        for (int j = 0; j < h->T; j++)
            if (h->utypes[j] == v) t = j;
        if (t < 0) continue;  // the reference prints "invalid type" and indexes out of bounds
        h->qm_hi[(size_t)idx * h->T + t] = LOWEST;
        h->qm_dirty = true;
        // every tq record of (for_rank, donor, type) loses one unit (adlb.c:1988-2004)
        for (size_t i = 0; i + 3 < h->tq.size();) {
            if (h->tq[i] == for_rank && h->tq[i + 2] == donor_rank && h->tq[i + 1] == v && --h->tq[i + 3] <= 0) {
                h->tq.erase(h->tq.begin() + (long)i, h->tq.begin() + (long)i + 4);
                hipSetDevice(h->device);
                k_add_bytes<<<1, 1, 0, h->stream>>>(h->d_ctr, -BYTES_TQ);
                AQ_HIP(hipGetLastError());
                h->tq_dirty = true;
                continue;
            }
            if (h->tq[i] == for_rank && h->tq[i + 2] == donor_rank && h->tq[i + 1] == v) h->tq_dirty = true;
            i += 4;
        }
    }
    return ADLBQ_OK;
}

int adlbq_rfr_retry(adlbq_server *h, int rqseqno, int *found, int *donor_rank) {
    if (!ok_handle(h) || !found || !donor_rank) return fail(ADLBQ_ERR_ARG, "adlbq_rfr_retry");
    hipSetDevice(h->device);
    int rc;
    if ((rc = sync_tables(h))) return rc;
    k_rfr_retry<<<1, 64, 0, h->stream>>>(donor_ctx(h), h->d_rq_rank, h->d_rq_types, h->d_rq_live, h->d_rq_seq,
                                         h->d_ctr, rqseqno, h->d_result);
    AQ_HIP(hipGetLastError());
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int) * 2, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    *found = h->h_result[0];
    *donor_rank = h->h_result[1];
    return ADLBQ_OK;
}

int adlbq_unit_target(adlbq_server *h, int wqseqno, int *target_rank) {
    if (!ok_handle(h) || !target_rank) return fail(ADLBQ_ERR_ARG, "adlbq_unit_target");
    long long slot;
    *target_rank = -1;
    if (!find_slot(h, wqseqno, &slot)) return fail(ADLBQ_ERR_ARG, "adlbq_unit_target: no such unit");
    hipSetDevice(h->device);
    const char *p = reinterpret_cast<const char *>(h->d_cold1 + slot) + 3 * sizeof(int);  // cold1.w
    AQ_HIP(hipMemcpyAsync(h->h_result, p, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    *target_rank = h->h_result[0];
    return ADLBQ_OK;
}

int adlbq_bytes(adlbq_server *h, double *curr, double *hwm) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_bytes");
    hipSetDevice(h->device);
    int rc;
    h->ctr_stale = true;
    if ((rc = refresh_counters(h))) return rc;
    if (curr) *curr = (double)h->ctr.bytes;
    if (hwm) *hwm = (double)h->ctr.bytes_hwm;
    return ADLBQ_OK;
}

int adlbq_bytes_adjust(adlbq_server *h, double delta) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_bytes_adjust");
    if (delta == 0) return ADLBQ_OK;
    hipSetDevice(h->device);
    k_add_bytes<<<1, 1, 0, h->stream>>>(h->d_ctr, (long long)delta);
    AQ_HIP(hipGetLastError());
    h->ctr_stale = true;
    return ADLBQ_OK;
}

// argmin nbytes_used over the other servers below THRESHOLD_TO_START_PUSH
// (strict <, lowest index wins): adlb.c:912-928, 516-528
static int reject_hint(const adlbq_server *h, double threshold) {
    double smallest = 999999999999.9;
    int cand = -1;
    for (int i = 0; i < h->S; i++) {
        const int srv = h->master + i;
        if (srv != h->my_world && h->qm_bytes[i] < threshold && h->qm_bytes[i] < smallest) {
            smallest = h->qm_bytes[i];
            cand = srv;
        }
    }
    return cand;
}

int adlbq_put_check(adlbq_server *h, int work_len, double max_malloc, int *rejected, int *hint_server_rank) {
    if (!ok_handle(h) || !rejected || !hint_server_rank) return fail(ADLBQ_ERR_ARG, "adlbq_put_check");
    double curr = 0;
    int rc;
    if ((rc = adlbq_bytes(h, &curr, nullptr))) return rc;
    *rejected = (curr + work_len) > max_malloc ? 1 : 0;
    *hint_server_rank = *rejected ? reject_hint(h, 0.95 * max_malloc) : -1;
    return ADLBQ_OK;
}

int adlbq_rq_delete(adlbq_server *h, int rqseqno, int *found) {
    if (!ok_handle(h) || !found) return fail(ADLBQ_ERR_ARG, "adlbq_rq_delete");
    hipSetDevice(h->device);
    k_rq_delete<<<1, 1, 0, h->stream>>>(rqseqno, h->d_rq_seq, h->d_rq_live, h->d_ctr, h->d_result);
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    *found = h->h_result[0];
    h->ctr_stale = true;
    return refresh_counters(h);
}

int adlbq_push_select(adlbq_server *h, double threshold, int *cand_server_rank, int *wqseqno) {
    if (!ok_handle(h) || !cand_server_rank || !wqseqno) return fail(ADLBQ_ERR_ARG, "adlbq_push_select");
    hipSetDevice(h->device);
    int rc;
    if ((rc = sync_tables(h))) return rc;
    *cand_server_rank = -1;
    *wqseqno = -1;
    int npages = (int)(h->open.pages.size());
    for (auto &b : h->rankb) npages += (int)b.pages.size();
    h->h_result[0] = INT_MAX;
    AQ_HIP(hipMemcpyAsync(h->d_result, h->h_result, sizeof(int), hipMemcpyHostToDevice, h->stream));
    if (npages)
        k_first_unpinned<<<npages, 256, 0, h->stream>>>(h->d_all_pages, h->d_all_fill, npages, h->d_meta, h->d_seq,
                                                        h->d_result);
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    if (h->h_result[0] == INT_MAX) return ADLBQ_OK;
    *cand_server_rank = reject_hint(h, threshold);  // argmin nbytes_used (adlb.c:516-528)
    *wqseqno = h->h_result[0];
    return ADLBQ_OK;
}

int adlbq_push_accept(adlbq_server *h, const int *units9, int *wqseqno) {
    if (!ok_handle(h) || !units9 || !wqseqno) return fail(ADLBQ_ERR_ARG, "adlbq_push_accept");
    int out3[3];
    int rc = put_impl(h, 1, units9, out3, nullptr, h->my_world);  // held for this server (adlb.c:2151, 2158)
    if (rc) return rc;
    *wqseqno = out3[0];
    return ADLBQ_OK;
}

// a unit left the store on the device: the host's maps and counts follow
static int unit_removed(adlbq_server *h, int seq, int target) {
    h->seq2slot[seq] = -1;
    h->live_units--;
    if (target >= 0) h->live_targeted--;
    AQ_HIP(hipMemsetAsync(h->d_seq2slot + seq, 0xff, sizeof(long long), h->stream));
    return ADLBQ_OK;
}

int adlbq_push_take(adlbq_server *h, int wqseqno, int *out10) {
    if (h) wq_changed(h);
    if (!ok_handle(h) || !out10) return fail(ADLBQ_ERR_ARG, "adlbq_push_take");
    hipSetDevice(h->device);
    long long slot;
    memset(out10, 0, sizeof(int) * 10);
    if (!find_slot(h, wqseqno, &slot)) return ADLBQ_OK;
    k_push_take<<<1, 1, 0, h->stream>>>((int)slot, wqseqno, h->d_prio, h->d_meta, h->d_seq, h->d_cold0, h->d_cold1,
                                        h->d_result, h->d_ctr);
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int) * 10, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    if (h->h_result[0] != 1) return ADLBQ_OK;  // out10 stays zero
    memcpy(out10, h->h_result, sizeof(int) * 10);
    return unit_removed(h, wqseqno, out10[5]);
}

int adlbq_push_commit(adlbq_server *h, int wqseqno, int *out3) {
    if (h) wq_changed(h);
    if (!ok_handle(h) || !out3) return fail(ADLBQ_ERR_ARG, "adlbq_push_commit");
    hipSetDevice(h->device);
    long long slot;
    out3[0] = 0;
    out3[1] = out3[2] = -1;
    if (!find_slot(h, wqseqno, &slot)) return ADLBQ_OK;
    int rc;
    if ((rc = sync_tables(h))) return rc;
    k_push_commit<<<1, 64, 0, h->stream>>>((int)slot, wqseqno, h->d_prio, h->d_meta, h->d_pin, h->d_seq, h->d_cold1,
                                           h->d_rq_rank, h->d_rq_types, h->d_rq_live, h->d_rq_seq, h->d_ctr,
                                           h->d_anchor, h->d_result);
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int) * 3, hipMemcpyDeviceToHost, h->stream));
    if ((rc = refresh_counters(h))) return rc;  // synchronises; the rq counts follow the device
    memcpy(out3, h->h_result, sizeof(int) * 3);
    return ADLBQ_OK;
}

int adlbq_push_discard(adlbq_server *h, int wqseqno, int *found) {
    if (h) wq_changed(h);
    if (!ok_handle(h) || !found) return fail(ADLBQ_ERR_ARG, "adlbq_push_discard");
    hipSetDevice(h->device);
    long long slot;
    *found = 0;
    if (!find_slot(h, wqseqno, &slot)) return ADLBQ_OK;
    k_push_discard<<<1, 1, 0, h->stream>>>((int)slot, wqseqno, h->d_meta, h->d_seq, h->d_cold0, h->d_cold1,
                                           h->d_result, h->d_ctr);
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int) * 2, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    *found = h->h_result[0];
    if (*found) return unit_removed(h, wqseqno, h->h_result[1]);
    return ADLBQ_OK;
}

int adlbq_info(adlbq_server *h, int *wq_count, int *wq_max_count, int *rq_count) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_info");
    hipSetDevice(h->device);
    int rc;
    if (h->ctr_stale && (rc = refresh_counters(h))) return rc;
    if (wq_count) *wq_count = (int)h->live_units;
    if (wq_max_count) *wq_max_count = (int)h->max_count;
    if (rq_count) *rq_count = h->ctr.rq_live;
    return ADLBQ_OK;
}

int adlbq_info_type(adlbq_server *h, int work_type, int *max_prio, int *num_max_prio, int *num_type) {
    if (!ok_handle(h) || !max_prio || !num_max_prio || !num_type) return fail(ADLBQ_ERR_ARG, "adlbq_info_type");
    auto it = h->tindex.find(work_type);
    if (it == h->tindex.end()) return fail(ADLBQ_ERR_TYPE, "adlbq_info_type: undeclared type");
    hipSetDevice(h->device);
    int rc;
    if ((rc = sync_tables(h))) return rc;
    int npages = (int)(h->open.pages.size());
    for (auto &b : h->rankb) npages += (int)b.pages.size();
    constexpr int IB = 1024;  // blocks of the fused reduction
    if (!h->d_info) {
        AQ_HIP(hipMalloc((void **)&h->d_info, sizeof(int) * (3 * IB + 1)));
        AQ_HIP(hipMemsetAsync(h->d_info, 0, sizeof(int) * (3 * IB + 1), h->stream));
    }
    if (npages) {
        k_info_fused<<<std::min(npages, IB), 256, 0, h->stream>>>(h->d_all_pages, h->d_all_fill, npages, h->d_prio,
                                                                  h->d_meta, it->second, h->T > VW_TYPES ? 1 : 0,
                                                                  h->d_info, h->d_result);
    } else {
        int init[3] = {LOWEST, 0, 0};
        AQ_HIP(hipMemcpyAsync(h->d_result, init, sizeof(init), hipMemcpyHostToDevice, h->stream));
    }
    AQ_HIP(hipMemcpyAsync(h->h_result, h->d_result, sizeof(int) * 3, hipMemcpyDeviceToHost, h->stream));
    AQ_HIP(hipStreamSynchronize(h->stream));
    *max_prio = h->h_result[0];
    *num_max_prio = h->h_result[1];
    *num_type = h->h_result[2];
    return ADLBQ_OK;
}

int adlbq_set_stream(adlbq_server *h, void *s) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_set_stream");
    hipStreamSynchronize(h->stream);
    h->stream = s ? (hipStream_t)s : h->own_stream;
    return ADLBQ_OK;
}

void *adlbq_get_stream(adlbq_server *h) { return h ? (void *)h->stream : nullptr; }

int adlbq_sync(adlbq_server *h) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_sync");
    hipSetDevice(h->device);
    AQ_HIP(hipStreamSynchronize(h->stream));
    return ADLBQ_OK;
}

int adlbq_profile_enable(adlbq_server *h, int on) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_profile_enable");
    h->profiling = on != 0;
    h->profile_only.clear();
    return ADLBQ_OK;
}

int adlbq_profile_only(adlbq_server *h, const char *stage) {
    if (!ok_handle(h)) return fail(ADLBQ_ERR_ARG, "adlbq_profile_only");
    h->profiling = true;
    h->profile_only = stage ? stage : "";
    return ADLBQ_OK;
}

int adlbq_profile_read(adlbq_server *h, const char *stage, double *total_ms, long long *launches) {
    if (!ok_handle(h) || !stage) return fail(ADLBQ_ERR_ARG, "adlbq_profile_read");
    hipSetDevice(h->device);
    AQ_HIP(hipStreamSynchronize(h->stream));
    auto &t = h->timers[stage];
    for (auto &pe : t.pending) {
        float ms = 0;
        hipEventElapsedTime(&ms, pe.first, pe.second);
        t.total_ms += ms;
        t.launches++;
        h->event_pool.push_back(pe.first);
        h->event_pool.push_back(pe.second);
    }
    t.pending.clear();
    if (total_ms) *total_ms = t.total_ms;
    if (launches) *launches = t.launches;
    return ADLBQ_OK;
}

long long adlbq_last_scan_units(adlbq_server *h) { return h ? h->last_scan_units : 0; }

int adlbq_set_param(adlbq_server *h, const char *name, long long value) {
    if (!h || !name) return fail(ADLBQ_ERR_ARG, "adlbq_set_param");
    std::string n(name);
    if (n == "chain_passes") {
        if (value < 0 || value > 8) return fail(ADLBQ_ERR_ARG, "chain_passes must be in [0, 8] (0 = auto)");
        h->chain_passes = (int)value;
        return ADLBQ_OK;
    }
    if (n == "profile_every") {
        h->profile_every = (int)std::max(1ll, value);
        return ADLBQ_OK;
    }
    if (n == "tindex_delta") {  // delta index capacity (0: merge every Put batch into the main index)
        if (value < 0 || value > (1ll << 26)) return fail(ADLBQ_ERR_ARG, "adlbq_set_param: tindex_delta");
        h->tdel_max = value;
        return ADLBQ_OK;
    }
    if (n == "split_prep") {
        h->split_prep = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "rank_in_select") {
        h->rank_in_select = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "put_match_block") {  // diagnostic: 0 = always the one-wave rq scan
        h->put_match_block = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "put_always_match") {  // diagnostic: run the put-side match even when rq is known empty
        h->put_always_match = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "kernel_stamps") {
        h->kstamps = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "chain_stamps") {
        h->chain_stamps = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "sort_fail_test") {  // test: every batch's candidate sort wait reports giving up
        h->sort_fail_test = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "rq_next") {  // test: the next rqseqno less one (only while nothing is parked)
        int rc;
        if ((rc = refresh_counters(h))) return rc;
        if (h->ctr.rq_live != 0 || value < h->ctr.rq_next || value > INT_MAX)
            return fail(ADLBQ_ERR_ARG, "rq_next: only forward, and only with no Reserve parked");
        k_set_rq_next<<<1, 1, 0, h->stream>>>(h->d_ctr, (int)value);
        AQ_HIP(hipGetLastError());
        return refresh_counters(h);
    }
    if (n == "chain_rounds") {
        if (value < -1 || value > 30) return fail(ADLBQ_ERR_ARG, "chain_rounds must be in [-1, 30] (-1 = auto)");
        h->chain_rounds = (int)value;
        return ADLBQ_OK;
    }
    if (n == "chain_warm") {
        if (value != -1 && (value < 0 || value > CHAIN_WARM || value % SEG != 0))
            return fail(ADLBQ_ERR_ARG, "chain_warm must be -1 (auto) or a multiple of the segment up to CHAIN_WARM");
        h->chain_warm = (int)value;
        return ADLBQ_OK;
    }
    if (n == "chain_modes") {
        h->chain_modes = value;
        return ADLBQ_OK;
    }
    if (n == "rq_wait_sync") {  // 1: rq backpressure synchronises the stream (the round-3 form)
        h->rq_wait_sync = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "targeted_diag") {
        h->targeted_diag = (int)value;
        return ADLBQ_OK;
    }
    if (n == "keyrank") {
        if (value != 0 && value != 1) return fail(ADLBQ_ERR_ARG, "keyrank must be 0 or 1");
        h->keyrank = (int)value;
        return ADLBQ_OK;
    }
    if (n == "keyrank_bin_max") {
        if (value < 0 || value > (1 << 24)) return fail(ADLBQ_ERR_ARG, "keyrank_bin_max out of range");
        h->kr_bin_max = (int)value;
        return ADLBQ_OK;
    }
    if (n == "fin_flat") {
        if (value < 0 || value > (1 << 20)) return fail(ADLBQ_ERR_ARG, "fin_flat out of range");
        h->fin_flat = (int)value;
        return ADLBQ_OK;
    }
    if (n == "group_launch") {
        if (value < 0 || value > 1) return fail(ADLBQ_ERR_ARG, "group_launch must be 0 or 1");
        h->group_launch = (int)value;
        return ADLBQ_OK;
    }
    if (n == "reserve_one") {
        h->reserve_one = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "select_wave") {
        h->select_wave = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "recycle_pages") {
        h->recycle_pages = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "targeted_scan") {
        if (value < -1 || value > 1) return fail(ADLBQ_ERR_ARG, "targeted_scan must be -1, 0 or 1");
        h->targeted_scan = (int)value;
        return ADLBQ_OK;
    }
    if (n == "fin_snap_diag") {
        h->fin_snap_diag = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "one_grid") {
        if (value < 0 || value > (1 << 20)) return fail(ADLBQ_ERR_ARG, "one_grid must be in [0, 2^20]");
        h->one_grid = (int)value;
        return ADLBQ_OK;
    }
    if (n == "unres_trust") {
        h->unres_trust = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "fuse_rank_chain") {
        h->fuse_rank_chain = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "bound_inject") {
        h->bound_inject = value ? 1 : 0;
        return ADLBQ_OK;
    }
    if (n == "small_pages") {  // the one-workgroup choice: largest open bucket (pages), 0 = off
        if (value < 0 || value > 4) return fail(ADLBQ_ERR_ARG, "small_pages must be in [0, 4]");
        h->small_pages = (int)value;
        return ADLBQ_OK;
    }
    if (n == "small_r") {  // ... and largest batch
        if (value < 0 || value > 1024) return fail(ADLBQ_ERR_ARG, "small_r must be in [0, 1024]");
        h->small_r = (int)value;
        return ADLBQ_OK;
    }
    if (n == "rank_grid") {  // test: k_rank's grid (0: sized by the rank hint)
        if (value < 0 || value > 4096) return fail(ADLBQ_ERR_ARG, "rank_grid must be in [0, 4096]");
        h->rank_grid = (int)value;
        return ADLBQ_OK;
    }
    return fail(ADLBQ_ERR_ARG, "adlbq_set_param: unknown parameter");
}

long long adlbq_stat(adlbq_server *h, const char *name) {
    if (!h || !name) return -1;
    hipSetDevice(h->device);
    std::string n(name);
    // host-side section timers need no device counters: no launch, no synchronisation
    const bool host_only = n.rfind("hacc:", 0) == 0 || n.rfind("host_ns:", 0) == 0 || n == "master";
    if (!host_only && refresh_counters(h)) return -1;
    if (n.rfind("kst_", 0) == 0 && h->d_kst && h->n_kst > 0) {
        // diagnostic: "kst_{hist,sel}_{1,2,3}" = median over workgroups of (stamp K - stamp 0) in ns,
        // "kst_{hist,sel}_start" = the spread of the start stamps, "kst_{hist,sel}_span" = first start to last end
        const int which = n.compare(4, 4, "hist") == 0 ? 0 : 1;
        const std::string what = n.substr(which == 0 ? 9 : 8);
        std::vector<unsigned long long> st(4 * (size_t)h->n_kst);
        if (hipMemcpy(st.data(), h->d_kst + (size_t)which * 4 * h->n_kst, sizeof(unsigned long long) * st.size(),
                      hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        unsigned long long s0 = ~0ull, s1 = 0, e1 = 0;
        std::vector<long long> d;
        const int k = (what.size() == 1) ? what[0] - '0' : 0;
        for (int i = 0; i < h->n_kst; i++) {
            const unsigned long long *r = &st[4 * (size_t)i];
            s0 = std::min(s0, r[0]);
            s1 = std::max(s1, r[0]);
            e1 = std::max(e1, r[3]);
            if (k >= 1 && k <= 3 && r[k] >= r[0]) d.push_back((long long)(r[k] - r[0]) * 10);
        }
        if (what == "start") return (long long)(s1 - s0) * 10;
        if (what.rfind("startp", 0) == 0 || what.rfind("endp", 0) == 0) {  // percentile of the starts / ends
            const bool st0 = what[0] == 's';
            const int pc = std::atoi(what.c_str() + (st0 ? 6 : 4));
            std::vector<long long> v;
            for (int i = 0; i < h->n_kst; i++) v.push_back((long long)(st[4 * (size_t)i + (st0 ? 0 : 3)] - s0) * 10);
            std::sort(v.begin(), v.end());
            return v[std::min(v.size() - 1, v.size() * (size_t)pc / 100)];
        }
        if (what == "span") return (long long)(e1 - s0) * 10;
        if (d.empty()) return -1;
        std::sort(d.begin(), d.end());
        return d[d.size() / 2];
    }
    if (n == "small_batches") return h->small_batches;
    if (n == "pages_recycled") return h->pages_recycled;
    if (n == "rq_compactions") return h->rq_compactions;
    if (n.rfind("diag", 0) == 0 && n.size() == 5 && n[4] >= '0' && n[4] <= '7') {
        h->ctr_stale = true;
        int rc;
        if ((rc = refresh_counters(h))) return rc;
        return h->ctr.diag[n[4] - '0'];
    }
    if (n == "open_pages") return (long long)h->open.pages.size();
    if (n == "pages_total") return h->n_pages;
    if (n == "chain_rounds") return h->ctr.chain_rounds;
    if (n == "chain_passes") return h->ctr.chain_passes;
    if (n == "chain_recomputed") return h->ctr.chain_recomputed;
    if (n == "chain_fallback") return h->ctr.chain_fallback;
    if (n == "chain_timeouts") return h->ctr.chain_timeouts;
    if ((n == "chain_start_spread" || n == "chain_end_abs") && h->d_stamps && h->n_stamps > 0) {
        // diagnostic, ns: the spread of the segments' first stamps, and the latest stamp of any
        // segment after the earliest first stamp
        std::vector<unsigned long long> st(8 * (size_t)h->n_stamps);
        if (hipMemcpy(st.data(), h->d_stamps, sizeof(unsigned long long) * st.size(), hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        unsigned long long lo = ~0ull, hi0 = 0, hi = 0;
        for (int q = 0; q < h->n_stamps; q++) {
            if (!st[8 * q]) continue;
            lo = std::min(lo, st[8 * q]);
            hi0 = std::max(hi0, st[8 * q]);
            for (int k = 1; k < 8; k++) hi = std::max(hi, st[8 * q + k]);
        }
        if (lo == ~0ull) return 0;
        return (long long)((n == "chain_start_spread" ? hi0 : hi) - lo) * 10;
    }
    if (n.rfind("chain_phase", 0) == 0 && h->d_stamps && h->n_stamps > 0) {
        // diagnostic: "chain_phaseK" = median over segments of (stamp K - stamp 0)
        // in ns; "chain_phaseK_max" = the largest; K = 1..7 (0 where unstamped)
        const bool mx = n.size() > 4 && n.substr(n.size() - 4) == "_max";
        const bool clk = n.size() > 4 && n.substr(n.size() - 4) == "_mhz";  // shader clock over phases 1-2
        const int k = n[11] - '0';
        if (k < 1 || k > 7) return -1;
        std::vector<unsigned long long> st(16 * (size_t)h->n_stamps);
        if (clk) {
            if (hipMemcpy(st.data(), h->d_stamps, sizeof(unsigned long long) * st.size(), hipMemcpyDeviceToHost) != hipSuccess)
                return -1;
            std::vector<long long> f;
            for (int q = 0; q < h->n_stamps; q++) {
                const unsigned long long *r = &st[8 * q], *c = &st[8 * ((size_t)h->n_stamps + q)];
                if (r[k] > r[1] && r[1]) f.push_back((long long)((c[k] - c[1]) * 100 / (r[k] - r[1])));
            }
            if (f.empty()) return 0;
            std::sort(f.begin(), f.end());
            return f[f.size() / 2];
        }
        st.resize(8 * (size_t)h->n_stamps);
        if (hipMemcpy(st.data(), h->d_stamps, sizeof(unsigned long long) * st.size(), hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
        std::vector<long long> d;
        for (int q = 0; q < h->n_stamps; q++)
            if (st[8 * q + k] && st[8 * q]) d.push_back((long long)(st[8 * q + k] - st[8 * q]) * 10);
        if (d.empty()) return 0;
        std::sort(d.begin(), d.end());
        return mx ? d.back() : d[d.size() / 2];
    }
    if (n == "master") return h->master;  // world rank of the first server (adlb.c:256)
    if (n == "parked") return h->ctr.n_parked_last;
    if (n == "one_batches") return h->one_batches;  // one-Reserve batches through k_reserve_one
    if (n == "rq_cap") return h->rq_cap;  // rq slots allocated
    if (n == "rq_slots") {                // rq slots in use, and rqseqnos handed out / compactions
        refresh_counters(h);
        return h->ctr.rq_n;
    }
    if (n == "rq_next") {
        refresh_counters(h);
        return h->ctr.rq_next;
    }
    if (n == "rq_reclaims") {
        refresh_counters(h);
        return h->ctr.rq_reclaims;
    }
    if (n == "spec_lists") return h->ctr.spec_page0;
    if (n == "rank_fast") return h->ctr.rank_fast;
    if (n == "tindex_merges") return h->tidx_merges;   // targeted index: incremental merges
    if (n == "tindex_delta_merges") return h->tidx_delta_merges;  // Put batches merged into the delta index
    if (n == "tindex_folds") return h->tidx_folds;      // delta folded into the main index
    if (n == "tindex_rebuilds") return h->tidx_rebuilds;  // and full rebuilds
    if (n == "candidates") {
        int v = 0;
        if (h->T > 0 && hipMemcpy(&v, h->d_candoff + h->T, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
        return v;
    }
    if (n == "device_sorted_lists") return h->n_segsort;  // candidate lists given a device-wide sort (cumulative)
    if (n.rfind("hacc:", 0) == 0) {  // cumulative host time of a section of the reserve call
        auto it = h->hacc.find(n.substr(5));
        return it == h->hacc.end() ? 0 : it->second;
    }
    if (n.rfind("host_ns:", 0) == 0) {  // host time issuing a profiled stage (adlbq_profile_only)
        auto it = h->timers.find(n.substr(8));
        return it == h->timers.end() ? 0 : it->second.host_ns;
    }
    if (n == "keyrank") return h->n_keyrank;               // batches ranked by keyrank (cumulative)
    if (n == "keyrank_failed") {                             // ... that failed over to k_rank, as of the newest landed batch
        refresh_counters(h);
        return h->ctr.kr_fail;
    }
    if (n == "keyrank_why" || n == "keyrank_maxbin") {  // the last failover's reason; the last batch's largest bin
        refresh_counters(h);
        return n == "keyrank_why" ? h->ctr.kr_why : h->ctr.kr_maxbin;
    }
    if (n == "sort_radix") return h->n_sort_radix;         // planned sorts issued as the list-stable radix sort
    if (n == "sort_async_bad") {  // ... whose plan did not hold (k_rank sorted them), as of the newest landed batch
        refresh_counters(h);
        return h->ctr.plan_missed;
    }
    if (n == "bound_faults") return h->ctr.bound_faults;
    if (n == "tscan_batches") return h->tscan_batches;
    if (n == "unres_trusted") return h->unres_trusted_calls;
    if (n == "sort_timeouts" || n == "batch_failed") {  // batches answered ADLB_ERROR because k_rank's wait
        refresh_counters(h);                                // for an in-launch sort gave up (0 unless broken)
        return h->ctr.batch_failed;
    }
    return -1;
}

}  // extern "C"
