// adlbq_reserve.hip -- batched FA_RESERVE matching (src/adlb.c:1199-1317) on gfx950.
//
// A batch of R Reserves is matched with results identical to R sequential
// calls of wq_find_pre_targeted_hi_prio / wq_find_hi_prio (src/xq.c:190-247)
// followed by the pin.  Pipeline (all on the handle's stream):
//
//   k_prep_hist    one launch, two roles: request type vectors -> 64-bit type
//                  masks, per-type demand, per-segment request counts, per-batch
//                  resets (prep_block); and pass 1 over the open (untargeted)
//                  bucket: per page and per type, histogram of
//                  distance-from-anchor bins, 8 B/unit read (hist_page)
//   k_thresholds   per type: the bin where the demand is reached and how many
//                  units of it are needed (exact bins: by wqseqno order); the
//                  chunk prefix of every column
//   k_select_open  pass 2: order-preserving compaction of the top units of each
//                  type into per-type candidate lists (prio desc, wqseqno asc)
//   k_sort_types   only for types whose threshold fell in a multi-priority bin
//   k_targeted     per target-rank bucket: that rank's Reserves in order against
//                  its own targeted units (pre-targeted scan, xq.c:219-247)
//   k_rank         packed global rank of every candidate
//   k_chain_pass   the untargeted choices in arrival order, as segment-parallel
//   k_chain_fix    passes with a fixed-point check (see the chain section)
//   k_finalize     pins, TA_RESERVE_RESP records; its last workgroup parks the
//                  unmatched hanging Reserves on rq (FIFO) with their RFR donors
#include <algorithm>
#include <climits>
#include <cstring>

#include "adlbq_donor.h"
#include "adlbq_impl.h"
#include "adlbq_rsx.h"

using namespace adlbq;


constexpr int SEG_BLOCKS = SEG / 64;   // SEG, CHAIN_WARM: adlbq_impl.h
constexpr int PREP_BLOCK = 256;        // prep_block workgroup
constexpr int RANK_FAST_T = 8;         // k_select_open ranks the candidates itself for up to this many types
constexpr int LV_STEP = 64;            // the chain's level rows are kept for every LV_STEP-th global rank
static_assert(SEG % 64 == 0 && CHAIN_WARM % SEG == 0, "chain segments are whole waves of prep_block");

__device__ __forceinline__ unsigned long long readlane64(unsigned long long v, int l) {
    unsigned int lo = __builtin_amdgcn_readlane((unsigned int)v, l);
    unsigned int hi = __builtin_amdgcn_readlane((unsigned int)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}

// Request type vectors -> 64-bit type masks (get_type_idx, adlb.c:3476-3485;
// -1 = any type) and per-type demand.  The workgroup's 256 request records are
// staged through LDS with coalesced loads (rows padded to 19 words: no bank
// conflicts).  Each wave also writes its chain segment's count of requests
// with a non-empty type set (the chain's level guess), tmatch starts at -1,
// and block 0 resets the chain's per-batch counters.

struct PrepArgs {
    const int *reqs;
    int R;
    const int *utypes;
    int T;
    unsigned long long *mask;
    int *dem;
    int *seg_cnt;
    DevCounters *ctr;
    int *tmatch;
    // per target-rank bucket lists of the batch's Reserves (k_targeted_idx), or tlist == nullptr
    const int *rank2b;  // [A] app rank -> bucket index or -1
    int A;
    int *tcnt;          // [buckets] appended entries (k_targeted_idx resets its own)
    int *tlist;         // [buckets][tcap] request indices, any order
    int tcap;
    int dem_extra;      // candidates listed per type beyond the demand (a steal group's export depth)
    int2 *rh;           // [R] out: (rank, hang) of each request, compact for k_finalize (or nullptr)
};

template <int TB>  // TB >= T; TB <= 8: the user types are compared in registers
__device__ __forceinline__ void prep_block(const PrepArgs &a, const int blk) {
    __shared__ int su[ADLBQ_MAX_TYPES], sd[ADLBQ_MAX_TYPES];
    const int *__restrict__ reqs = a.reqs, *__restrict__ utypes = a.utypes;
    const int R = a.R, T = a.T;
    unsigned long long *__restrict__ mask = a.mask;
    int *dem = a.dem, *__restrict__ seg_cnt = a.seg_cnt, *__restrict__ tmatch = a.tmatch;
    DevCounters *ctr = a.ctr;
    const int j0 = blk * PREP_BLOCK, nj = min(PREP_BLOCK, R - j0);
    // this thread's request record, straight into registers (9 x 8 B: a record is 72 B,
    // so every record is 8-B aligned; the wave's loads cover one contiguous 4.6 KB run)
    static_assert(ADLBQ_RESERVE_INTS == 18, "record layout");
    int row[ADLBQ_RESERVE_INTS];
    const bool mine = (int)threadIdx.x < nj;  // (a larger block's threads past PREP_BLOCK idle: nj <= PREP_BLOCK)
    if (mine) {
        const int2 *src = reinterpret_cast<const int2 *>(reqs + (long long)ADLBQ_RESERVE_INTS * (j0 + threadIdx.x));
#pragma unroll
        for (int i = 0; i < ADLBQ_RESERVE_INTS / 2; i++) {
            const int2 v = src[i];
            row[2 * i] = v.x;
            row[2 * i + 1] = v.y;
        }
    }
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        su[t] = utypes[t];
        sd[t] = 0;
    }
    if (blk == 0 && threadIdx.x == 0) ctr->chain_rounds = 0;
    // small T: user types in registers; a type equal to an earlier one never matches
    // (get_type_idx returns the first declared match)
    int ur[TB <= 8 ? TB : 1];
    bool uok[TB <= 8 ? TB : 1];
    if constexpr (TB <= 8) {
        // every load unconditional (a clamped index) under one uniform branch: a load per "t < T"
        // branch waited for the one before
        if (T > 0) {
#pragma unroll
            for (int t = 0; t < TB; t++) ur[t] = utypes[t < T ? t : T - 1];
        } else {
#pragma unroll
            for (int t = 0; t < TB; t++) ur[t] = 0;
        }
#pragma unroll
        for (int t = 0; t < TB; t++) {
            uok[t] = t < T;
#pragma unroll
            for (int t2 = 0; t2 < t; t2++) uok[t] = uok[t] && ur[t2] != ur[t];
        }
    }
    __syncthreads();
    // larger T: the user types sorted (value, then declared index) for a binary search per slot,
    // and the slots outside [smallest, largest] type (the -2 padding) rejected at once
    __shared__ int sv[ADLBQ_MAX_TYPES], si[ADLBQ_MAX_TYPES];
    if constexpr (TB > 8) {
        if (threadIdx.x < T) {
            const int v = su[threadIdx.x];
            int r = 0;
            for (int u = 0; u < T; u++) {
                const int x = su[u];
                r += (x < v || (x == v && u < (int)threadIdx.x)) ? 1 : 0;
            }
            sv[r] = v;
            si[r] = threadIdx.x;
        }
        __syncthreads();
    }
    const int j = j0 + threadIdx.x;
    unsigned long long m = 0;
    if (mine) {
        tmatch[j] = -1;
        if (a.rh != nullptr) a.rh[j] = make_int2(row[0], row[1]);
        const int *rt = row + 2;
        bool wild = false;
#pragma unroll
        for (int i = 0; i < NREQ; i++) {
            const int v = rt[i];
            wild |= v == -1;
            if constexpr (TB <= 8) {
#pragma unroll
                for (int t = 0; t < TB; t++) m |= (uok[t] && v == ur[t]) ? (1ull << t) : 0ull;
            } else {
                if (v == -1 || T == 0 || v < sv[0] || v > sv[T - 1]) continue;
                int lo = 0, hi = T - 1;  // first sorted entry >= v: the first declared match (get_type_idx)
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (sv[mid] < v) lo = mid + 1;
                    else hi = mid;
                }
                if (sv[lo] == v) m |= 1ull << si[lo];
            }
        }
        if (wild) m = T >= 64 ? ~0ull : ((1ull << T) - 1);
        mask[j] = m;
        if (a.tlist != nullptr && m) {  // the Reserve's rank owns targeted units: list it under that bucket
            const int r = row[0];
            const int b = (r >= 0 && r < a.A) ? a.rank2b[r] : -1;
            if (b >= 0) {
                const int k = atomicAdd(&a.tcnt[b], 1);
                if (k < a.tcap) a.tlist[(long long)b * a.tcap + k] = j;
            }
        }
    }
    const unsigned long long nz = __ballot(m != 0ull);
    if ((threadIdx.x & 63) == 0 && j < R && (int)threadIdx.x < PREP_BLOCK) seg_cnt[j >> 6] = __popcll(nz);  // per 64 requests
    if constexpr (TB <= 8) {  // per-type demand: one LDS add per wave and type
#pragma unroll
        for (int t = 0; t < TB; t++) {
            const int c = __popcll(__ballot((m >> t) & 1ull));
            if ((threadIdx.x & 63) == 0 && c) atomicAdd(&sd[t], c);
        }
    } else {
        for (unsigned long long b = m; b; b &= b - 1) atomicAdd(&sd[__ffsll((long long)b) - 1], 1);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        const int d = sd[t] + (blk == 0 ? a.dem_extra : 0);
        if (d) atomicAdd(&dem[t], d);
    }
}

// ---------------------------------------------------------------- pass 1
// One workgroup per page: each wave owns a quarter of the page and issues all
// of its loads (8 x 16 B per lane) before counting.  The histogram is kept in
// HK lane-interleaved copies so that lanes hitting the same (type, bin) column
// (most units fall in a few far bins) do not serialise one LDS atomic.
constexpr int HK = 4;

// lanes below this one with their bit set in m
__device__ __forceinline__ unsigned int mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((unsigned int)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned int)m, 0u));
}

// diagnostic ("kernel_stamps"): per workgroup, the constant clock (100 MHz) at
// phase boundaries of pass 1 / pass 2, [workgroup][4]
__device__ __forceinline__ void kstamp(unsigned long long *kst, int bid, int ph) {
    if (kst != nullptr && threadIdx.x == 0) kst[(long long)bid * 4 + ph] = __builtin_amdgcn_s_memrealtime();
}

struct HistArgs {
    const int *pages;
    int npages, tail_fill;
    const int *prio;
    const uint32_t *meta;
    int T;
    const long long *anchor;
    unsigned short *gh;
    unsigned int *csum;
    const long long *gcut;   // [T] guessed cut (LLONG_MAX: none)
    unsigned int *spec;      // [npages][4][SPEC_CAP] per wave: (column << 12 | slot-in-page), slot order
    int *specn;              // [npages][4] entries found (> SPEC_CAP: overflowed, not usable)
    const int *pbase, *pwide;  // per page id: packed-offset base, wide flag
    unsigned int *zcs;         // the other chunk-sum buffer (the previous scan's): k_thresholds zeroes it
    long long zn;
    int pg0;                   // >= 0: the open pages are pg0, pg0 + 1, ... (no page-table read before the loads)
    unsigned long long *kst = nullptr;  // diagnostic stamps, or nullptr
    int all_narrow = 0;        // every open page is narrow (packed offsets): pwide is not read
};

// A quarter page (16 units per lane) of the scan columns.  A narrow page's
// prios come from the offsets packed into meta (4 B per unit); only a wide
// page reads the prio column as well.
__device__ __forceinline__ void load_quarter(const int *__restrict__ prio, const uint32_t *__restrict__ meta,
                                             const int *__restrict__ pbase, const int *__restrict__ pwide,
                                             int pg, int fill, int w, int4 (&pv)[4], uint4 (&mv)[4]) {
    const int lane = threadIdx.x & 63;
    const long long base = (long long)pg << PAGE_SHIFT;
    const int4 *P4 = reinterpret_cast<const int4 *>(prio + base);
    const uint4 *M4 = reinterpret_cast<const uint4 *>(meta + base);
    const int wide = pwide[pg], pb = pbase[pg];  // in flight with the meta loads
    // unconditional loads (slot 0 past the fill, masked after; the masks opaque to the optimiser):
    // loads under a per-lane branch were issued one at a time
    unsigned int km[4];
    int ic[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int idx = (w * 4 + k) * 64 + lane;
        km[k] = idx * 4 < fill ? ~0u : 0u;
        ic[k] = idx * 4 < fill ? idx : 0;
        mv[k] = M4[ic[k]];
    }
    asm volatile("" : "+v"(km[0]), "+v"(km[1]), "+v"(km[2]), "+v"(km[3]));
#pragma unroll
    for (int k = 0; k < 4; k++) mv[k] = make_uint4(mv[k].x & km[k], mv[k].y & km[k], mv[k].z & km[k], mv[k].w & km[k]);
    if (wide) {
#pragma unroll
        for (int k = 0; k < 4; k++) pv[k] = P4[ic[k]];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int m = (int)km[k];
            pv[k] = make_int4(pv[k].x & m, pv[k].y & m, pv[k].z & m, pv[k].w & m);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
            pv[k] = make_int4(pb + (int)(mv[k].x >> M_OFF_SHIFT), pb + (int)(mv[k].y >> M_OFF_SHIFT),
                              pb + (int)(mv[k].z >> M_OFF_SHIFT), pb + (int)(mv[k].w >> M_OFF_SHIFT));
    }
}

// The far bins, lumped (T <= 8).  With a guessed cut gc below its anchor an,
// a type's units in bin lump_bin(an, gc) or deeper -- deeper than about twice
// the guessed depth -- all belong to the type's last bin NB - 1, and pass 1
// counts them per type with one ballot per type instead of binning each one.
// When the guess holds, every threshold lies above the lump; when it does not,
// the lump is a multi-priority bin like any other (listed, then sorted).
// Pass 1, k_thresholds and pass 2 bin by this same rule.  NB: nothing lumped.
__host__ __device__ __forceinline__ int lump_bin(long long an, long long gc) {
    if (gc == LLONG_MAX || gc > an || an - gc >= (1ll << 30)) return NB;
    long long d = 2 * (an - gc) + 2;
    int b;  // bin_of(d), host and device
    if (d < NBX) b = (int)d;
    else {
        int o = 0;
        while ((d >> (o + 1)) != 0) o++;
        b = o < OCT_H ? NBX + 2 * (o - 5) + (int)((d >> (o - 1)) & 1) : NBX + NBH + (o - OCT_H);
        if (b > NB - 1) b = NB - 1;
    }
    return b + 1 >= NB - 1 ? NB : b + 1;
}

// Pass 1 over one page: per (type, bin) column the available units (LDS
// copies, then the page's row and the chunk sums), and a speculative list per
// quarter page, in slot order.  QW quarters per wave: 1 (four waves per page)
// or 2 (two waves per page, two pages per workgroup: every page of the metric
// queue resident at once, where four-wave pages ran in two rounds).  NARROW:
// the page's prios are its base plus the offsets packed into meta, so only the
// meta column is loaded (the wide form holds the prio column as well).
//   LUMP (T <= 8): a unit is near when it lies above its type's lump
//   (lump_bin), and the list is every near unit.  On a narrow page a unit is
//   classified through an LDS table indexed by its meta's status and type
//   bits: {far cut in the page's offsets, counter increment}; an unavailable
//   unit's entry {INT_MAX, 0} makes it far and uncounted.  A far unit adds to
//   8-bit per-type counters in a register (four types each); a near one (a
//   few per wave when the guess holds) is staged in LDS, then binned one per
//   lane.  Should a quarter's near units overflow the list, they are binned
//   from the registers and the list is marked unusable.  A wide page bins
//   every unit, its far ones into the lump.
//   Otherwise (T > 8) every unit is binned and the list holds the units at or
//   above the guessed cut.
#ifndef ADLBQ_HIST_PPW
#define ADLBQ_HIST_PPW 2  // pages per pass-1 workgroup at T <= 8: 1 (four waves each), 2 or 4
#endif
#ifndef ADLBQ_HIST_PRE2
#define ADLBQ_HIST_PRE2 0  // pairs at T <= 4: the second quarter's loads up front too (six waves per SIMD)
#endif
constexpr int HIST_TAB = 32;  // LUMP table entries: status (meta bits 8-9) x type (bits 0-2), 2 words each
__device__ __forceinline__ unsigned int tab_idx(uint32_t m) { return ((m >> 5) & 0x18u) | (m & 7u); }
// LDS words of one page's pass-1 state: histogram copies, staged near units, table
__host__ __device__ constexpr int hist_page_words(int C, bool lump) {
    return HK * C + 8 * SPEC_CAP + (lump ? 2 * HIST_TAB : 0);
}

template <bool NARROW, bool LUMP, int TB, int QW>
__device__ __forceinline__ void hist_page_body(const HistArgs &a, const int p, const int pg, const int fill,
                                               unsigned int *__restrict__ hist /* [C][HK], stage, table */,
                                               const bool valid) {
    static_assert(QW == 1 || ((QW == 2 || QW == 4) && LUMP), "several quarters per wave: T <= 8");
    constexpr int NT = 256 / QW;  // threads per page
    __shared__ int sanc[ADLBQ_MAX_TYPES], scv[ADLBQ_MAX_TYPES], slb[ADLBQ_MAX_TYPES];
    const int tid = (int)threadIdx.x & (NT - 1);
    const int T = a.T, C = T * NB, wv = tid >> 6, lane = tid & 63;
    const long long base = (long long)pg << PAGE_SHIFT;
    const uint4 *M4 = reinterpret_cast<const uint4 *>(a.meta + base);
    const int4 *P4 = reinterpret_cast<const int4 *>(a.prio + base);
    // a narrow page's first quarter of meta, loaded before the table is set up;
    // a second quarter (QW 2) at the top of its turn of the quarter loop (with
    // every page resident, the first quarters' loads already keep HBM busy; both
    // at once would not fit the registers of six waves per SIMD).  A wide page
    // loads per quarter.
    uint4 cur[4];
    auto load_meta = [&](int w) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int idx = (w * 4 + k) * 64 + lane;
            cur[k] = idx * 4 < fill ? M4[idx] : make_uint4(0, 0, 0, 0);
        }
    };
    if (NARROW) load_meta(wv * QW);
    // PRE: the next quarter's loads in flight while a quarter is counted (nxt)
    constexpr bool PRE = QW > 1 && (QW == 4 || (ADLBQ_HIST_PRE2 && TB <= 4));
    uint4 nxt[PRE ? 4 : 1];
    auto load_next = [&](int w) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int idx = (w * 4 + k) * 64 + lane;
            nxt[k] = NARROW && idx * 4 < fill ? M4[idx] : make_uint4(0, 0, 0, 0);
        }
    };
    if constexpr (PRE) load_next(wv * QW + 1);
    const int pb = NARROW ? a.pbase[pg] : 0;
    // the table path needs every offset above LOWEST (a base above it)
    const bool fast = NARROW && LUMP && pb > LOWEST;
    uint2 *tab = reinterpret_cast<uint2 *>(hist + HK * C + 8 * SPEC_CAP);
    if (tid < 4 * T) {
        const int t = tid % T, st = tid / T;  // status: bit 0 LIVE, bit 1 PINNED
        const long long an = a.anchor[t], gc = a.gcut[t];
        const int lb = LUMP ? lump_bin(an, gc) : NB;
        const long long fc = lb < NB ? an - bin_lo(lb) - pb : (long long)INT_MIN;  // far: value <= fc
        const int fci = (int)std::max(std::min(fc, (long long)INT_MAX), (long long)INT_MIN);
        if (st == 0) {  // (both pages of a workgroup write the same values)
            sanc[t] = (int)an;
            slb[t] = lb;
            scv[t] = LUMP ? fci : (int)std::max(std::min(gc, (long long)INT_MAX), (long long)INT_MIN);
        }
        if (fast)
            tab[(st << 3) | t] = st == 1 ? make_uint2((unsigned int)fci, 1u << (8 * (t & 3)))
                                         : make_uint2((unsigned int)INT_MAX, 0u);
    }
    if (fast && tid == 0) tab[0] = make_uint2((unsigned int)INT_MAX, 0u);  // slots past the fill (meta 0)
    for (int c = tid; c < C * HK; c += NT) hist[c] = 0;
    __syncthreads();
    if (a.kst) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (valid && tid == 0) a.kst[(long long)p * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    }
    unsigned int *my = hist + (lane % HK);
    const unsigned long long lt = lanemask_lt();
    if (LUMP && fast) {
        unsigned int c0 = 0u, c1 = 0u;  // far units per type, 8 bits each: types 0-3, 4-7 (<= 32 per lane)
#pragma unroll 1
        for (int qq = 0; qq < QW; qq++) {
            const int w = wv * QW + qq;
            if constexpr (PRE) {
                if (qq > 0) {
#pragma unroll
                    for (int j = 0; j < 4; j++) cur[j] = nxt[j];
                    if (qq + 1 < QW) load_next(w + 1);
                }
            } else if (qq > 0) {
                load_meta(w);
            }
            // per-lane values recomputed in each turn, not hoisted out of the loop (registers)
            int ln = lane;
            asm volatile("" : "+v"(ln));
            unsigned int *myq = hist + (ln % HK);
            unsigned int *stg = hist + HK * C + w * 2 * SPEC_CAP;  // near units: (type << 12 | slot), prio
            unsigned int *__restrict__ sp = a.spec + ((long long)p * 4 + w) * SPEC_CAP;
            int sn = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                __builtin_amdgcn_sched_barrier(0);  // one sixteenth's table reads at a time (registers)
                const uint32_t mm[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
                uint2 e[4];
#pragma unroll
                for (int q = 0; q < 4; q++) e[q] = tab[tab_idx(mm[q])];
                unsigned long long b[4];
                bool ne[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const bool far = (int)(mm[q] >> M_OFF_SHIFT) <= (int)e[q].x;
                    ne[q] = !far;
                    if constexpr (TB <= 4) {
                        c0 += far ? e[q].y : 0u;
                    } else {
                        const bool hi = (mm[q] & 4u) != 0u;
                        c0 += (far && !hi) ? e[q].y : 0u;
                        c1 += (far && hi) ? e[q].y : 0u;
                    }
                    b[q] = __builtin_amdgcn_ballot_w64(!far);
                }
                asm volatile("" : "+v"(c0), "+v"(c1));  // summed here, not deferred (registers)
                if (!(b[0] | b[1] | b[2] | b[3])) continue;
                int pos = sn + (int)mbcnt64(b[0]) + (int)mbcnt64(b[1]) + (int)mbcnt64(b[2]) + (int)mbcnt64(b[3]);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (ne[q]) {
                        if (pos < SPEC_CAP) {
                            stg[pos] = ((mm[q] & M_TYPE) << 12) | (unsigned int)((w * 4 + k) * 256 + ln * 4 + q);
                            stg[SPEC_CAP + pos] = (unsigned int)(pb + (int)(mm[q] >> M_OFF_SHIFT));
                        }
                        pos++;
                    }
                }
                sn += __popcll(b[0]) + __popcll(b[1]) + __popcll(b[2]) + __popcll(b[3]);
            }
            if (sn <= SPEC_CAP) {  // the staged near units: binned one per lane, listed with their columns
                __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
                for (int i = ln; i < sn; i += 64) {
                    const unsigned int ev = stg[i];
                    const int t = (int)(ev >> 12), pr = (int)stg[SPEC_CAP + i];
                    const int col = t * NB + bin_of32((unsigned int)sanc[t] - (unsigned int)pr);
                    atomicAdd(&myq[col * HK], 1u);
                    sp[i] = ((unsigned int)col << 12) | (ev & (PAGE - 1));
                }
            } else {  // overflow (no usable guess): the near units binned from the registers, no list
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    __builtin_amdgcn_sched_barrier(0);  // a sixteenth at a time (registers)
                    uint32_t mm[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
#pragma unroll
                    for (int q = 0; q < 4; q++) asm volatile("" : "+v"(mm[q]));  // recomputed here, not kept live from above
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int off = (int)(mm[q] >> M_OFF_SHIFT);
                        if (off > (int)tab[tab_idx(mm[q])].x) {
                            const int t = mm[q] & M_TYPE;
                            atomicAdd(&myq[(t * NB + bin_of32((unsigned int)sanc[t] - (unsigned int)(pb + off))) * HK], 1u);
                        }
                    }
                }
            }
            if (valid && ln == 0) a.specn[(long long)p * 4 + w] = sn;
        }
        // the far counts: 16-bit lanes of the even and odd bytes, summed over the wave
        unsigned int f[4] = {c0 & 0x00ff00ffu, (c0 >> 8) & 0x00ff00ffu, c1 & 0x00ff00ffu, (c1 >> 8) & 0x00ff00ffu};
#pragma unroll
        for (int i = 0; i < (TB <= 4 ? 2 : 4); i++)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) f[i] += __shfl_xor(f[i], o, 64);
        if (lane == 0)
#pragma unroll
            for (int u = 0; u < TB; u++) {
                // type u: word (u >> 2) * 2 + (u & 1), half (u >> 1) & 1
                const unsigned int v = (f[(u >> 2) * 2 + (u & 1)] >> (16 * ((u >> 1) & 1))) & 0xffffu;
                if (u < T && v) atomicAdd(&hist[(u * NB + NB - 1) * HK], v);
            }
    } else {
#pragma unroll 1
        for (int qq = 0; qq < QW; qq++) {
            const int w = wv * QW + qq;
            unsigned int *__restrict__ sp = a.spec + ((long long)p * 4 + w) * SPEC_CAP;
            int sn = 0;
            int4 pv[NARROW ? 1 : 4];
            if constexpr (!NARROW) {
                load_meta(w);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int idx = (w * 4 + k) * 64 + lane;
                    pv[k] = idx * 4 < fill ? P4[idx] : make_int4(0, 0, 0, 0);
                }
            } else if (qq > 0) {
                if constexpr (PRE) {
#pragma unroll
                    for (int j = 0; j < 4; j++) cur[j] = nxt[j];
                    if (qq + 1 < QW) load_next(w + 1);
                } else {
                    load_meta(w);
                }
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t mm[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
                int pr[4];
                if constexpr (NARROW) {
#pragma unroll
                    for (int q = 0; q < 4; q++) pr[q] = pb + (int)(mm[q] >> M_OFF_SHIFT);
                } else {
                    pr[0] = pv[k].x, pr[1] = pv[k].y, pr[2] = pv[k].z, pr[3] = pv[k].w;
                }
                int col[4];
                bool in[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const bool av = (mm[q] & (M_LIVE | M_PINNED)) == M_LIVE && pr[q] > LOWEST;
                    const int t = mm[q] & M_TYPE;
                    const int bq = bin_of32((unsigned int)sanc[t] - (unsigned int)pr[q]);  // distance < 2^32
                    if constexpr (LUMP) {  // a wide page (or a base at LOWEST): the far ones into the lump
                        in[q] = av && bq < slb[t];
                        col[q] = t * NB + (in[q] ? bq : NB - 1);
                    } else {
                        in[q] = av && pr[q] >= scv[t];
                        col[q] = t * NB + bq;
                    }
                    if (av) atomicAdd(&my[col[q] * HK], 1u);
                }
                const unsigned long long b0 = __ballot(in[0]), b1 = __ballot(in[1]), b2 = __ballot(in[2]),
                                         b3 = __ballot(in[3]);
                if (!(b0 | b1 | b2 | b3)) continue;
                int pos = sn + __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (in[q]) {
                        if (pos < SPEC_CAP)
                            sp[pos] = ((unsigned int)col[q] << 12) | (unsigned int)((w * 4 + k) * 256 + lane * 4 + q);
                        pos++;
                    }
                }
                sn += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
            }
            if (valid && lane == 0) a.specn[(long long)p * 4 + w] = sn;
        }
    }
    __syncthreads();
    if (valid && a.kst && tid == 0) a.kst[(long long)p * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    if (valid) {
        unsigned int *cs = a.csum + (long long)(p / CHUNK) * C;
        unsigned short *g = a.gh + (long long)p * C;
        for (int c = tid; c < C; c += NT) {
            unsigned int v = 0;
#pragma unroll
            for (int k = 0; k < HK; k++) v += hist[c * HK + k];
            g[c] = (unsigned short)v;
            if (v) atomicAdd(&cs[c], v);
        }
    }
    if (a.kst) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (valid && tid == 0) a.kst[(long long)p * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
}

// Pass 1's shape for T <= TB: two pages per workgroup (two waves each) for
// T <= 8 (ADLBQ_HIST_PPW); otherwise one page (four waves).
__host__ __device__ constexpr int hist_pp(int TB) { return TB <= 8 ? ADLBQ_HIST_PPW : 1; }
// minimum waves per SIMD k_prep_hist is compiled for: for the pairs eight at
// T <= 4 (<= 64 VGPRs), six at T <= 8 (<= 80), so that 2,442 pages and the
// request preparation fit at once
#ifndef ADLBQ_HIST_WAVES
#define ADLBQ_HIST_WAVES 8
#endif
__host__ __device__ constexpr int hist_waves(int TB) {
    return hist_pp(TB) == 1 ? 1 : hist_pp(TB) == 4 ? 4 : TB <= 4 && !ADLBQ_HIST_PRE2 ? ADLBQ_HIST_WAVES : 6;
}

template <int TB>
__device__ __forceinline__ void hist_pages(const HistArgs &a, const int q, unsigned int *__restrict__ hist) {
    constexpr int PP = hist_pp(TB);
    const int half = (int)threadIdx.x / (256 / PP);  // the workgroup's page
    const int p = q * PP + half;
    const bool valid = p < a.npages;  // the last workgroup's second page may not exist (it still takes the barriers)
    const int pv = valid ? p : a.npages - 1;
    const int pg = a.pg0 >= 0 ? a.pg0 + pv : a.pages[pv];
    const int fill = !valid ? 0 : (p == a.npages - 1) ? a.tail_fill : PAGE;
    unsigned int *h = hist + half * hist_page_words(a.T * NB, TB <= 8);
    if (valid && a.kst && (threadIdx.x & (256 / PP - 1)) == 0) a.kst[(long long)p * 4] = __builtin_amdgcn_s_memrealtime();
    // every open page narrow (the host's count): no dependent load of the flag before the meta loads
    if (!a.all_narrow && a.pwide[pg]) hist_page_body<false, (TB <= 8), TB, PP>(a, p, pg, fill, h, valid);
    else hist_page_body<true, (TB <= 8), TB, PP>(a, p, pg, fill, h, valid);
}

// Pass 1 and the request preparation in one launch (they are independent):
// workgroups [0, nprep) prepare 256 requests each, the rest count one page.
constexpr int PREP_LDS = 0;  // the request records go straight to registers


// The lowest prio in bins 0..th of a type with anchor an (bin_of: exact bins
// below NBX, then powers of two); no bin (th < 0) cuts above every prio.
__device__ __forceinline__ long long cut_of(int th, long long an) {
    if (th < 0) return 1ll << 40;
    const long long dmax = bin_hi(th);
    return std::max(an - dmax, (long long)LOWEST + 1);
}

// Type t's threshold, by wave 0 of the workgroup whose column of type t
// arrived last (lane b = bin b): the bin where the demand is reached and how
// many units of it are needed; the next anchor and guessed cut.
// d: the type's demand (prep's atomics), x: lane b's column total (bin b), both from the caller: the
// totals are the caller's own sums, and the demand was loaded with the tile totals (no second round)
__device__ void type_threshold(const int t, const int d, const long long x, int *theta, int *need, int *candlen,
                               int *needsort, int *binoff, int *type_cnt,
                               const long long *__restrict__ anchor, long long *__restrict__ anchor_next,
                               long long *__restrict__ gcut_next, int guess, const long long *__restrict__ gcut,
                               int T) {
    const int lane = threadIdx.x & 63;
    // the last column of type t: wave 0, lane b = bin b (NB == 64)
    static_assert(NB == 64, "one lane per bin");
    if (lane == 0) type_cnt[t] = 0;  // for the next batch
    long long incl = x;  // inclusive prefix over bins
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const long long cum = incl - x;
    int th = -1, nd = 0, len = 0;
    if (d > 0) {
        binoff[t * NB + lane] = (int)cum;
        const unsigned long long nz = __ballot(x > 0), hit = __ballot(incl >= d);
        if (nz && lane == 0) {
            // the live maximum is at most anchor - (smallest distance of the first
            // non-empty bin): the next batch's anchor (applied when this batch ends)
            const int bb = __ffsll((long long)nz) - 1;
            // a lump (T <= 8) starts at its lump bin
            const int lb = (T <= 8 && bb == NB - 1) ? lump_bin(anchor[t], gcut[t]) : NB;
            anchor_next[t] = anchor[t] - bin_lo(lb < NB ? lb : bb);
        }
        if (hit) {
            th = __ffsll((long long)hit) - 1;
            const long long cth = __shfl(cum, th, 64), ith = __shfl(incl, th, 64);
            if (th < NBX) {  // one priority value: the first (d - cum) by wqseqno
                nd = (int)(d - cth);
                len = d;
            } else {         // several values: take the whole bin, sort later
                nd = INT_MAX;
                len = (int)ith;
            }
        } else {             // fewer available units than demand: take all
            th = NB - 1;
            nd = INT_MAX;
            len = (int)__shfl(incl, 63, 64);
        }
    }
    if (lane == 0) {
        if (guess && d > 0) {  // next batch's pass-1 guess: this cut less a margin of half its depth
            const long long an = anchor[t], cut = cut_of(th, an);
            gcut_next[t] = cut - std::max(2ll, (an - cut) / 2);
        }
        theta[t] = th;
        need[t] = nd;
        candlen[t] = len;
        needsort[t] = (th >= NBX && len > 1) ? 1 : 0;
    }
}

// ---------------------------------------------------------------- thresholds
// One workgroup per (row tile, type): TH_ROWS chunk rows of the type's NB
// columns (lane = column, four waves of 16 rows; every load a 256-byte row
// segment).  The tile's exclusive prefix goes back into the chunk sums in
// place, its column totals to the tile area after them (csum + nchunks * C,
// [nrt][C], agent-scope stores).  The tile of a type that arrives last (one
// counter per type) turns the tile totals into their exclusive prefix in place
// (k_select_open / k_select_wave add it), writes the column totals, and finds
// the bin where the type's demand is reached and how many units of it are
// needed.  Candidate list offsets (the prefix of candlen over types) follow in
// pass 2.
constexpr int TH_THREADS = 256;
constexpr int TH_ROWS = 64;  // chunk rows per tile (16 per wave)
__host__ __device__ constexpr int th_tiles(int nchunks) { return (nchunks + TH_ROWS - 1) / TH_ROWS; }
__device__ __forceinline__ void thresholds_body(unsigned int *zcs, long long zn, int T, const int *__restrict__ dem, unsigned int *csum,
                                                     int nchunks, int *theta, int *need, int *candlen,
                                                     int *needsort, int *binoff, unsigned int *coltot,
                                                     int *type_cnt, const long long *__restrict__ anchor,
                                                     long long *__restrict__ anchor_next,
                                                     long long *__restrict__ gcut_next, int guess,
                                                     const long long *__restrict__ gcut, const int bid_, const int nbk_) {
    static_assert(NB == 64 && TH_THREADS == 256 && TH_ROWS == 64, "lane = column, four waves of 16 rows");
    __shared__ unsigned int wsum[4][64];
    __shared__ bool s_last;
    const int nrt = th_tiles(nchunks), C = T * NB;
    const int rt = bid_ % nrt, t = bid_ / nrt, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = t * NB + lane;
    unsigned int *tile = csum + (long long)nchunks * C;
    const int r0 = rt * TH_ROWS + w * 16;
    unsigned int v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = r0 + i < nchunks ? csum[(long long)(r0 + i) * C + c] : 0u;
    unsigned int run = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) run += v[i];
    wsum[w][lane] = run;
    __syncthreads();
    unsigned int x = 0;
#pragma unroll
    for (int q = 0; q < 3; q++)
        if (q < w) x += wsum[q][lane];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        if (r0 + i < nchunks) csum[(long long)(r0 + i) * C + c] = x;
        x += v[i];
    }
    if (w == 3) {  // x: the tile's column total
        __hip_atomic_store(tile + (long long)rt * C + c, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&type_cnt[t], 1) == nrt - 1;
    // the previous scan's chunk sums (consumed): zeroed for the scan after this one, a slice per workgroup
    if (zn > 0) {
        const long long per = (zn + nbk_ - 1) / nbk_, z0 = (long long)bid_ * per;
        for (long long i = z0 + threadIdx.x; i < min(zn, z0 + per); i += TH_THREADS) zcs[i] = 0u;
    }
    __syncthreads();
    if (!s_last || threadIdx.x >= 64) return;
    const int d = __hip_atomic_load(dem + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // with the tile totals
    unsigned int tot = 0;
    for (int r0 = 0; r0 < nrt; r0 += 8) {  // eight tiles' loads in flight at a time
        unsigned int y[8];
#pragma unroll
        for (int i = 0; i < 8; i++)
            y[i] = r0 + i < nrt ? __hip_atomic_load(tile + (long long)(r0 + i) * C + c, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : 0u;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (r0 + i < nrt) tile[(long long)(r0 + i) * C + c] = tot;  // exclusive prefix over the tiles, read by pass 2
            tot += y[i];
        }
    }
    __hip_atomic_store(coltot + c, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for pass 2 and the export
    type_threshold(t, d, (long long)tot, theta, need, candlen, needsort, binoff, type_cnt, anchor, anchor_next,
                   gcut_next, guess, gcut, T);
}

// The exclusive prefix of seg_cnt per 64 requests (jp[q] = requests before 64 q that may take an
// untargeted unit): the chain's level guess reads one word instead of summing up to 1,024 (one
// dependent load round fewer in its prologue).  One workgroup of TH_THREADS.
__device__ __forceinline__ void seg_prefix(const int *__restrict__ seg_cnt, int nq, int *jp) {
    __shared__ int wtot[TH_THREADS / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int base = 0;
    constexpr int PER = 4;  // consecutive entries per thread, their loads in flight together
    for (int q0 = 0; q0 < nq; q0 += TH_THREADS * PER) {
        const int qa = q0 + tid * PER;
        int v[PER], sum = 0;
        unsigned int okm = 0u;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            okm |= (qa + k < nq ? 1u : 0u) << k;
            v[k] = seg_cnt[qa + k < nq ? qa + k : 0];
        }
        asm volatile("" : "+v"(okm));  // masks opaque to the optimiser (no load sunk into a branch)
#pragma unroll
        for (int k = 0; k < PER; k++) {
            v[k] &= 0 - (int)((okm >> k) & 1u);
            sum += v[k];
        }
        int x = sum;  // inclusive scan over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wtot[w] = x;
        __syncthreads();
        int pre = base;
        for (int k = 0; k < w; k++) pre += wtot[k];
        pre += x - sum;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            if (qa + k < nq) jp[qa + k] = pre;
            pre += v[k];
        }
        int tot = 0;
        for (int k = 0; k < TH_THREADS / 64; k++) tot += wtot[k];
        base += tot;
        __syncthreads();
    }
    if (tid == 0) jp[nq] = base;
}

__global__ __launch_bounds__(TH_THREADS) void k_thresholds(unsigned int *zcs, long long zn, int T, const int *__restrict__ dem, unsigned int *csum,
                                                     int nchunks, int *theta, int *need, int *candlen,
                                                     int *needsort, int *binoff, unsigned int *coltot,
                                                     int *type_cnt, const long long *__restrict__ anchor,
                                                     long long *__restrict__ anchor_next,
                                                     long long *__restrict__ gcut_next, int guess,
                                                     const long long *__restrict__ gcut, const int *seg_cnt = nullptr,
                                                     int nq = 0, int *jp = nullptr) {
    if (jp != nullptr && blockIdx.x == gridDim.x - 1) {  // the launch's extra workgroup
        seg_prefix(seg_cnt, nq, jp);
        return;
    }
    thresholds_body(zcs, zn, T, dem, csum, nchunks, theta, need, candlen, needsort, binoff, coltot, type_cnt, anchor,
                    anchor_next, gcut_next, guess, gcut, blockIdx.x, gridDim.x - (jp != nullptr ? 1 : 0));
}

// Pass 1 and the request preparation in one launch (they are independent):
// workgroups [0, nprep) prepare 256 requests each, the rest count one page.
template <int TB>
__device__ __forceinline__ void prep_hist_body(PrepArgs pa, int nprep, HistArgs ha, const int bid_) {
    static_assert(PREP_BLOCK == 256, "one launch shape for both roles");
    extern __shared__ unsigned int lds[];
    if ((int)bid_ < nprep) {
        prep_block<TB>(pa, bid_);
    } else {
        hist_pages<TB>(ha, bid_ - nprep, lds);
    }
}

template <int TB>
__global__ __launch_bounds__(256, hist_waves(TB)) void k_prep_hist(PrepArgs pa, int nprep, HistArgs ha) {
    prep_hist_body<TB>(pa, nprep, ha, blockIdx.x);
}

// ---------------------------------------------------------------- pass 2
// Order-preserving compaction of the candidates (the units of each type in the
// bins up to its threshold) into per-type lists in (prio desc, wqseqno asc)
// order.  One workgroup per page, each wave a quarter of it:
//   1. all loads issued up front; a unit is a candidate iff prio >= cut[t]
//      (equivalent to bin_of(anchor - prio) <= theta[t]);
//   2. each wave appends its candidates, in slot order, to an LDS list
//      (key = column << 12 | slot-in-page) and counts them per column;
//   3. per column: page prefix + counts of the earlier waves;
//   4. a candidate's rank in its column = that start + the number of equal
//      columns earlier in the wave's list (64 list entries per step).
template <int TB>  // TB >= T; the candidates are ranked here only for TB <= RT
__device__ __forceinline__ void select_open_body(
    const int *__restrict__ pages, int npages, int tail_fill, const int *__restrict__ prio,
    const uint32_t *__restrict__ meta, const int *__restrict__ seqa, int T, const long long *__restrict__ anchor,
    const int *__restrict__ theta, const int *__restrict__ need,
    const int *__restrict__ binoff, const unsigned int *__restrict__ csum, const unsigned short *__restrict__ gh,
    const int *__restrict__ candlen, int *__restrict__ candoff_out,
    unsigned long long *__restrict__ ckey, int *__restrict__ cslot, const long long *__restrict__ gcut,
    const unsigned int *__restrict__ spec, const int *__restrict__ specn, const int *__restrict__ pbase,
    const int *__restrict__ pwide, DevCounters *ctr, unsigned int *__restrict__ crank, int *__restrict__ lv,
    unsigned char *__restrict__ rtype, int R, const int bid_, const int nbk_, unsigned long long *kst = nullptr) {
    constexpr int RT = TB <= RANK_FAST_T ? TB : 1;  // types of the fast ranking
    kstamp(kst, bid_, 0);
    extern __shared__ unsigned int lds[];  // wc[4][C], then list[4][1024]
    __shared__ long long sanc[ADLBQ_MAX_TYPES], scut[ADLBQ_MAX_TYPES];
    __shared__ int sth[ADLBQ_MAX_TYPES], sneed[ADLBQ_MAX_TYPES], soff[ADLBQ_MAX_TYPES], slen[RT];
    __shared__ int slb[TB <= 8 ? TB : 1];  // pass 1's lump bins (T <= 8)
    __shared__ int sbo[RT * NB];  // binoff (fast ranking)
    const int C = T * NB, w = threadIdx.x >> 6, lane = threadIdx.x & 63, p = bid_;
    unsigned int *wc = lds;
    unsigned int *list = lds + 4 * C + w * 1024;
    const long long base = (long long)pages[p] << PAGE_SHIFT;
    const int fill = (p == npages - 1) ? tail_fill : PAGE;
    // Pass 1's speculative list of this wave's quarter is usable when it did
    // not overflow and, for every type with demand, the guessed cut is at or
    // below the real one (lane t checks type t; T <= 64): then the list holds
    // every candidate and the page's columns are not read again.
    // All of the prologue's loads are issued together: lane t's type-t
    // parameters, the list (read whether or not it is used) and, below, the
    // page prefix rows.
    const bool tl = lane < T;
    const int th_l = tl ? theta[lane] : -1, nd_l = tl ? need[lane] : 0, len_l = tl ? candlen[lane] : 0;
    const long long an_l = tl ? anchor[lane] : 0, gc_l = tl ? gcut[lane] : 0;
    const int sn = specn[(long long)p * 4 + w];
    // binoff for the fast ranking (T <= 8: at most two columns per thread), in flight with the rest
    int bo_r[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const int c = threadIdx.x + q * 256;
        bo_r[q] = (TB <= RANK_FAST_T && crank != nullptr && c < C) ? binoff[c] : 0;
    }
    const unsigned int *__restrict__ sp = spec + ((long long)p * 4 + w) * SPEC_CAP;
    unsigned int se[SPEC_CAP / 64];
#pragma unroll
    for (int k = 0; k < SPEC_CAP / 64; k++) se[k] = sp[k * 64 + lane];
    const long long cut_l = cut_of(th_l, an_l);
    // T <= 8: the list holds every unit above its type's lump, usable when no
    // threshold lies in a lump; otherwise every unit at or above the guessed cut
    const int lb_l = (TB <= 8 && tl) ? lump_bin(an_l, gc_l) : NB;
    const bool use_spec = (TB <= 8 ? __ballot(th_l >= 0 && th_l >= lb_l) : __ballot(th_l >= 0 && gc_l > cut_l)) == 0 &&
                          sn <= SPEC_CAP;  // wave-uniform
    int4 pv[4];
    uint4 mv[4];
    if (!use_spec) load_quarter(prio, meta, pbase, pwide, pages[p], fill, w, pv, mv);
    // diagnostic: 1 used; else -(entries) when the list overflowed, or -100000 - (a type whose threshold passed the list)
    if (p == 0 && threadIdx.x < 64) {
        const unsigned long long bad = TB <= 8 ? __ballot(th_l >= 0 && th_l >= lb_l) : __ballot(th_l >= 0 && gc_l > cut_l);
        if (threadIdx.x == 0)
            ctr->spec_page0 = use_spec ? 1 : sn > SPEC_CAP ? -sn : -100000 - (bad ? __ffsll((long long)bad) - 1 : 99);
    }
    // rank of this page's first unit in each of the thread's columns (only
    // columns at or below a threshold): the chunk's exclusive prefix
    // (k_thresholds) plus the counts of the chunk's earlier pages (hist_page)
    constexpr int CPT = (ADLBQ_MAX_TYPES * NB) / 256;  // columns per thread, at most
    unsigned int ppv[CPT];
    const int p0 = (p / CHUNK) * CHUNK;
#pragma unroll
    for (int r = 0; r < CPT; r++) {
        const int c = threadIdx.x + r * 256;
        ppv[r] = 0;
        if (r * 256 >= C) break;
        const int thc = __shfl(th_l, (c / NB) & 63, 64);
        if (c < C && (c % NB) <= thc) {
            const int nch = (npages + CHUNK - 1) / CHUNK;  // the tile prefixes follow the chunk sums
            unsigned int v = csum[(long long)(p / CHUNK) * C + c] + csum[(long long)(nch + p / CHUNK / TH_ROWS) * C + c];
            unsigned short g[CHUNK - 1];
#pragma unroll
            for (int q = 0; q < CHUNK - 1; q++) g[q] = p0 + q < p ? gh[(long long)(p0 + q) * C + c] : (unsigned short)0;
#pragma unroll
            for (int q = 0; q < CHUNK - 1; q++) v += g[q];
            ppv[r] = v;
        }
    }
    if (w == 0 && tl) {
        sanc[lane] = an_l;
        sth[lane] = th_l;
        sneed[lane] = nd_l;
        scut[lane] = cut_l;
        if (lane < RT) slen[lane] = len_l;
        if (TB <= 8 && lane < TB) slb[lane] = lb_l;
    }
    // ranks computed here (k_rank then skips its tiles) when every threshold
    // lies in an exact bin: every candidate list is then in (prio desc,
    // position asc) order by construction, and a unit of another type u with
    // the same prio precedes this one iff it lies earlier in the open bucket
    const bool fast = TB <= RANK_FAST_T && crank != nullptr && __ballot(tl && th_l >= NBX) == 0;
    if (fast)  // binoff (only read for the types with demand, the ones k_thresholds wrote it for)
#pragma unroll
        for (int q = 0; q < 2; q++)
            if (threadIdx.x + q * 256 < C) sbo[threadIdx.x + q * 256] = bo_r[q];
    for (int c = threadIdx.x; c < 4 * C; c += blockDim.x) wc[c] = 0;
    if (threadIdx.x < 64) {  // candidate list offsets: exclusive prefix of candlen over types
        const int len = len_l;
        int x = len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (threadIdx.x >= o) x += y;
        }
        if (threadIdx.x < T) soff[threadIdx.x] = x - len;
        if (p == 0 && threadIdx.x < T) candoff_out[threadIdx.x] = x - len;
        if (p == 0 && threadIdx.x == T - 1) candoff_out[T] = x;
    }
    __syncthreads();
    kstamp(kst, bid_, 1);
    int n = 0;  // this wave's candidates so far (uniform)
    const unsigned long long lt = lanemask_lt();
    if (use_spec) {  // filter the list: entries in bins up to the type's threshold
#pragma unroll
        for (int k = 0; k < SPEC_CAP / 64; k++) {
            if (k * 64 >= sn) break;
            const unsigned int e = se[k];
            const int col = (int)(e >> 12), ct = col / NB;
            const bool c = k * 64 + lane < sn && col - ct * NB <= sth[ct];
            const unsigned long long b = __ballot(c);
            if (c) {
                list[n + __popcll(b & lt)] = e;
                atomicAdd(&wc[w * C + col], 1u);
            }
            n += __popcll(b);
        }
    } else
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int pr[4] = {pv[k].x, pv[k].y, pv[k].z, pv[k].w};
        const uint32_t mm[4] = {mv[k].x, mv[k].y, mv[k].z, mv[k].w};
        bool cnd[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            cnd[q] = (mm[q] & (M_LIVE | M_PINNED)) == M_LIVE && (long long)pr[q] >= scut[mm[q] & M_TYPE];
        const unsigned long long b0 = __ballot(cnd[0]), b1 = __ballot(cnd[1]), b2 = __ballot(cnd[2]),
                                 b3 = __ballot(cnd[3]);
        if (!(b0 | b1 | b2 | b3)) continue;
        int pos = n + __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (cnd[q]) {
                const int t = mm[q] & M_TYPE;
                const int bq = bin_of(sanc[t] - pr[q]);
                const int col = t * NB + ((TB <= 8 && bq >= slb[t]) ? NB - 1 : bq);  // pass 1's lump
                atomicAdd(&wc[w * C + col], 1u);
                list[pos++] = ((unsigned int)col << 12) | (unsigned int)((w * 4 + k) * 256 + lane * 4 + q);
            }
        }
        n += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < CPT; r++) {
        const int c = threadIdx.x + r * 256;
        if (c < C && (c % NB) <= sth[c / NB]) {
            unsigned int run = ppv[r];
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const unsigned int x = wc[v * C + c];
                wc[v * C + c] = run;
                run += x;
            }
        }
    }
    __syncthreads();
    kstamp(kst, bid_, 2);
    unsigned int *run = wc + w * C;
    // the fast ranking's per-type constants, uniform over the wave (from LDS once)
    long long an_u[RT];
    int th_u[RT], nd_u[RT], len_u[RT];
    if (fast) {
#pragma unroll
        for (int u = 0; u < RT; u++) {
            const bool ok = u < T;
            an_u[u] = ok ? sanc[u] : 0;
            th_u[u] = ok ? sth[u] : -1;
            nd_u[u] = ok ? sneed[u] : 0;
            len_u[u] = ok ? slen[u] : 0;
        }
    }
    for (int i0 = 0; i0 < n; i0 += 64) {
        const int i = i0 + lane;
        const unsigned int e = i < n ? list[i] : 0u;
        const int col = (int)(e >> 12), so = (int)(e & (PAGE - 1));
        // key order = (prio desc, position in the open bucket asc): the bucket
        // holds its units in wqseqno order, so this is the reference's order.
        // An exact bin fixes the prio (anchor - bin); only a multi-prio bin reads it.
        const int ct = col / NB, cb = col - ct * NB;
        const int pr = i >= n ? 0 : cb < NBX ? (int)(sanc[ct] - cb) : prio[base + so];
        const unsigned int bpos = ((unsigned int)p << PAGE_SHIFT) | (unsigned int)so;
        // fast ranking: per type u, the column holding prio pr (exact bins at
        // or below u's threshold), else -1 (u has no unit of prio pr among its
        // candidates: all of them are better, or none)
        int tcol[RT], cnt[RT];
        if (fast) {
#pragma unroll
            for (int u = 0; u < RT; u++) {
                const long long bu = an_u[u] - (long long)pr;
                tcol[u] = (bu >= 0 && bu <= th_u[u]) ? u * NB + (int)bu : -1;
                cnt[u] = 0;
            }
        }
        // earlier lanes of this step with a given column: one ballot per column bit, then per
        // wanted column x the AND of B_b or ~B_b by x's bits (no 64-step walk over the lanes)
        constexpr int CBITS = TB <= 4 ? 8 : TB <= 8 ? 9 : 12;  // bits of a column index (T * NB columns)
        unsigned long long cb_[CBITS];
#pragma unroll
        for (int b = 0; b < CBITS; b++) cb_[b] = __ballot((col >> b) & 1);
        const unsigned long long vm = __ballot(i < n) & lt;
        auto earlier_in = [&](int x) {
            unsigned long long m = vm;
#pragma unroll
            for (int b = 0; b < CBITS; b++) m &= ((x >> b) & 1) ? cb_[b] : ~cb_[b];
            return __popcll(m);
        };
        const int rank = earlier_in(col);
        if (fast) {
#pragma unroll
            for (int u = 0; u < RT; u++) cnt[u] = tcol[u] >= 0 ? earlier_in(tcol[u]) : 0;
        }
        if (i < n) {
            const unsigned int r = run[col] + rank;
            const int t = col / NB, b = col - t * NB;
            if (b < sth[t] || b >= NBX || (int)r < sneed[t]) {  // exact threshold bin: its first `need` only
                const long long at = (long long)soff[t] + binoff[col] + r;
                ckey[at] = make_key(pr, bpos);
                cslot[at] = (int)(base + so);
                if (fast) {
                    // global rank: per type u, its candidates better than this one
                    int lb[RT], g = 0;
#pragma unroll
                    for (int u = 0; u < RT; u++) {
                        lb[u] = 0;
                        if (tcol[u] >= 0) {
                            int c = (int)run[tcol[u]] + cnt[u];  // units of prio pr earlier in the bucket
                            if (tcol[u] - u * NB == th_u[u]) c = min(c, nd_u[u]);  // the threshold bin's first `need`
                            lb[u] = sbo[tcol[u]] + c;
                        } else if (an_u[u] >= (long long)pr) {
                            lb[u] = len_u[u];  // every candidate of u is better
                        }
                        g += lb[u];
                    }
                    crank[at] = ((unsigned int)g << 6) | (unsigned int)t;
                    if (lv != nullptr && g < R) rtype[g] = (unsigned char)t;
                    // level rows, sampled every LV_STEP ranks (rtype completes them between samples)
                    if (lv != nullptr && (g & (LV_STEP - 1)) == 0 && g < R)
#pragma unroll
                        for (int u = 0; u < RT; u++)
                            if (u < T) lv[(long long)(g / LV_STEP) * T + u] = lb[u];
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (i < n) atomicAdd(&run[col], 1u);  // after every lane of the step has read run[]
        __builtin_amdgcn_wave_barrier();
    }
    if (fast && p == 0 && threadIdx.x == 0) ctr->rank_fast = 1;
    if (!fast && crank != nullptr && p == 0 && threadIdx.x == 0) ctr->rank_fast = 0;
    // the next batch's hint for skipping k_rank: ranked here, and every type has candidates
    const bool empty = __ballot(tl && len_l <= 0) != 0ull;
    if (crank != nullptr && p == 0 && threadIdx.x == 0) ctr->rank_covered = (fast && !empty) ? 1 : 0;
    if (kst) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        kstamp(kst, bid_, 3);
    }
}

// Pass 2 with one wave per page (T <= 8): the page's four quarter lists in
// slot order, one after the other, against one running count per column
// (the page's prefix, then each list's candidates as they are ranked).  With
// 64-thread workgroups every page is resident at once (2,442 pages at the
// metric size against ~4,000 such workgroups), where k_select_open's
// four-wave workgroups ran in two rounds (82 VGPRs, 20 KB of LDS each).
// Results as k_select_open's.
#ifndef ADLBQ_SELW_LAZY
#define ADLBQ_SELW_LAZY 1  // k_select_wave reads a list's second 64 entries only when it has them
#endif
#ifndef ADLBQ_SELW_GATE
#define ADLBQ_SELW_GATE 1  // k_select_wave reads a column's page prefix only at or below its threshold
#endif
template <int TB>
__device__ __forceinline__ void select_wave_body(
    const int *__restrict__ pages, int npages, int tail_fill, const int *__restrict__ prio,
    const uint32_t *__restrict__ meta, int T, const long long *__restrict__ anchor,
    const int *__restrict__ theta, const int *__restrict__ need,
    const int *__restrict__ binoff, const unsigned int *__restrict__ csum, const unsigned short *__restrict__ gh,
    const int *__restrict__ candlen, int *__restrict__ candoff_out,
    unsigned long long *__restrict__ ckey, int *__restrict__ cslot, const long long *__restrict__ gcut,
    const unsigned int *__restrict__ spec, const int *__restrict__ specn, const int *__restrict__ pbase,
    const int *__restrict__ pwide, DevCounters *ctr, unsigned int *__restrict__ crank, int *__restrict__ lv,
    unsigned char *__restrict__ rtype, int R,
    unsigned long long *kst, const int p) {
    static_assert(TB <= 8 && TB <= RANK_FAST_T, "one wave per page: T <= 8");
    constexpr int RT = TB;
    constexpr int CPL = TB * NB / 64;  // columns per lane
    extern __shared__ unsigned int lds[];  // run[C], then list[1024]
    __shared__ long long sanc[TB], scut[TB];
    __shared__ int sth[TB], sneed[TB], soff[TB], slen[TB], slb[TB];
    __shared__ int sbo[TB * NB];
    const int C = T * NB, lane = threadIdx.x;
    kstamp(kst, p, 0);
    unsigned int *run = lds;
    unsigned int *list = lds + C;
    const long long base = (long long)pages[p] << PAGE_SHIFT;
    const int fill = (p == npages - 1) ? tail_fill : PAGE;
    const bool tl = lane < T;
    const int th_l = tl ? theta[lane] : -1, nd_l = tl ? need[lane] : 0, len_l = tl ? candlen[lane] : 0;
    const long long an_l = tl ? anchor[lane] : 0, gc_l = tl ? gcut[lane] : 0;
    int sn[4];
#pragma unroll
    for (int q = 0; q < 4; q++) sn[q] = specn[(long long)p * 4 + q];
    int bo_r[CPL];
#pragma unroll
    for (int r = 0; r < CPL; r++) {
        const int c = lane + r * 64;
        bo_r[r] = (crank != nullptr && c < C) ? binoff[c] : 0;
    }
    unsigned int se[4][SPEC_CAP / 64];
#pragma unroll
    for (int q = 0; q < 4; q++) se[q][0] = spec[((long long)p * 4 + q) * SPEC_CAP + lane];
    const long long cut_l = cut_of(th_l, an_l);
    const int lb_l = tl ? lump_bin(an_l, gc_l) : NB;
    const bool lists_ok = __ballot(th_l >= 0 && th_l >= lb_l) == 0;  // no threshold in a lump
    if (p == 0 && lane == 0) ctr->spec_page0 = lists_ok && sn[0] <= SPEC_CAP ? 1 : sn[0] > SPEC_CAP ? -sn[0] : -100000;
    // the page's first rank in each column at or below its threshold: the chunk's
    // exclusive prefix plus the counts of the chunk's earlier pages
    unsigned int ppv[CPL];
    const int p0 = (p / CHUNK) * CHUNK;
#pragma unroll
    for (int r = 0; r < CPL; r++) {
        // every lane loads (a column past the threshold or the list reads column 0 of the same rows: one
        // line, no traffic to speak of) and masks after: loads under a branch were issued one column
        // group at a time
        const int c = lane + r * 64;
        const int thc = __shfl(th_l, (c / NB) & 63, 64);
        const bool use = c < C && (c % NB) <= thc;
        const int cc = (ADLBQ_SELW_GATE ? use : c < C) ? c : 0;  // ungated: the loads need not wait for theta
        const int nch = (npages + CHUNK - 1) / CHUNK;  // the tile prefixes follow the chunk sums
        const unsigned int v0 = csum[(long long)(p / CHUNK) * C + cc],
                           v1 = csum[(long long)(nch + p / CHUNK / TH_ROWS) * C + cc];
        unsigned int g[CHUNK - 1];
#pragma unroll
        for (int q = 0; q < CHUNK - 1; q++) g[q] = gh[(long long)(p0 + q < p ? p0 + q : p0) * C + cc];
        unsigned int km = use ? ~0u : 0u, gm = 0u;  // opaque to the optimiser (no select sunk into a branch)
#pragma unroll
        for (int q = 0; q < CHUNK - 1; q++) gm |= (p0 + q < p ? 1u : 0u) << q;
        asm volatile("" : "+v"(km), "+v"(gm));
        unsigned int v = v0 + v1;
#pragma unroll
        for (int q = 0; q < CHUNK - 1; q++) v += g[q] & (0u - ((gm >> q) & 1u));
        ppv[r] = v & km;
    }
    // the lists' further entries: read when the list is that long (rarely; a list is
    // typically a few dozen entries at the metric size)
#pragma unroll
    for (int q = 0; q < 4; q++)
#pragma unroll
        for (int k = 1; k < SPEC_CAP / 64; k++)
            se[q][k] = (!ADLBQ_SELW_LAZY || sn[q] > k * 64) ? spec[((long long)p * 4 + q) * SPEC_CAP + k * 64 + lane] : 0u;
    if (tl) {
        sanc[lane] = an_l;
        sth[lane] = th_l;
        sneed[lane] = nd_l;
        scut[lane] = cut_l;
        slen[lane] = len_l;
        slb[lane] = lb_l;
    }
    const bool fast = crank != nullptr && __ballot(tl && th_l >= NBX) == 0;
#pragma unroll
    for (int r = 0; r < CPL; r++) {
        const int c = lane + r * 64;
        if (c < C) {
            run[c] = ppv[r];
            if (fast) sbo[c] = bo_r[r];
        }
    }
    {  // candidate list offsets: exclusive prefix of candlen over types
        int x = len_l;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (tl) soff[lane] = x - len_l;
        if (p == 0 && tl) candoff_out[lane] = x - len_l;
        if (p == 0 && lane == T - 1) candoff_out[T] = x;
    }
    __syncthreads();
    kstamp(kst, p, 1);
    long long an_u[RT];
    int th_u[RT], nd_u[RT], len_u[RT];
#pragma unroll
    for (int u = 0; u < RT; u++) {
        const bool ok = u < T;
        an_u[u] = ok ? sanc[u] : 0;
        th_u[u] = ok ? sth[u] : -1;
        nd_u[u] = ok ? sneed[u] : 0;
        len_u[u] = ok ? slen[u] : 0;
    }
    const unsigned long long lt = lanemask_lt();
    // The quarters' candidates in slot order, listed together and ranked in one
    // go when they are pass 1's lists (at most 4 * SPEC_CAP entries; typically
    // one 64-wide step for the page), a quarter read again ranked on its own.
    int n = 0, w = 0;
#pragma unroll 1
    while (true) {
        bool rank_now = w == 4;
        if (w < 4) {
            int snw = sn[0];
#pragma unroll
            for (int q = 1; q < 4; q++)
                if (w == q) snw = sn[q];
            const bool sp = lists_ok && snw <= SPEC_CAP;
            if (!sp && n > 0) {
                rank_now = true;  // rank what is listed before the quarter is read again
            } else if (sp) {  // pass 1's list, filtered by the thresholds
#pragma unroll
                for (int k = 0; k < SPEC_CAP / 64; k++) {
                    if (k * 64 >= snw) break;
                    unsigned int e = se[0][k];
#pragma unroll
                    for (int q = 1; q < 4; q++)
                        if (w == q) e = se[q][k];
                    const int col = (int)(e >> 12), ct = col / NB;
                    const bool c = k * 64 + lane < snw && col - ct * NB <= sth[ct];
                    const unsigned long long b = __ballot(c);
                    if (c) list[n + __popcll(b & lt)] = e;
                    n += __popcll(b);
                }
            } else {  // the quarter's columns read again
                int4 pv[4];
                uint4 mv[4];
                load_quarter(prio, meta, pbase, pwide, pages[p], fill, w, pv, mv);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int pr[4] = {pv[k].x, pv[k].y, pv[k].z, pv[k].w};
                    const uint32_t mm[4] = {mv[k].x, mv[k].y, mv[k].z, mv[k].w};
                    bool cnd[4];
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        cnd[q] = (mm[q] & (M_LIVE | M_PINNED)) == M_LIVE && (long long)pr[q] >= scut[mm[q] & M_TYPE];
                    const unsigned long long b0 = __ballot(cnd[0]), b1 = __ballot(cnd[1]), b2 = __ballot(cnd[2]),
                                             b3 = __ballot(cnd[3]);
                    if (!(b0 | b1 | b2 | b3)) continue;
                    int pos = n + __popcll(b0 & lt) + __popcll(b1 & lt) + __popcll(b2 & lt) + __popcll(b3 & lt);
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if (cnd[q]) {
                            const int t = mm[q] & M_TYPE;
                            const int bq = bin_of(sanc[t] - pr[q]);
                            const int col = t * NB + (bq >= slb[t] ? NB - 1 : bq);  // pass 1's lump
                            list[pos++] = ((unsigned int)col << 12) | (unsigned int)((w * 4 + k) * 256 + lane * 4 + q);
                        }
                    }
                    n += __popcll(b0) + __popcll(b1) + __popcll(b2) + __popcll(b3);
                }
            }
            if (!rank_now) {
                w++;
                rank_now = !sp || w == 4;
            }
        }
        if (!rank_now) continue;
        if (w == 4) kstamp(kst, p, 2);
        __builtin_amdgcn_wave_barrier();  // one wave: its LDS operations complete in order
        for (int i0 = 0; i0 < n; i0 += 64) {
            const int i = i0 + lane;
            const unsigned int e = i < n ? list[i] : 0u;
            const int col = (int)(e >> 12), so = (int)(e & (PAGE - 1));
            const int ct = col / NB, cb = col - ct * NB;
            const int pr = i >= n ? 0 : cb < NBX ? (int)(sanc[ct] - cb) : prio[base + so];
            const unsigned int bpos = ((unsigned int)p << PAGE_SHIFT) | (unsigned int)so;
            int tcol[RT], cnt[RT];
            if (fast) {
#pragma unroll
                for (int u = 0; u < RT; u++) {
                    const long long bu = an_u[u] - (long long)pr;
                    tcol[u] = (bu >= 0 && bu <= th_u[u]) ? u * NB + (int)bu : -1;
                    cnt[u] = 0;
                }
            }
            constexpr int CBITS = TB <= 4 ? 8 : 9;  // bits of a column index (T * NB columns)
            unsigned long long cb_[CBITS];
#pragma unroll
            for (int b = 0; b < CBITS; b++) cb_[b] = __ballot((col >> b) & 1);
            const unsigned long long vm = __ballot(i < n) & lt;
            auto earlier_in = [&](int x) {
                unsigned long long m = vm;
#pragma unroll
                for (int b = 0; b < CBITS; b++) m &= ((x >> b) & 1) ? cb_[b] : ~cb_[b];
                return __popcll(m);
            };
            const int rank = earlier_in(col);
            if (fast) {
#pragma unroll
                for (int u = 0; u < RT; u++) cnt[u] = tcol[u] >= 0 ? earlier_in(tcol[u]) : 0;
            }
            if (i < n) {
                const unsigned int r = run[col] + rank;
                const int t = col / NB, b = col - t * NB;
                if (b < sth[t] || b >= NBX || (int)r < sneed[t]) {  // exact threshold bin: its first `need` only
                    const long long at = (long long)soff[t] + binoff[col] + r;
                    ckey[at] = make_key(pr, bpos);
                    cslot[at] = (int)(base + so);
                    if (fast) {
                        int lb[RT], g = 0;
#pragma unroll
                        for (int u = 0; u < RT; u++) {
                            lb[u] = 0;
                            if (tcol[u] >= 0) {
                                int c = (int)run[tcol[u]] + cnt[u];
                                if (tcol[u] - u * NB == th_u[u]) c = min(c, nd_u[u]);
                                lb[u] = sbo[tcol[u]] + c;
                            } else if (an_u[u] >= (long long)pr) {
                                lb[u] = len_u[u];
                            }
                            g += lb[u];
                        }
                        crank[at] = ((unsigned int)g << 6) | (unsigned int)t;
                        if (lv != nullptr && g < R) rtype[g] = (unsigned char)t;
                        if (lv != nullptr && (g & (LV_STEP - 1)) == 0 && g < R)
#pragma unroll
                            for (int u = 0; u < RT; u++)
                                if (u < T) lv[(long long)(g / LV_STEP) * T + u] = lb[u];
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (i < n) atomicAdd(&run[col], 1u);  // after every lane of the step has read run[]
            __builtin_amdgcn_wave_barrier();
        }
        n = 0;
        if (w == 4) break;
    }
    kstamp(kst, p, 3);
    if (p == 0 && lane == 0) ctr->rank_fast = fast ? 1 : 0;
    const bool empty = __ballot(tl && len_l <= 0) != 0ull;
    if (crank != nullptr && p == 0 && lane == 0) ctr->rank_covered = (fast && !empty) ? 1 : 0;
}

template <int TB>
__global__ __launch_bounds__(64) void k_select_wave(
    const int *__restrict__ pages, int npages, int tail_fill, const int *__restrict__ prio,
    const uint32_t *__restrict__ meta, int T, const long long *__restrict__ anchor,
    const int *__restrict__ theta, const int *__restrict__ need,
    const int *__restrict__ binoff, const unsigned int *__restrict__ csum, const unsigned short *__restrict__ gh,
    const int *__restrict__ candlen, int *__restrict__ candoff_out,
    unsigned long long *__restrict__ ckey, int *__restrict__ cslot, const long long *__restrict__ gcut,
    const unsigned int *__restrict__ spec, const int *__restrict__ specn, const int *__restrict__ pbase,
    const int *__restrict__ pwide, DevCounters *ctr, unsigned int *__restrict__ crank, int *__restrict__ lv,
    unsigned char *__restrict__ rtype, int R,
    unsigned long long *kst) {
    select_wave_body<TB>(pages, npages, tail_fill, prio, meta, T, anchor, theta, need, binoff, csum, gh, candlen,
                         candoff_out, ckey, cslot, gcut, spec, specn, pbase, pwide, ctr, crank, lv, rtype, R, kst,
                         blockIdx.x);
}

template <int TB>  // TB >= T; the candidates are ranked here only for TB <= RT
__global__ __launch_bounds__(256) void k_select_open(
    const int *__restrict__ pages, int npages, int tail_fill, const int *__restrict__ prio,
    const uint32_t *__restrict__ meta, const int *__restrict__ seqa, int T, const long long *__restrict__ anchor,
    const int *__restrict__ theta, const int *__restrict__ need,
    const int *__restrict__ binoff, const unsigned int *__restrict__ csum, const unsigned short *__restrict__ gh,
    const int *__restrict__ candlen, int *__restrict__ candoff_out,
    unsigned long long *__restrict__ ckey, int *__restrict__ cslot, const long long *__restrict__ gcut,
    const unsigned int *__restrict__ spec, const int *__restrict__ specn, const int *__restrict__ pbase,
    const int *__restrict__ pwide, DevCounters *ctr, unsigned int *__restrict__ crank, int *__restrict__ lv,
    unsigned char *__restrict__ rtype, int R, unsigned long long *kst) {
    select_open_body<TB>(pages, npages, tail_fill, prio, meta, seqa, T, anchor, theta, need, binoff, csum, gh, candlen, candoff_out, ckey, cslot, gcut, spec, specn, pbase, pwide, ctr, crank, lv, rtype, R, blockIdx.x, gridDim.x, kst);
}

// ---------------------------------------------------------------- per-type sort (multi-priority bins only)
constexpr int SORT_BLK = 2048;  // entries per LDS bitonic block of sort_type
__device__ inline void bitonic_desc_blk(unsigned long long *sk, int *ss) {
    for (int k = 2; k <= SORT_BLK; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < SORT_BLK; i += blockDim.x) {
                int ixj = i ^ j;
                if (ixj > i) {
                    unsigned long long a = sk[i], b = sk[ixj];
                    bool sw = ((i & k) == 0) ? (a < b) : (a > b);
                    if (sw) {
                        sk[i] = b;
                        sk[ixj] = a;
                        int t = ss[i];
                        ss[i] = ss[ixj];
                        ss[ixj] = t;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// Type t's candidate list by key, descending: SORT_BLK-entry bitonic blocks in
// LDS (sk, ss), then pairwise merges through key2/slot2.  Any block size.
__device__ void sort_type(const int off, const int n, unsigned long long *key, int *slot, unsigned long long *key2,
                          int *slot2, unsigned long long *sk, int *ss) {
    for (int c0 = 0; c0 < n; c0 += SORT_BLK) {
        const int m = min(SORT_BLK, n - c0);
        for (int i = threadIdx.x; i < SORT_BLK; i += blockDim.x) {
            sk[i] = i < m ? key[off + c0 + i] : 0ull;
            ss[i] = i < m ? slot[off + c0 + i] : -1;
        }
        __syncthreads();
        bitonic_desc_blk(sk, ss);
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            key[off + c0 + i] = sk[i];
            slot[off + c0 + i] = ss[i];
        }
        __syncthreads();
    }
    if (n <= SORT_BLK) return;
    __threadfence();
    __syncthreads();
    unsigned long long *sK = key + off, *dK = key2 + off;
    int *sS = slot + off, *dS = slot2 + off;
    constexpr int ITEMS = 4;
    for (long long wdt = SORT_BLK; wdt < n; wdt *= 2) {
        for (long long a0 = 0; a0 < n; a0 += 2 * wdt) {
            const long long na = min((long long)n - a0, wdt);
            const long long nb = max(0ll, min((long long)n - a0 - wdt, wdt));
            const unsigned long long *A = sK + a0, *B = sK + a0 + na;
            const int *AS = sS + a0, *BS = sS + a0 + na;
            const long long tot = na + nb;
            for (long long o0 = 0; o0 < tot; o0 += (long long)blockDim.x * ITEMS) {
                const long long d = o0 + (long long)threadIdx.x * ITEMS;
                if (d >= tot) continue;
                long long lo = max(0ll, d - nb), hi = min(d, na);
                while (lo < hi) {  // number of A elements among the first d outputs
                    long long mid = (lo + hi) >> 1;
                    if (A[mid] >= B[d - 1 - mid]) lo = mid + 1;
                    else hi = mid;
                }
                long long i = lo, j = d - lo;
                for (int e = 0; e < ITEMS && d + e < tot; e++) {
                    bool takeA = j >= nb || (i < na && A[i] >= B[j]);
                    if (takeA) {
                        dK[a0 + d + e] = A[i];
                        dS[a0 + d + e] = AS[i];
                        i++;
                    } else {
                        dK[a0 + d + e] = B[j];
                        dS[a0 + d + e] = BS[j];
                        j++;
                    }
                }
            }
        }
        __threadfence();
        __syncthreads();
        unsigned long long *tk = sK; sK = dK; dK = tk;
        int *ts = sS; sS = dS; dS = ts;
    }
    if (sK != key + off) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            key[off + i] = sK[i];
            slot[off + i] = sS[i];
        }
    }
}

// Export path only (a reserve batch sorts inside k_rank).
__global__ __launch_bounds__(1024) void k_sort_types(const int *__restrict__ needsort, const int *__restrict__ candoff,
                                                     const int *__restrict__ candlen, unsigned long long *key,
                                                     int *slot, unsigned long long *key2, int *slot2) {
    const int t = blockIdx.x;
    if (!needsort[t] || candlen[t] <= 1) return;
    __shared__ unsigned long long sk[SORT_BLK];
    __shared__ int ss[SORT_BLK];
    sort_type(candoff[t], candlen[t], key, slot, key2, slot2, sk, ss);
}

// ---------------------------------------------------------------- targeted phase
__global__ __launch_bounds__(256) void k_targeted(const int *__restrict__ bucket_ranks, const int *__restrict__ pstart,
                                                  const int *__restrict__ rpages, const int *__restrict__ rfill,
                                                  const int *__restrict__ prio, uint32_t *meta,
                                                  const unsigned long long *__restrict__ mask,
                                                  const int *__restrict__ reqs, int R, int *tmatch,
                                                  int *seg_cnt) {
    __shared__ int list[1024];
    __shared__ int nlist, wcnt[4];
    __shared__ unsigned long long red[4];
    const int b = blockIdx.x, r = bucket_ranks[b], p0 = pstart[b], np = pstart[b + 1] - p0;
    if (np <= 0) return;
    const long long total = (long long)(np - 1) * PAGE + rfill[b];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) nlist = 0;
    __syncthreads();
    for (int j0 = 0; j0 < R; j0 += 256) {
        const int j = j0 + threadIdx.x;
        const bool is = j < R && reqs[(long long)ADLBQ_RESERVE_INTS * j] == r;
        const unsigned long long bal = __ballot(is);
        if (lane == 0) wcnt[w] = __popcll(bal);
        __syncthreads();
        int woff = nlist;
        for (int q = 0; q < w; q++) woff += wcnt[q];
        if (is) list[woff + __popcll(bal & lanemask_lt())] = j;
        __syncthreads();
        if (threadIdx.x == 0) nlist += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
        __syncthreads();
        if (nlist > 768 || j0 + 256 >= R) {
            for (int e = 0; e < nlist; e++) {
                const int jj = list[e];
                const unsigned long long m = mask[jj];
                unsigned long long best = 0;
                for (long long L = threadIdx.x; L < total; L += blockDim.x) {
                    const long long slot = ((long long)rpages[p0 + (L >> PAGE_SHIFT)] << PAGE_SHIFT) + (L & (PAGE - 1));
                    const uint32_t mt = (uint32_t)ld_agent(reinterpret_cast<const int *>(meta + slot));
                    if ((mt & (M_LIVE | M_PINNED)) != M_LIVE) continue;
                    if (!((m >> (mt & M_TYPE)) & 1ull)) continue;
                    const int pr = prio[slot];
                    if (pr <= LOWEST) continue;
                    const unsigned long long k = make_key(pr, (unsigned int)L);
                    best = k > best ? k : best;
                }
                best = wave_max_u64(best);
                if (lane == 0) red[w] = best;
                __syncthreads();
                if (threadIdx.x == 0) {
                    unsigned long long bb = red[0];
                    for (int q = 1; q < 4; q++) bb = red[q] > bb ? red[q] : bb;
                    if (bb) {
                        const long long L = (long long)(~(unsigned int)(bb & 0xffffffffu));
                        const long long slot =
                            ((long long)rpages[p0 + (L >> PAGE_SHIFT)] << PAGE_SHIFT) + (L & (PAGE - 1));
                        tmatch[jj] = (int)slot;
                        atomicSub(&seg_cnt[jj >> 6], 1);
                        // taken for this rank's later Reserves (this block owns the bucket): a write-through
                        // store, drained before the barrier; the block's scans read meta with sc1 loads
                        st_agent(reinterpret_cast<int *>(meta + slot), (int)(meta[slot] | M_PINNED));
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                }
                __syncthreads();
            }
            if (threadIdx.x == 0) nlist = 0;
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------- targeted phase over a sorted index
// The pre-targeted match (wq_find_pre_targeted_hi_prio, xq.c:219-247) of a
// rank's Reserves, in order, against that rank's bucket.  Instead of one scan
// of the bucket per Reserve, the bucket's units are kept in an index sorted
// by (bucket, type, prio desc, bucket position asc) -- one stable radix sort,
// rebuilt only after targeted Puts (k_tindex_keys, rsx_sort_pairs) -- with the range
// of every (bucket, type) as lower bounds (k_tindex_bounds; after an
// incremental merge, k_tindex_shift).  A Reserve's best unit is then
// the best head among its types' ranges: lane t of wave 0 keeps type t's
// head, skips units no longer available (pinned, deleted, prio <= LOWEST),
// and the wave takes the minimum of (prio desc, position asc).
constexpr int TIDX_TYPE_BITS = 6, TIDX_PRIO_BITS = 32;
constexpr int TIDX_BUCKET_SHIFT = TIDX_TYPE_BITS + TIDX_PRIO_BITS;  // bucket index above type and prio
constexpr int TIDX_KEY_BITS = TIDX_BUCKET_SHIFT + 20;               // buckets < 2^20

__global__ __launch_bounds__(256) void k_tindex_keys(const int *__restrict__ pstart, const int *__restrict__ rpages,
                                                     const int *__restrict__ rfill, int nb,
                                                     const int *__restrict__ prio, const uint32_t *__restrict__ meta,
                                                     unsigned long long *keys, int *vals) {
    // block = one page of the concatenated rank-bucket page list
    const int gp = blockIdx.x;
    int lo = 0, hi = nb;  // bucket b with pstart[b] <= gp < pstart[b+1]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pstart[mid] <= gp) lo = mid; else hi = mid;
    }
    const int b = lo, pi = gp - pstart[b], last = pstart[b + 1] - 1;
    const int fill = gp == last ? rfill[b] : PAGE;
    const long long base = (long long)rpages[gp] << PAGE_SHIFT;
    for (int q = threadIdx.x; q < PAGE; q += blockDim.x) {
        const long long o = (long long)gp * PAGE + q;
        if (q < fill) {
            const unsigned int t = meta[base + q] & M_TYPE;
            const unsigned int inv = ~((unsigned int)prio[base + q] ^ 0x80000000u);  // prio descending
            keys[o] = ((unsigned long long)b << TIDX_BUCKET_SHIFT) | ((unsigned long long)t << TIDX_PRIO_BITS) | inv;
            vals[o] = pi * PAGE + q;  // position in the bucket (wqseqno order)
        } else {
            keys[o] = ~0ull;  // holes sort last
            vals[o] = -1;
        }
    }
}

// (bucket, type) group g's range as lower bounds, empty groups included:
// tstart[g] = #entries of groups < g, tend[g] = #entries of groups <= g
__device__ __forceinline__ int tidx_lower(const unsigned long long *__restrict__ keys, int n, unsigned long long v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void k_tindex_bounds(const unsigned long long *__restrict__ keys, int n, int G, int *tstart, int *tend) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    tstart[g] = tidx_lower(keys, n, (unsigned long long)g << TIDX_PRIO_BITS);
    tend[g] = tidx_lower(keys, n, (unsigned long long)(g + 1) << TIDX_PRIO_BITS);
}

// after merging m sorted new keys into the index: every group's bounds move up
// by the new keys of the groups before it (groups past G_old held n_old)
__global__ void k_tindex_shift(const unsigned long long *__restrict__ nkeys, int m, int G_old, int n_old, int G,
                               int *tstart, int *tend) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const int os = g < G_old ? tstart[g] : n_old, oe = g < G_old ? tend[g] : n_old;
    tstart[g] = os + tidx_lower(nkeys, m, (unsigned long long)g << TIDX_PRIO_BITS);
    tend[g] = oe + tidx_lower(nkeys, m, (unsigned long long)(g + 1) << TIDX_PRIO_BITS);
}

// One block per target-rank bucket: that rank's Reserves in arrival order
// against its targeted units (wq_find_pre_targeted_hi_prio, xq.c:219-247).  The
// Reserves come from the list prep_block built (sorted here into arrival
// order), or -- when more Reserves named the rank than the list holds -- from a
// scan of the batch, TGT_REQ at a time.  Per batch, every type's head of the
// bucket's sorted index is prefetched into an LDS cache: about twice the
// Reserves that can take the type, all loads in flight together, unavailable
// units (pinned, deleted, prio <= LOWEST) dropped.  Wave 0 then serves the
// Reserves in order from LDS: lane t offers type t's head, the wave takes the
// minimum of (prio desc, position asc), the winner advances.  A type whose
// cache runs dry walks its range in global memory (a deep run of pinned
// units).  The pins are k_finalize's.
constexpr int TGT_REQ = 1024;    // Reserves per batch of the block
constexpr int TGT_CACHE = 1024;  // cached index entries per block (32 KB of LDS in all: five blocks per CU)
constexpr int TGT_PER = TGT_CACHE / 256;

__device__ __forceinline__ long long tidx_slot(const int *__restrict__ rpages, int p0, int L) {
    return ((long long)rpages[p0 + (L >> PAGE_SHIFT)] << PAGE_SHIFT) + (L & (PAGE - 1));
}

// The delta index: the keys of targeted units Put since the main index was
// last merged or rebuilt, sorted the same way, with its own group bounds.  A
// group's entries are the merge of its main and delta ranges; a delta entry
// of a bucket always lies later in the bucket than its main entries (Puts
// append), so (inverted prio, bucket position) orders the two alike.
struct TDelta {
    const unsigned long long *keys;
    const int *vals;
    const int *start, *end;  // [groups] lower bounds, as tstart / tend
    int n;                   // 0: no delta
};

// cache / walk key of an index entry: inverted prio << 32 | position in the bucket + 1
// (never 0: 0 marks an empty cache, ~0 no head)
__device__ __forceinline__ unsigned long long tidx_ck(unsigned long long k, int L) {
    return ((k & 0xffffffffull) << 32) | ((unsigned int)L + 1u);
}

// first index in [lo, hi) of a group whose entry comes after key ck (a walk restart)
__device__ __forceinline__ int tidx_after(const unsigned long long *__restrict__ keys, const int *__restrict__ vals,
                                          int lo, int hi, unsigned long long ck) {
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (tidx_ck(keys[mid], vals[mid]) <= ck) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_targeted_idx(const int *__restrict__ bucket_ranks,
                                                      const int *__restrict__ pstart, const int *__restrict__ rpages,
                                                      const unsigned long long *__restrict__ tkeys,
                                                      const int *__restrict__ tvals, const int *__restrict__ tstart,
                                                      const int *__restrict__ tend, TDelta dl, int T, const uint32_t *meta,
                                                      const unsigned long long *__restrict__ mask,
                                                      const int *__restrict__ reqs, int R, int *tmatch, int *seg_cnt,
                                                      int *tcnt, const int *__restrict__ tlist, int tcap,
                                                      int tdiag) {
    __shared__ int sreq[TGT_REQ];                   // the batch's Reserves in arrival order
    __shared__ unsigned long long smk[TGT_REQ];     // their type masks
    __shared__ unsigned long long ckey[TGT_CACHE];  // cached heads: inverted prio << 32 | position in the bucket
    __shared__ int cslot[TGT_CACHE], cex[TGT_CACHE + 1];
    __shared__ int dem[64], coff[65], cmid[64], gbase[64], gend[64], dbase[64], dend[64], ccnt[64];
    __shared__ int gnext[64], dnext[64], amain[64];
    __shared__ int4 s_st[64];                    // the block serve: per type {hd, cached, offset, more}
    __shared__ unsigned long long s_ball[64];    // ... and the lanes choosing it
    __shared__ unsigned long long cut[64];
    __shared__ int nlist, wcnt[4], wsum[4], s_over;
    const int b = blockIdx.x, r = bucket_ranks[b], p0 = pstart[b];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if (pstart[b + 1] - p0 <= 0) {
        if (tid == 0) tcnt[b] = 0;
        return;
    }
    const bool has_delta = dl.n > 0;
    if (tid < 64) {
        gbase[tid] = tid < T ? tstart[b * 64 + tid] : 0;
        gend[tid] = tid < T ? tend[b * 64 + tid] : 0;
        dbase[tid] = (tid < T && has_delta) ? dl.start[b * 64 + tid] : 0;
        dend[tid] = (tid < T && has_delta) ? dl.end[b * 64 + tid] : 0;
    }
    if (tid == 0) {
        const int n = tcnt[b];
        s_over = n > tcap;
        nlist = s_over ? 0 : n;
        tcnt[b] = 0;  // for the next batch (prep_block appends again)
    }
    __syncthreads();
    const bool over = s_over;
    int j0 = 0;  // scan position (overflow)
    while (true) {
        // ---- the next batch of this rank's Reserves, in arrival order
        int n;
        if (!over) {
            n = nlist;
            for (int k = tid; k < n; k += blockDim.x) sreq[k] = tlist[(long long)b * tcap + k];
            __syncthreads();
            int v[TGT_REQ / 256], pos[TGT_REQ / 256];  // rank of each among the distinct request indices
#pragma unroll
            for (int q = 0; q < TGT_REQ / 256; q++) {
                const int k = tid + q * 256;
                v[q] = k < n ? sreq[k] : INT_MAX;
                pos[q] = 0;
            }
            for (int k = 0; k < n; k++) {
                const int x = sreq[k];
#pragma unroll
                for (int q = 0; q < TGT_REQ / 256; q++) pos[q] += x < v[q];
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < TGT_REQ / 256; q++)
                if (tid + q * 256 < n) sreq[pos[q]] = v[q];
        } else {
            if (tid == 0) nlist = 0;
            __syncthreads();
            for (; j0 < R; j0 += 256) {
                const int j = j0 + tid;
                const bool is = j < R && reqs[(long long)ADLBQ_RESERVE_INTS * j] == r;
                const unsigned long long bal = __ballot(is);
                if (lane == 0) wcnt[w] = __popcll(bal);
                __syncthreads();
                int woff = nlist;
                for (int q = 0; q < w; q++) woff += wcnt[q];
                if (is) sreq[woff + __popcll(bal & lanemask_lt())] = j;
                __syncthreads();
                if (tid == 0) nlist += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
                __syncthreads();
                if (nlist > TGT_REQ - 256) {
                    j0 += 256;
                    break;
                }
            }
            n = nlist;
        }
        __syncthreads();
        if (n == 0) break;
        if (tdiag & 1) break;  // diagnostic ("targeted_diag" 1): the request lists only (wrong results)
        for (int k = tid; k < n; k += blockDim.x) smk[k] = mask[sreq[k]];
        if (tid < 64) {
            dem[tid] = 0;
            cut[tid] = ~0ull;
            gnext[tid] = 0;
            dnext[tid] = 0;
            ccnt[tid] = 0;
        }
        __syncthreads();
        // ---- per type: the Reserves that can take it (each takes at most one unit)
        for (int k = tid; k < n; k += blockDim.x)
            for (unsigned long long m = smk[k]; m; m &= m - 1) atomicAdd(&dem[__ffsll((long long)m) - 1], 1);
        __syncthreads();
        // ---- cache regions: per type, twice the demand + 8 of the main range, then as many of
        // the delta range (less when the cache is short)
        if (tid == 0) {
            int tot = 0;
            for (int t = 0; t < T; t++)
                tot += min(2 * dem[t] + 8, gend[t] - gbase[t]) + min(2 * dem[t] + 8, dend[t] - dbase[t]);
            const bool big = tot > TGT_CACHE;
            int acc = 0;
            for (int t = 0; t < T; t++) {
                const int wt = big ? dem[t] : 2 * dem[t] + 8;
                const int wm = max(0, min(min(wt, gend[t] - gbase[t]), TGT_CACHE - acc));
                const int wd = max(0, min(min(wt, dend[t] - dbase[t]), TGT_CACHE - acc - wm));
                coff[t] = acc;
                cmid[t] = acc + wm;
                acc += wm + wd;
                // a range cut short: the cache is valid only up to its last fetched entry (set
                // below); cut short with nothing fetched, the cache holds nothing of the type
                if ((gbase[t] + wm < gend[t] && wm == 0) || (dbase[t] + wd < dend[t] && wd == 0)) cut[t] = 0ull;
            }
            coff[T] = acc;
        }
        __syncthreads();
        const int F = coff[T];
        // ---- fetch: thread tid takes flat entries [tid * TGT_PER, +TGT_PER), three dependent rounds of loads
        unsigned long long kv[TGT_PER];
        long long sl[TGT_PER];
        int gi[TGT_PER], ty[TGT_PER];
        bool av[TGT_PER], dpart[TGT_PER];
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) {
            const int f = tid * TGT_PER + q;
            gi[q] = -1;
            ty[q] = 0;
            dpart[q] = false;
            kv[q] = ~0ull;
            if (f < F) {
                int lo = 0, hi = T;  // type of flat entry f: coff[t] <= f < coff[t+1]
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (coff[mid] <= f) lo = mid; else hi = mid;
                }
                ty[q] = lo;
                dpart[q] = f >= cmid[lo];
                gi[q] = dpart[q] ? dbase[lo] + (f - cmid[lo]) : gbase[lo] + (f - coff[lo]);
                kv[q] = dpart[q] ? dl.keys[gi[q]] : tkeys[gi[q]];
            }
        }
        int L[TGT_PER];
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) L[q] = gi[q] >= 0 ? (dpart[q] ? dl.vals[gi[q]] : tvals[gi[q]]) : 0;
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) sl[q] = gi[q] >= 0 ? tidx_slot(rpages, p0, L[q]) : 0;
        // the last fetched entry of a range cut short bounds the cache's valid prefix
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) {
            const int f = tid * TGT_PER + q;
            if (gi[q] < 0) continue;
            const int t = ty[q];
            const bool last_m = !dpart[q] && f == cmid[t] - 1 && gi[q] + 1 < gend[t];
            const bool last_d = dpart[q] && f == coff[t + 1] - 1 && gi[q] + 1 < dend[t];
            if (last_m || last_d) atomicMin(&cut[t], tidx_ck(kv[q], L[q]));
        }
        int cnt = 0;
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) {
            av[q] = false;
            if (gi[q] >= 0) {
                const uint32_t mt = meta[sl[q]];
                const int pr = (int)(~(unsigned int)kv[q] ^ 0x80000000u);
                av[q] = (mt & (M_LIVE | M_PINNED)) == M_LIVE && pr > LOWEST;
            }
            cnt += av[q];
        }
        // block exclusive scan of the availability flags over the flat order
        int x = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int pre = x - cnt;
        for (int q = 0; q < w; q++) pre += wsum[q];
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) {
            const int f = tid * TGT_PER + q;
            if (f < F) cex[f] = pre;
            pre += av[q];
        }
        if (tid == 255) cex[F] = pre;
        __syncthreads();
        // where the walk resumes after the cache: per range, the fetched entries up to the cut
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) {
            if (gi[q] < 0 || tidx_ck(kv[q], L[q]) > cut[ty[q]]) continue;
            atomicAdd(dpart[q] ? &dnext[ty[q]] : &gnext[ty[q]], 1);
        }
        if (tid < T) amain[tid] = cex[cmid[tid]] - cex[coff[tid]];  // available main entries of the type
        // the main range's available entries, compacted in order at the region's start ...
        int at[TGT_PER];
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) {
            const int f = tid * TGT_PER + q;
            at[q] = -1;
            if (f < F && av[q]) {
                const int t = ty[q];
                at[q] = coff[t] + (cex[f] - cex[coff[t]]);  // main first, then delta (flat order)
                ckey[at[q]] = tidx_ck(kv[q], L[q]);
            }
        }
        __syncthreads();
        // ... then both runs merged in place: an entry moves up by the entries of the other run before it
        if (has_delta) {
#pragma unroll
            for (int q = 0; q < TGT_PER; q++) {
                if (at[q] < 0) continue;
                const int t = ty[q], c0 = coff[t], am = amain[t], ad = cex[coff[t + 1]] - cex[cmid[t]];
                const unsigned long long k = ckey[at[q]];
                int lo, hi;
                if (!dpart[q]) { lo = c0 + am; hi = c0 + am + ad; }  // delta run
                else { lo = c0; hi = c0 + am; }                      // main run
                const int base = lo;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (ckey[mid] < k) lo = mid + 1;
                    else hi = mid;
                }
                at[q] = dpart[q] ? at[q] - am + (lo - base) : at[q] + (lo - base);
            }
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < TGT_PER; q++) {
            if (at[q] < 0) continue;
            const unsigned long long k = tidx_ck(kv[q], L[q]);
            ckey[at[q]] = k;
            cslot[at[q]] = (int)sl[q];
            if (k <= cut[ty[q]]) atomicAdd(&ccnt[ty[q]], 1);  // the valid prefix of the merged cache
        }
        __syncthreads();
        if (tdiag & 2) break;  // diagnostic ("targeted_diag" 2): lists and cache fill only (wrong results)
        // ---- serve the Reserves in order (wave 0): lane t holds type t's head
        // (and the one after it) in registers; per Reserve a scalar loop over
        // its types compares the heads (readlane), the winner's lane advances
        if (w == 0) {
            const bool tl = lane < T;
            const int co = tl ? coff[lane] : 0, cn = tl ? ccnt[lane] : 0;
            const int ge = tl ? gend[lane] : 0, de = tl ? dend[lane] : 0;
            int hd = 0;                                      // cached heads consumed
            int gn = tl ? gbase[lane] + gnext[lane] : 0;     // main and delta positions past the cache
            int dn = tl ? dbase[lane] + dnext[lane] : 0;
            // head key / slot and the next three cached entries in registers: a Reserve's advance is
            // register moves (an LDS read per advance made every Reserve wait for the one before);
            // the ring is refilled from the cache after each block of 64, or when it runs dry
            unsigned long long hk = ~0ull, k1 = ~0ull, k2 = ~0ull, k3 = ~0ull;
            unsigned long long lastk = 0ull;  // key of the type's last unit taken (0: none)
            int hs = -1, s1 = -1, s2 = -1, s3 = -1;
            auto fill = [&]() {  // type lane, cached heads left: the head and the ring from entry hd on
                if (!tl || hd >= cn) return;
                const int b = co + hd;
                hk = ckey[b];
                hs = cslot[b];
                k1 = hd + 1 < cn ? ckey[b + 1] : ~0ull;
                s1 = hd + 1 < cn ? cslot[b + 1] : -1;
                k2 = hd + 2 < cn ? ckey[b + 2] : ~0ull;
                s2 = hd + 2 < cn ? cslot[b + 2] : -1;
                k3 = hd + 3 < cn ? ckey[b + 3] : ~0ull;
                s3 = hd + 3 < cn ? cslot[b + 3] : -1;
            };
            auto walk = [&](unsigned long long &k, int &sl) {  // next available unit past the cache (slow path)
                k = ~0ull;
                sl = -1;
                while (gn < ge || dn < de) {
                    const unsigned long long km = gn < ge ? tidx_ck(tkeys[gn], tvals[gn]) : ~0ull;
                    const unsigned long long kd = dn < de ? tidx_ck(dl.keys[dn], dl.vals[dn]) : ~0ull;
                    const bool fromd = kd < km;
                    const unsigned long long kk = fromd ? kd : km;
                    const int pr = (int)(~(unsigned int)(kk >> 32) ^ 0x80000000u);
                    if (pr <= LOWEST) {  // prio descending: nothing after it matches either
                        if (fromd) dn = de;
                        else gn = ge;
                        continue;
                    }
                    const int LL = (int)(unsigned int)kk - 1;
                    const long long ss = tidx_slot(rpages, p0, LL);
                    if (fromd) dn++;
                    else gn++;
                    if ((meta[ss] & (M_LIVE | M_PINNED)) == M_LIVE) {
                        k = kk;
                        sl = (int)ss;
                        break;
                    }
                }
            };
            fill();
            for (int k0 = 0; k0 < n; k0 += 64) {
                const unsigned long long mv = k0 + lane < n ? smk[k0 + lane] : 0ull;
                const int jv = k0 + lane < n ? sreq[k0 + lane] : 0;
                const int kn = min(64, n - k0);
                int myslot = -1;  // lane kk: the unit Reserve k0 + kk takes (written after the block)
                bool solved = false;
                if (tdiag & 8) {  // A/B ("targeted_diag" 8): measured slower than the serve below (config 4)
                    // ---- the block in parallel (lane i = Reserve k0 + i), Jacobi rounds on the choice
                    // types: lane i's candidate of type t is cached entry hd_t + #{earlier lanes choosing
                    // t}; lane k is exact by round k + 1, and the fixed point is the serial answer unless
                    // some lane needs an entry past a type's cache with more units behind it (a walk):
                    // then the block goes one by one below.  Per round: one ballot per wanted type
                    // (into LDS), then each lane's types' state, counts and keys in two LDS rounds.
                    s_st[lane] = make_int4(tl ? hd : 0, tl ? cn : 0, tl ? co : 0,
                                           (tl && (gn < ge || dn < de || (hd >= cn && hk != ~0ull))) ? 1 : 0);
                    unsigned long long want = mv;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) want |= __shfl_xor(want, o, 64);
                    want = readlane64(want, 0);
                    int tt[4];  // this lane's first four types (-1: none); the rest in `rest`
                    unsigned long long rest = mv;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        tt[q] = rest ? __ffsll((long long)rest) - 1 : -1;
                        rest &= rest - 1;
                    }
                    const unsigned long long lt = lanemask_lt();
                    int ch = -1;
                    bool unc = false;
                    for (int round = 0; round <= kn; round++) {
                        for (unsigned long long wm = want; wm; wm &= wm - 1) {
                            const int t = __ffsll((long long)wm) - 1;
                            const unsigned long long b = __ballot(ch == t);
                            if (lane == 0) s_ball[t] = b;
                        }
                        __builtin_amdgcn_wave_barrier();  // one wave's LDS operations stay in order
                        unsigned long long best = ~0ull;
                        int nc = -1;
                        unc = false;
                        auto look = [&](int t, const int4 st, unsigned long long b) {
                            const int idx = st.x + (int)__popcll(b & lt);
                            if (idx < st.y) {
                                const unsigned long long kt = ckey[st.z + idx];
                                if (kt < best) best = kt, nc = t;
                            } else if (st.w) {
                                unc = true;
                            }
                        };
                        int4 st4[4];
                        unsigned long long b4[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            st4[q] = s_st[tt[q] >= 0 ? tt[q] : 0];
                            b4[q] = s_ball[tt[q] >= 0 ? tt[q] : 0];
                        }
#pragma unroll
                        for (int q = 0; q < 4; q++)
                            if (tt[q] >= 0) look(tt[q], st4[q], b4[q]);
                        for (unsigned long long mm = rest; mm; mm &= mm - 1) {
                            const int t = __ffsll((long long)mm) - 1;
                            look(t, s_st[t], s_ball[t]);
                        }
                        const bool changed = nc != ch;
                        ch = nc;
                        __builtin_amdgcn_wave_barrier();  // the reads above before the next round's writes
                        if (!__ballot(changed)) break;
                    }
                    if (!__ballot(unc)) {
                        solved = true;
                        // s_ball holds the final choices' ballots (the last round changed nothing)
                        if (ch >= 0) {
                            const int4 st = s_st[ch];
                            myslot = cslot[st.z + st.x + (int)__popcll(s_ball[ch] & lt)];
                        }
                        const int took = (tl && ((want >> lane) & 1ull)) ? (int)__popcll(s_ball[lane]) : 0;
                        if (took > 0) {
                            hd += took;
                            lastk = ckey[co + hd - 1];
                            hk = ~0ull;  // fill() below reloads the head and the ring (or leaves none)
                            hs = -1;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                for (int kk = 0; kk < kn && !solved; kk++) {
                    const unsigned long long m = readlane64(mv, kk);
                    // a type whose cache ran dry walks before it competes (uniform loop over such types)
                    const unsigned long long dry = __ballot(tl && hk == ~0ull && hd >= cn && (gn < ge || dn < de)) & m;
                    if (dry && ((dry >> lane) & 1ull) && !(tdiag & 4)) walk(hk, hs);  // diag 4: no walks
                    unsigned long long best = ~0ull;
                    int bt = -1;
                    for (unsigned long long mm = m; mm; mm &= mm - 1) {
                        const int t = __ffsll((long long)mm) - 1;
                        const unsigned long long kt = readlane64(hk, t);
                        if (kt < best) {
                            best = kt;
                            bt = t;
                        }
                    }
                    if (bt < 0 || best == ~0ull) continue;
                    // no global store in the loop: a walk's loads make the compiler wait for every
                    // outstanding memory operation at the loop's join (vmcnt counts stores and atomics)
                    const int sl = __builtin_amdgcn_readlane(hs, bt);
                    if (lane == kk) myslot = sl;
                    if (lane == bt) {  // advance: the next cached head, else the walk later
                        lastk = hk;
                        if (hd < cn) hd++;
                        hk = k1, hs = s1, k1 = k2, s1 = s2, k2 = k3, s2 = s3, k3 = ~0ull, s3 = -1;
                        if (hk == ~0ull) fill();  // the ring ran dry (the cache may hold more)
                    }
                }
                fill();
                if (lane < kn && myslot >= 0) {  // the block's choices, one lane each
                    tmatch[jv] = myslot;
                    atomicSub(&seg_cnt[jv >> 6], 1);
                }
            }
            // overflow only: the next Reserves of the rank resume after the last unit taken of each type
            if (over && tl && lastk != 0ull) {
                gbase[lane] = tidx_after(tkeys, tvals, gbase[lane], ge, lastk);
                if (has_delta) dbase[lane] = tidx_after(dl.keys, dl.vals, dbase[lane], de, lastk);
            }
        }
        __syncthreads();
        if (!over || j0 >= R) break;
    }
}

// ---------------------------------------------------------------- untargeted choices in arrival order
//
// After the scan every type t has a candidate list in global preference order
// (packed ranks ascending, k_rank).  Request j takes the best head among its
// types: cand_t[pos_t(j)], pos_t(j) = how many earlier requests took type t.
// The state before request j is the vector pos(j); the sequential order is a
// chain of T-way merges.  It is solved in parallel by *segments*:
//
//   * the batch is cut into segments of SEG requests, one wavefront each; a
//     wavefront solves its segment exactly from a given start vector (64-lane
//     blocks, Jacobi rounds inside a block: lane k is exact by round k+1);
//   * pass 1 starts every segment from a guess: the "level" state
//     pos_t = #{type-t candidates with global rank < J}, J = requests before the
//     segment that take an untargeted unit.  The multi-type requests keep the
//     list heads level, so the guess is close (|error|_1 ~ 10 at config 2);
//   * pass k > 1 starts segment s from the end state segment s-1 reached in
//     pass k-1.  Two trajectories of the merge coalesce once the multi-type
//     requests have levelled the heads (~150 requests), so an end state is exact
//     as soon as its segment coalesced, whatever its start was.  A segment whose
//     start did not change is not recomputed;
//   * a pass in which no start changed is a fixed point, and the fixed point
//     is the sequential result (segment 0 starts from 0; by induction every
//     start is exact).  After CHAIN_PASSES passes without one, k_chain_fix
//     walks the segments in order from the exact prefix and recomputes only
//     those whose start still differs (adversarial inputs; tests force it).


__device__ __forceinline__ unsigned long long wave_or_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
    return v;
}

// Packed global rank of every candidate: (rank among all candidates of the
// batch by (prio desc, wqseqno asc)) << 6 | type.  A smaller packed value is a
// better unit, so the chain compares heads with one 32-bit min and reads the
// winning type from the low bits.  rank = position in its own list + for every
// other type u the number of u's candidates with a better key (a lower bound).
// The lists are sorted, so for a tile of 256 consecutive candidates of one
// type the lower bounds in list u lie between those of the tile's first and
// last keys: one wave finds both (32-ary searches, three probe rounds), loads
// that stretch of list u into LDS and the tile's threads search it there.
// The waves of a workgroup take the other types in turn.
constexpr int RANK_TILE = 256, RANK_SPAN = 1024;  // 32 KB of spans: five workgroups per CU

__device__ __forceinline__ int lower_bound_key(const unsigned long long *L, int n, unsigned long long key) {
    int lo = 0, hi = n;  // first position whose key is not better than `key` (L descending)
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (L[mid] > key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Types whose threshold fell in a multi-priority bin (needsort) are sorted
// first, inside this launch: the first workgroups to draw a ticket each sort
// one such type (sort_type), release it and raise its flag; every workgroup
// waits for those flags (relaxed poll, agent acquire).  Sorters are running
// before anyone waits for them, so the waits cannot deadlock.  Without such a
// type (the usual case) nobody draws a ticket or waits.
// The chain's level guess for T <= 8: row g / LV_STEP (g < R, g a multiple of
// LV_STEP) holds, for the candidate at global rank g, the number of candidates
// of each type ranked before it -- the lower bounds k_rank computes anyway --
// i.e. the state in which the first g candidates in preference order are taken.
struct LevelRows {
    int *lv;              // [R][T], or nullptr (T > 8)
    int R;
    unsigned char *rtype;  // [R] type of the candidate at rank g (with lv)
};

struct RankSort {
    const int *needsort;
    unsigned long long *ckey2;
    int *cslot, *cslot2;
    int *sync;  // [t] sorted epochs, [ADLBQ_MAX_TYPES] ticket, [ADLBQ_MAX_TYPES + 1] timed-out waits
    unsigned int epoch;
    int fail_test;  // adlbq_set_param("sort_fail_test"): count one timed-out wait (tests the error path)
};

// k_rank's arguments
struct RankArgs {
    int T;
    const int *candoff, *candlen;
    unsigned long long *ckey;  // sorted in this launch: not restrict
    unsigned int *crank, *csum;
    long long ncsum;
    const unsigned long long *mask;
    const int *tmatch;
    int R;
    int *seg_cnt;
    RankSort rs;
    LevelRows lr;
    const DevCounters *ctr;
};

// The rank work of workgroup bid of nb (NT threads).
template <int NT>
__device__ __forceinline__ void rank_body(const RankArgs &ra, const int bid, const int nb) {
    constexpr int NW = NT / 64, SROWS = NW > 3 ? NW : 3;  // span: NW search rows, at least the sort's 24 KB
    const int T = ra.T;
    const int *__restrict__ candoff = ra.candoff;
    const int *__restrict__ candlen = ra.candlen;
    unsigned long long *ckey = ra.ckey;
    unsigned int *__restrict__ crank = ra.crank;
    unsigned int *__restrict__ csum = ra.csum;
    const long long ncsum = ra.ncsum;
    const unsigned long long *__restrict__ mask = ra.mask;
    const int *__restrict__ tmatch = ra.tmatch;
    const int R = ra.R;
    int *seg_cnt = ra.seg_cnt;
    const RankSort &rs = ra.rs;
    const LevelRows &lr = ra.lr;
    const DevCounters *ctr = ra.ctr;
    __shared__ int soff[ADLBQ_MAX_TYPES + 1], slen[ADLBQ_MAX_TYPES], stile[ADLBQ_MAX_TYPES + 1];
    __shared__ unsigned long long span[SROWS][RANK_SPAN];  // also the sort's LDS blocks
    static_assert(sizeof(unsigned long long) * SROWS * RANK_SPAN >= (sizeof(unsigned long long) + sizeof(int)) * SORT_BLK,
                  "sort_type's LDS fits in span");
    __shared__ unsigned long long s_first, s_last, s_sortmask;
    __shared__ int s_a0[NW], s_len[NW], s_tk, s_fast;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (rs.fail_test && bid == 0 && tid == 0) atomicAdd(rs.sync + ADLBQ_MAX_TYPES + 1, 1);
    // every input of the prologue in one round of loads: list offsets / lengths,
    // the sort flags, the fast-ranking flag k_select_open left
    if (tid <= T) soff[tid] = candoff[tid];
    if (tid < 64) {
        const int len = tid < T ? candlen[tid] : 0;
        const int ns = tid < T ? rs.needsort[tid] : 0;
        if (tid < T) slen[tid] = len;
        const int fast = tid == 0 ? ctr->rank_fast : 0;
        const unsigned long long m = __ballot(ns == 1 && len > 1);  // 2: already sorted
        if (tid == 0) {
            s_sortmask = m;
            s_fast = fast;
        }
    }
    // the scan's chunk sums are consumed (k_select_open): leave them zeroed for the next batch
    for (long long i = (long long)bid * blockDim.x + threadIdx.x; i < ncsum; i += (long long)nb * blockDim.x)
        csum[i] = 0;
    __syncthreads();
    const unsigned long long sortmask = s_sortmask;
    if (sortmask) {
        const int nsort = __popcll(sortmask);
        if (tid == 0) {
            const int tk = __hip_atomic_fetch_add(rs.sync + ADLBQ_MAX_TYPES, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tk == (int)nb - 1)  // every ticket drawn: reset for the next batch
                __hip_atomic_store(rs.sync + ADLBQ_MAX_TYPES, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_tk = tk;
        }
        __syncthreads();
        // the block with ticket tk sorts the tk-th, (tk + grid)-th, ... type that needs it:
        // the first blocks to run take the work, and a grid smaller than the sort count
        // (the small grid of a rank hint) still sorts every list
        for (int q = s_tk; q < nsort; q += nb) {
            unsigned long long mm = sortmask;
            for (int r = 0; r < q; r++) mm &= mm - 1;
            const int t = __ffsll((long long)mm) - 1;
            unsigned long long *sk = &span[0][0];
            int *ss = reinterpret_cast<int *>(sk + SORT_BLK);
            sort_type(soff[t], slen[t], ckey, rs.cslot, rs.ckey2, rs.cslot2, sk, ss);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(rs.sync + t, (int)rs.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (tid < 64) {
            bool ok = true;
            if ((sortmask >> lane) & 1ull) {
                for (int spin = 0; __hip_atomic_load(rs.sync + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                                   (int)rs.epoch; spin++) {
                    if (spin >= (1 << 22)) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            if (!ok) atomicAdd(rs.sync + ADLBQ_MAX_TYPES + 1, 1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    {
        // the chain's level guess counts the requests that take an untargeted
        // unit: drop those whose types have no candidate at all (prep_block
        // counted every non-empty type set, k_targeted the targeted matches)
        unsigned long long cm = 0;
        for (int t = 0; t < T; t++) cm |= slen[t] > 0 ? (1ull << t) : 0ull;
        const unsigned long long all = T >= 64 ? ~0ull : ((1ull << T) - 1);
        if (cm != all) {
            // eight groups of 64 per wave per step, their loads in flight together (a small grid
            // walks the whole batch: 16 waves over 1,024 groups at 65,536 Reserves)
            constexpr int DU = 8;
            const int waves = nb * (NT / 64);
            for (int g0 = bid * (NT / 64) + w; g0 * 64 < R; g0 += waves * DU) {
                unsigned long long m[DU];
                int tmv[DU];
                unsigned int okm = 0u;  // unconditional loads, masked after (opaque masks)
#pragma unroll
                for (int i = 0; i < DU; i++) {
                    const int j = (g0 + i * waves) * 64 + lane;
                    okm |= (j < R ? 1u : 0u) << i;
                    m[i] = mask[j < R ? j : 0];
                    tmv[i] = tmatch[j < R ? j : 0];
                }
                asm volatile("" : "+v"(okm));
#pragma unroll
                for (int i = 0; i < DU; i++) m[i] &= 0ull - (unsigned long long)((okm >> i) & 1u);
#pragma unroll
                for (int i = 0; i < DU; i++) {
                    const int g = g0 + i * waves;
                    const unsigned long long b = __ballot(m[i] != 0ull && !(m[i] & cm) && tmv[i] < 0);
                    if (lane == 0 && b) atomicSub(&seg_cnt[g], __popcll(b));
                }
            }
        }
    }
    if (tid == 0) {
        int acc = 0;
        for (int t = 0; t < T; t++) {
            stile[t] = acc;
            acc += (slen[t] + NT - 1) / NT;
        }
        stile[T] = acc;
    }
    __syncthreads();
    if (s_fast) return;  // k_select_open ranked the candidates and wrote the level rows
    for (int tile = bid; tile < stile[T]; tile += nb) {
        int t = 0;
        while (t + 1 < T && stile[t + 1] <= tile) t++;
        const int i0 = (tile - stile[t]) * NT, n = min(NT, slen[t] - i0);
        const unsigned long long *Lt = ckey + soff[t];
        const unsigned long long key = tid < n ? Lt[i0 + tid] : 0ull;
        if (tid == 0) s_first = key;
        if (tid == n - 1) s_last = key;
        __syncthreads();
        const unsigned long long kf = s_first, kl = s_last;
        unsigned int g = (unsigned int)(i0 + tid);
        int lbv[8];  // per type: candidates ranked before this one (level rows, T <= 8)
#pragma unroll
        for (int u = 0; u < 8; u++) lbv[u] = u == t ? i0 + tid : 0;
        for (int r0 = 0; r0 < T; r0 += NW) {  // wave w takes type r0 + w; every wave meets every barrier
            const int u = r0 + w;
            int a0 = 0, len = -1;
            if (u < T && u != t && slen[u] > 0) {
                const unsigned long long *L = ckey + soff[u];
                // lanes 0-31 search kf, lanes 32-63 search kl (32-ary, all probes of a round in flight)
                const unsigned long long kk = lane < 32 ? kf : kl;
                const int sl = lane & 31;
                int lo = 0, hi = slen[u];
                while (true) {
                    const int lo_f = __builtin_amdgcn_readlane(lo, 0), hi_f = __builtin_amdgcn_readlane(hi, 0);
                    const int lo_l = __builtin_amdgcn_readlane(lo, 32), hi_l = __builtin_amdgcn_readlane(hi, 32);
                    if (hi_f <= lo_f && hi_l <= lo_l) break;
                    const int step = (hi - lo + 31) >> 5;
                    const int idx = lo + sl * step;
                    const bool better = hi > lo && idx < hi && L[idx] > kk;
                    const unsigned long long bal = __ballot(better);
                    const int c = __popcll(lane < 32 ? (bal & 0xffffffffull) : (bal >> 32));
                    if (hi > lo) {
                        const int nlo = c == 0 ? lo : lo + (c - 1) * step + 1;
                        const int nhi = min(hi, lo + c * step);
                        lo = nlo;
                        hi = step == 1 ? nlo : nhi;
                    }
                }
                a0 = __builtin_amdgcn_readlane(lo, 0);
                len = __builtin_amdgcn_readlane(lo, 32) - a0;  // the tile's lower bounds lie in [a0, a0 + len]
                if (len <= RANK_SPAN)
                    for (int q = lane; q < len; q += 64) span[w][q] = L[a0 + q];
            }
            if (lane == 0) {
                s_a0[w] = a0;
                s_len[w] = len;
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < NW; q++) {
                const int lq = s_len[q], aq = s_a0[q];
                if (lq < 0 || tid >= n) continue;
                const int lb = lq <= RANK_SPAN ? lower_bound_key(span[q], lq, key)
                                               : lower_bound_key(ckey + soff[r0 + q] + aq, lq, key);
                g += (unsigned int)(aq + lb);
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (u == r0 + q) lbv[u] = aq + lb;
            }
            __syncthreads();
        }
        if (tid < n) crank[soff[t] + i0 + tid] = (g << 6) | (unsigned int)t;
        if (lr.lv != nullptr && tid < n && (int)g < lr.R) lr.rtype[g] = (unsigned char)t;
        if (lr.lv != nullptr && tid < n && (int)g < lr.R && (g & (LV_STEP - 1)) == 0) {
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (u < T) lr.lv[(long long)(g / LV_STEP) * T + u] = lbv[u];
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(RANK_TILE) void k_rank(RankArgs ra) { rank_body<RANK_TILE>(ra, blockIdx.x, gridDim.x); }

// ---------------------------------------------------------------- ordered choice: rounds over segment prefixes
//
// Segment s (SEG requests, one wavefront) turns a start state (lane t = head
// position of type t) into its choices and a per-type delta D_s = end - start.
// The sequential chain is start_0 = 0, start_s = sum_{q<s} D_q.  Launches:
//
//   k_chain0      round 0: every segment from a guessed start (the level
//                 state, optionally after a warm-up replay for T <= 8);
//   k_chainr x K  round k: every segment compares its start S_s with
//                 P_s = sum_{q<s} D_q (the deltas of the previous round) and
//                 re-solves from P_s when they differ, seeded with its previous
//                 choices (a Jacobi iteration converges from any seed; the
//                 seed makes an unchanged segment cost one round per block).
//
// After every round the deltas are summed by the arrivals themselves: the
// last arriver of each group of contiguous segments writes the group's local
// exclusive prefix LP and total GT, the last group writes the group offsets
// GO, so P_s = GO[g(s)] + LP[s] for the next launch.  A round in which no
// delta changed leaves every S_s == P_s: the fixed point, which is the
// sequential result (P_0 = 0; induction on s); the `clean` flag then turns the
// remaining round launches into no-ops.  A start error that no choice in a
// segment depends on passes through as a constant shift, so one round repairs
// it everywhere at once (in place of one segment per pass).  If the last round
// is still not clean, its last arriver walks the segments in order from the
// exact prefix, re-solving only those whose start differs.  No wavefront ever
// waits for another: only arrival counters and kernel boundaries order them.

constexpr int CH_GROUPS = 8;
constexpr unsigned char CHT_NONE = 255;

struct ChainArgs {
    const unsigned long long *mask;  // [R] type masks (0: no untargeted choice)
    const int *tmatch;               // [R] slot matched in the targeted phase, or -1
    int R, T, nseg, warm;            // warm: requests replayed before a segment in round 0 (T <= 8)
    int gs;                          // segments per arrival group (contiguous)
    const int *candoff, *candlen;    // [T]
    const unsigned int *crank;       // packed ranks, per type ascending
    int *umatch;                     // [R] out: candidate index or -1
    unsigned char *cht;              // [R] the choice's type index (CHT_NONE: none), the next round's seed
    const int *seg_cnt;              // [R/64] requests of each 64 that may take an untargeted unit
    int *S, *D;                      // [nseg][T] start used and delta, written by this launch
    const int *Sp, *Dp;              // [nseg][T] the same from the previous launch (double-buffered)
    int *LP;                         // [nseg][T] exclusive prefix of D in the group
    int *GT, *GO;                    // [CH_GROUPS][T] group totals, exclusive prefix over groups
    int *clean;                      // [1] set by a round that changed no delta
    unsigned long long *counters;    // [CH_GROUPS + 1] two-level arrival counters (zero between launches)
    DevCounters *ctr;
    const int *lv;                   // [R][T] k_rank's level rows (T <= 8), else nullptr
    const unsigned char *rtype;      // [R] type index of the candidate at each global rank (with lv)
    unsigned long long *stamps;      // [nseg][8] s_memrealtime per phase (diagnostic build of the run), or nullptr
    // k_rank_chain0 (k_rank's blocks in the chain's launch): their arrival counter (monotone) and the
    // value it reaches once this launch's rank blocks are done; nullptr when k_rank ran as a launch
    const unsigned long long *rdone;
    unsigned long long rtarget;
    const int *needsort;             // [T] (k_thresholds): a list k_rank sorts
    const int *jpref;                // [R/64 + 1] exclusive prefix of seg_cnt (k_thresholds), or nullptr: summed here
};

// diagnostic phase stamps (100 MHz constant clock), lane 0 of a segment
__device__ __forceinline__ void chain_stamp(const ChainArgs &a, int s, int ph) {
    if (a.stamps != nullptr) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) {
            a.stamps[s * 8 + ph] = __builtin_amdgcn_s_memrealtime();
            a.stamps[(a.nseg + s) * 8 + ph] = __builtin_amdgcn_s_memtime();  // shader clock
        }
    }
}

__device__ __forceinline__ void st_sc1(int *p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ld_sc1(const int *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Level guess for the state after J untargeted choices: pos_t = number of
// type-t candidates whose global rank is below J (every head at one level).
// 64-ary search, all TB types at once: three dependent probes per lane.
template <int TB>
__device__ __forceinline__ int level_guess(const ChainArgs a, int J) {
    const int lane = threadIdx.x;
    const unsigned int key = (unsigned int)J << 6;
    int my = 0;
    for (int g = 0; g < a.T; g += TB) {
        // every load unconditional (clamped index, masked after; masks opaque to the optimiser): a load
        // per type under its own condition was issued only after the one before had returned
        int lo[TB], hi[TB], off[TB];
#pragma unroll
        for (int q = 0; q < TB; q++) {
            const int t = min(g + q, a.T - 1);
            off[q] = a.candoff[t];
            hi[q] = a.candlen[t];
        }
        unsigned int tm = 0u;
#pragma unroll
        for (int q = 0; q < TB; q++) tm |= (g + q < a.T && J > 0 ? 1u : 0u) << q;
        asm volatile("" : "+v"(tm));
#pragma unroll
        for (int q = 0; q < TB; q++) {
            lo[q] = 0;
            hi[q] &= 0 - (int)((tm >> q) & 1u);
        }
        while (true) {
            bool open = false;
#pragma unroll
            for (int q = 0; q < TB; q++) open |= hi[q] > lo[q];
            if (!open) break;
            unsigned int v[TB], pm = 0u;
            int step[TB];
#pragma unroll
            for (int q = 0; q < TB; q++) {
                step[q] = (hi[q] - lo[q] + 63) >> 6;
                const int idx = lo[q] + lane * step[q];
                const bool ok = hi[q] > lo[q] && idx < hi[q];
                pm |= (ok ? 1u : 0u) << q;
                v[q] = a.crank[ok ? off[q] + idx : 0];
            }
            asm volatile("" : "+v"(pm));
#pragma unroll
            for (int q = 0; q < TB; q++) v[q] |= ((pm >> q) & 1u) - 1u;  // ~0u where not probed
#pragma unroll
            for (int q = 0; q < TB; q++) {
                if (hi[q] <= lo[q]) continue;
                const int c = __popcll(__ballot(v[q] < key));  // probes below key (a prefix: sorted)
                const int nlo = c == 0 ? lo[q] : lo[q] + (c - 1) * step[q] + 1;
                const int nhi = min(hi[q], lo[q] + c * step[q]);
                lo[q] = nlo;
                hi[q] = step[q] == 1 ? nlo : nhi;
            }
        }
#pragma unroll
        for (int q = 0; q < TB; q++)
            if (lane == g + q) my = lo[q];
    }
    return my;
}

// Requests [jb, j1) of segment s (j1 = its end) from the state my_start (lane
// t = type t) at jb; results are written from j0 = s * SEG on, and my_rec
// receives the state at j0 (jb < j0 only for round 0's warm-up).  All
// per-type state is uniform (T <= TB <= 8).  win holds, per type, the WL
// candidates following the start (~0u past the list end); a replay of WL
// requests consumes at most WL of any type.  seeded: the Jacobi rounds start
// from the choices of the previous solve (cht) instead of the single-type ones.
constexpr int CH_NONE = 63;  // no choice (T <= 8: never a type index)

// LDS after the windows and the sentinel row: the staged type masks of the
// segment's requests from pass 1's first request on (8 B each; so the block
// loop is not unrolled and one copy of the Jacobi loop stays in the
// instruction cache), then the segment's own choices (1 B each, the seed of
// the next solve).
template <int TB>
__device__ __forceinline__ unsigned long long *staged_masks(const ChainArgs a, unsigned int *win) {
    return reinterpret_cast<unsigned long long *>(win + TB * (SEG + a.warm) + 64);
}
template <int TB>
__device__ __forceinline__ unsigned char *staged_seeds(const ChainArgs a, unsigned int *win) {
    return reinterpret_cast<unsigned char *>(staged_masks<TB>(a, win) + (SEG + a.warm));
}

// load: masks of [jb, jb + WL) and (seeded) the segment's choices come from
// global memory into the staged area; otherwise they are staged already, the
// mask of request jb at index mk0.
template <int TB>
__device__ __forceinline__ int seg_solve_small(const ChainArgs a, int s, int jb, int my_start, unsigned int *win,
                                               int WL, bool seeded, bool load, int mk0, int my_off, int my_len,
                                               int &my_rec, int &rounds) {
    const int lane = threadIdx.x, j0 = s * SEG, j1 = min(a.R, j0 + SEG);
    int st[TB], off[TB], c0[TB];
    constexpr int NI = (SEG + CHAIN_WARM) / 64;  // WL <= SEG + CHAIN_WARM
    unsigned int wv[TB][NI];                      // every window load in flight before the first LDS write
    unsigned long long *smk = staged_masks<TB>(a, win);
    unsigned char *ssd = staged_seeds<TB>(a, win);
    unsigned long long mk[SEG_BLOCKS];
    int tm[SEG_BLOCKS];
    unsigned char sd[SEG_BLOCKS];
    if (load) {  // a re-solve of one segment (jb == j0): its masks, results of the targeted phase, seeds
        unsigned int okm = 0u;  // unconditional loads, masked after (as in the chain's prologue)
#pragma unroll
        for (int i = 0; i < SEG_BLOCKS; i++) {
            const int j = jb + i * 64 + lane;
            okm |= (j < j1 ? 1u : 0u) << i;
            mk[i] = a.mask[j < j1 ? j : 0];
            tm[i] = a.tmatch[j < j1 ? j : 0];
        }
        if (seeded) {
#pragma unroll
            for (int i = 0; i < SEG_BLOCKS; i++) {
                const int j = jb + i * 64 + lane;
                sd[i] = a.cht[j < j1 ? j : 0];
            }
        }
        asm volatile("" : "+v"(okm));
#pragma unroll
        for (int i = 0; i < SEG_BLOCKS; i++) {
            const unsigned int b = (okm >> i) & 1u;
            mk[i] &= 0ull - (unsigned long long)b;
            tm[i] &= 0 - (int)b;
            sd[i] = (seeded && b) ? sd[i] : CHT_NONE;
        }
    }
#pragma unroll
    for (int q = 0; q < TB; q++) {
        st[q] = __builtin_amdgcn_readlane(my_start, q);
        off[q] = __builtin_amdgcn_readlane(my_off, q);  // lane t holds type t's list offset and length
        const int len = __builtin_amdgcn_readlane(my_len, q);
        c0[q] = 0;
#pragma unroll
        for (int i = 0; i < NI; i++) {
            const int p = st[q] + i * 64 + lane;
            wv[q][i] = (i * 64 < WL && p < len) ? a.crank[off[q] + p] : ~0u;
        }
    }
#pragma unroll
    for (int q = 0; q < TB; q++)
#pragma unroll
        for (int i = 0; i < NI; i++)
            if (i * 64 < WL) win[q * WL + i * 64 + lane] = wv[q][i];
    if (load) {
#pragma unroll
        for (int i = 0; i < SEG_BLOCKS; i++) {
            smk[i * 64 + lane] = tm[i] < 0 ? mk[i] : 0ull;
            ssd[i * 64 + lane] = sd[i];
        }
        mk0 = 0;
    }
    const int sent = TB * (SEG + a.warm);  // 64 words of ~0u after the windows (the kernels' prologue)
    // one wave owns win: its LDS ops complete in order, only the compiler must not reorder
    __builtin_amdgcn_wave_barrier();
    if (!seeded) chain_stamp(a, s, 6);
    my_rec = my_start;
    const int nblk = (min(j1, jb + WL) - jb + 63) / 64;
#pragma unroll 1
    for (int bi = 0; bi < nblk; bi++) {
        const int b0 = jb + bi * 64;
        if (b0 == j0) {
#pragma unroll
            for (int q = 0; q < TB; q++)
                if (lane == q) my_rec = st[q] + c0[q];
        }
        const int j = b0 + lane;
        const unsigned long long m = smk[mk0 + bi * 64 + lane];
        // a type the request lacks reads the sentinel row (~0u): no select in the round
        int base[TB];
#pragma unroll
        for (int q = 0; q < TB; q++) base[q] = ((m >> q) & 1ull) ? q * WL + c0[q] : sent;
        int ch;
        if (seeded) {  // jb == j0
            const unsigned char sv = ssd[bi * 64 + lane];
            ch = sv == CHT_NONE ? CH_NONE : (int)sv;
        } else {
            ch = (m && !(m & (m - 1))) ? (__ffsll((long long)m) - 1) : CH_NONE;
        }
        unsigned long long chg;
        do {
            unsigned int v[TB];
#pragma unroll
            for (int q = 0; q < TB; q++) v[q] = win[base[q] + (int)mbcnt64(__ballot(ch == q))];
            unsigned int best = v[0];
#pragma unroll
            for (int q = 1; q < TB; q++) best = min(best, v[q]);
            const int nch = (int)(best & 63u);  // packed rank's type; ~0u (no head) gives CH_NONE
            chg = __ballot(nch != ch);
            ch = nch;
            rounds++;
        } while (chg);
        int res = -1;
#pragma unroll
        for (int q = 0; q < TB; q++) {
            const unsigned long long B = __ballot(ch == q);
            if (ch == q) res = off[q] + st[q] + c0[q] + (int)mbcnt64(B);
            c0[q] += __popcll(B);
        }
        if (b0 >= j0) {
            const unsigned char c = ch == CH_NONE ? CHT_NONE : (unsigned char)ch;
            ssd[(b0 - j0) + lane] = c;
            if (j < j1) {
                a.umatch[j] = res;
                a.cht[j] = c;
            }
        }
    }
    int my_end = my_start;
#pragma unroll
    for (int q = 0; q < TB; q++)
        if (lane == q) my_end = st[q] + c0[q];
    return my_end;
}

// Any T <= 64 (the wide variant).  Per type t an LDS record {lanes of the
// block choosing t (64-bit), choices of t in earlier blocks, list offset +
// start}.  A Jacobi round costs the same for any T: every lane clears the
// ballot word of its previous choice and ORs its bit into the one of its new
// choice (one wave's LDS operations complete in order), then reads the
// records of its own types (up to four in registers; more walk the mask) and
// the window entry each points at.
struct TypeRec {
    unsigned long long bal;
    int c0, offst;
};

__device__ __forceinline__ unsigned int head_of(const TypeRec *rec, const unsigned int *win, int t) {
    const TypeRec r = rec[t];
    return win[t * SEG + r.c0 + (int)mbcnt64(r.bal)];
}

__device__ __forceinline__ int seg_solve_wide(const ChainArgs a, int s, int my_start, unsigned int *win,
                                              TypeRec *rec, bool seeded, int my_off, int my_len, int &rounds) {
    const int lane = threadIdx.x, T = a.T, j0 = s * SEG, j1 = min(a.R, j0 + SEG);
    for (int g = 0; g < T; g += 8) {  // 8 types x SEG_BLOCKS loads in flight per lane
        unsigned int wv[8][SEG_BLOCKS];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int t = g + q < T ? g + q : 0;
            const int st = __builtin_amdgcn_readlane(my_start, t), off = __builtin_amdgcn_readlane(my_off, t);
            const int len = g + q < T ? __builtin_amdgcn_readlane(my_len, t) : 0;
#pragma unroll
            for (int i = 0; i < SEG_BLOCKS; i++) {
                const int p = st + i * 64 + lane;
                wv[q][i] = p < len ? a.crank[off + p] : ~0u;
            }
        }
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (g + q < T)
#pragma unroll
                for (int i = 0; i < SEG_BLOCKS; i++) win[(g + q) * SEG + i * 64 + lane] = wv[q][i];
    }
    if (lane < T) {
        rec[lane].bal = 0ull;
        rec[lane].c0 = 0;
        rec[lane].offst = my_off + my_start;
    }
    unsigned long long mk[SEG_BLOCKS];
    unsigned char sd[SEG_BLOCKS];
    {
        unsigned int okm = 0u;  // unconditional loads, masked after (as in the chain's prologue)
        int tmv[SEG_BLOCKS];
#pragma unroll
        for (int i = 0; i < SEG_BLOCKS; i++) {
            const int j = j0 + i * 64 + lane;
            okm |= (j < j1 ? 1u : 0u) << i;
            tmv[i] = a.tmatch[j < j1 ? j : 0];
            mk[i] = a.mask[j < j1 ? j : 0];
        }
        if (seeded) {
#pragma unroll
            for (int i = 0; i < SEG_BLOCKS; i++) {
                const int j = j0 + i * 64 + lane;
                sd[i] = a.cht[j < j1 ? j : 0];
            }
        }
        asm volatile("" : "+v"(okm));
#pragma unroll
        for (int i = 0; i < SEG_BLOCKS; i++) {
            const bool ok = ((okm >> i) & 1u) && tmv[i] < 0;
            mk[i] = ok ? mk[i] : 0ull;
            sd[i] = (seeded && ((okm >> i) & 1u)) ? sd[i] : CHT_NONE;
        }
    }
    // one wave owns win and rec: its LDS ops complete in order, only the compiler must not reorder
    __builtin_amdgcn_wave_barrier();
    for (int bi = 0; bi < SEG_BLOCKS; bi++) {
        const int b0 = j0 + bi * 64;
        if (b0 >= j1) break;
        const int j = b0 + lane;
        const unsigned long long m = mk[bi];
        // the lane's first four types in registers, the rest (rare) by a walk over the mask
        int ty[4];
        unsigned long long rest = m;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            ty[q] = rest ? __ffsll((long long)rest) - 1 : -1;
            rest &= rest - 1;
        }
        int ch = seeded ? (sd[bi] == CHT_NONE ? -1 : (int)sd[bi])
                        : ((m && !(m & (m - 1))) ? ty[0] : -1);
        int prev = -1;
        unsigned long long chg;
        do {
            if (prev >= 0) rec[prev].bal = 0ull;
            __builtin_amdgcn_wave_barrier();
            if (ch >= 0) atomicOr(&rec[ch].bal, 1ull << lane);
            __builtin_amdgcn_wave_barrier();
            unsigned int best = ~0u;
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (ty[q] >= 0) best = min(best, head_of(rec, win, ty[q]));
            for (unsigned long long r = rest; r; r &= r - 1) best = min(best, head_of(rec, win, __ffsll((long long)r) - 1));
            const int nch = best == ~0u ? -1 : (int)(best & 63u);
            chg = __ballot(nch != ch);
            prev = ch;
            ch = nch;
            rounds++;
            __builtin_amdgcn_wave_barrier();
        } while (chg);
        // converged: the ballot words hold the final choices; results, then the block's counts
        int res = -1;
        if (ch >= 0) {
            const TypeRec r = rec[ch];
            res = r.offst + r.c0 + (int)mbcnt64(r.bal);
        }
        __builtin_amdgcn_wave_barrier();
        if (ch >= 0) {
            rec[ch].bal = 0ull;
            atomicAdd(&rec[ch].c0, 1);
        }
        __builtin_amdgcn_wave_barrier();
        if (j < j1) {
            a.umatch[j] = res;
            a.cht[j] = ch < 0 ? CHT_NONE : (unsigned char)ch;
        }
    }
    __builtin_amdgcn_wave_barrier();
    return my_start + (lane < T ? rec[lane].c0 : 0);
}

// load: the segment's inputs come from global memory (a new launch, or the
// walk over other segments); otherwise round 0 staged them (T <= 8) and the
// masks of request jb sit at mk0.
template <int TB>
__device__ __forceinline__ int seg_solve(const ChainArgs a, int s, int jb, int my_start, unsigned int *win,
                                         bool seeded, bool load, int mk0, int my_off, int my_len, int &my_rec,
                                         int &rounds) {
    if constexpr (TB <= 8) {
        return seg_solve_small<TB>(a, s, jb, my_start, win, s * SEG - jb + SEG, seeded, load, mk0, my_off, my_len,
                                   my_rec, rounds);
    } else {
        my_rec = my_start;
        TypeRec *rec = reinterpret_cast<TypeRec *>(win + a.T * SEG);
        return seg_solve_wide(a, s, my_start, win, rec, seeded, my_off, my_len, rounds);
    }
}

// After a round: segment s publishes its start and delta (sc1 stores, drained
// before the arrival), then arrives at its group, and the group at the top
// counter.  When the next launch takes prefix starts, the last arriver of each
// group also sums the group's deltas (LP, GT) and the last group the group
// offsets (GO).  The very last arriver of the launch records the round, sets
// `clean` when nothing was re-solved (never in round 0) and, in the final round
// launch, walks what is still inconsistent.
constexpr unsigned long long CNT20 = (1ull << 20) - 1;

template <int TB>
__device__ __forceinline__ bool chain_arrive(const ChainArgs a, int s, int sv, int dv, int solved, int bad, int rounds,
                                             int round, int passes, bool final, bool prefix, unsigned int *win) {
    const int lane = threadIdx.x, T = a.T, nseg = a.nseg;
    if (lane < T) {
        st_sc1(a.S + s * T + lane, sv);
        st_sc1(a.D + s * T + lane, dv);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int g = s / a.gs, g0 = g * a.gs, gn = min(nseg, g0 + a.gs) - g0, ng = (nseg + a.gs - 1) / a.gs;
    // fields packed in one 64-bit add: arrivals (bits 0-19), possibly inconsistent
    // segments (20-39), segment re-solves (40-63)
    const unsigned long long mine = ((unsigned long long)solved << 40) | ((unsigned long long)bad << 20) | 1ull;
    int last = 0;
    unsigned long long v = 0;
    if (lane == 0) {
        if (rounds) atomicAdd(&a.ctr->chain_rounds, rounds);  // diagnostic, no return
        v = atomicAdd(&a.counters[g], mine) + mine;
        last = (int)(v & CNT20) == gn;
    }
    if (!__builtin_amdgcn_readfirstlane(last)) return false;
    chain_stamp(a, s, 6);
    // the group's last arriver: local exclusive prefix of the deltas, and the group total
    if (prefix && lane < T) {
        int acc = 0;
        for (int q0 = 0; q0 < gn; q0 += 16) {
            int d[16];
#pragma unroll
            for (int i = 0; i < 16; i++) d[i] = q0 + i < gn ? ld_sc1(a.D + (g0 + q0 + i) * T + lane) : 0;
#pragma unroll
            for (int i = 0; i < 16; i++)
                if (q0 + i < gn) {
                    st_sc1(a.LP + (g0 + q0 + i) * T + lane, acc);
                    acc += d[i];
                }
        }
        st_sc1(a.GT + g * T + lane, acc);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    unsigned long long tot = 0;
    if (lane == 0) {
        const unsigned long long up = (v & ~CNT20) | 1ull;  // the group's counts, one arrival
        tot = atomicAdd(&a.counters[CH_GROUPS], up) + up;
        last = (int)(tot & CNT20) == ng;
    }
    if (!__builtin_amdgcn_readfirstlane(last)) return false;
    chain_stamp(a, s, 7);
    // ---- the last arriver of the launch
    if (prefix && lane < T) {
        int x[CH_GROUPS];
#pragma unroll
        for (int q = 0; q < CH_GROUPS; q++) x[q] = q < ng ? ld_sc1(a.GT + q * T + lane) : 0;
        int acc = 0;
#pragma unroll
        for (int q = 0; q < CH_GROUPS; q++)
            if (q < ng) {
                a.GO[q * T + lane] = acc;
                acc += x[q];
            }
    }
    const unsigned long long totu =
        ((unsigned long long)(unsigned int)__builtin_amdgcn_readfirstlane((int)(tot >> 32)) << 32) |
        (unsigned long long)(unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)tot);  // no sign extension
    const int nbad = (int)((totu >> 20) & CNT20), nsolved = (int)(totu >> 40);
    const bool clean = nbad == 0;  // every start equals its predecessor's end
    if (lane == 0) {
        for (int q = 0; q <= CH_GROUPS; q++) a.counters[q] = 0;  // for the next launch (kernel boundary in between)
        *a.clean = clean ? 1 : 0;
        // sc1: a finalize fused into this launch snapshots them from another XCD
        if (round == 0) {
            st_sc1(&a.ctr->chain_passes, passes);
            st_sc1(&a.ctr->chain_recomputed, nsolved);
            st_sc1(&a.ctr->chain_fallback, 0);
        } else {
            st_sc1(&a.ctr->chain_passes, ld_sc1(&a.ctr->chain_passes) + 1);
            st_sc1(&a.ctr->chain_recomputed, ld_sc1(&a.ctr->chain_recomputed) + nsolved);
        }
    }
    if (!final || clean) return true;
    const int my_off = lane <= T ? ld_sc1(a.candoff + lane) : 0, my_len = lane < T ? ld_sc1(a.candlen + lane) : 0;
    // ---- walk: every segment before the first inconsistent one (start !=
    // predecessor's end) is exact; from there on, in order, re-solve each
    // segment whose start differs from its exact start.  Only the inconsistent
    // segments and the successors of re-solved ones can differ: a consistent
    // segment after an exact one is exact (its start is that one's end).  So the
    // walk finds the inconsistent segments 64 at a time (lane = segment) and
    // visits those, plus the successor of a re-solve whose new end differs from
    // the successor's start, instead of stepping through every segment.
    int redo = 0, rounds_w = 0;
    int first = nseg;
    for (int c0 = 0; c0 < nseg && first == nseg; c0 += 64) {
        const int q = c0 + lane;
        bool bad = false;
        if (q < nseg)
            for (int t = 0; t < T; t++)
                bad |= ld_sc1(a.S + q * T + t) !=
                       (q ? ld_sc1(a.S + (q - 1) * T + t) + ld_sc1(a.D + (q - 1) * T + t) : 0);
        const unsigned long long bb = __ballot(bad);
        if (bb) first = c0 + __ffsll((long long)bb) - 1;
    }
    int last_redo = -2, new_end = 0, carry = 0;
    for (int c0 = first & ~63; c0 < nseg; c0 += 64) {
        const int q = c0 + lane;
        bool bad = false;
        if (q < nseg && q > 0 && q >= first)
            for (int t = 0; t < T; t++)
                bad |= ld_sc1(a.S + q * T + t) != ld_sc1(a.S + (q - 1) * T + t) + ld_sc1(a.D + (q - 1) * T + t);
        unsigned long long bm = __ballot(bad) | (unsigned long long)carry;
        carry = 0;
        while (bm) {
            const int i = __ffsll((long long)bm) - 1;
            bm &= bm - 1;
            const int qq = c0 + i;
            // the exact start: the re-solved predecessor's new end, else its recorded end
            const int st = lane >= T || qq == 0 ? 0
                           : last_redo == qq - 1
                               ? new_end
                               : ld_sc1(a.S + (qq - 1) * T + lane) + ld_sc1(a.D + (qq - 1) * T + lane);
            const int sq = lane < T ? ld_sc1(a.S + qq * T + lane) : 0;
            if (!__ballot(lane < T && sq != st)) continue;
            int rec;
            __builtin_amdgcn_wave_barrier();  // win is refilled
            new_end = seg_solve<TB>(a, qq, qq * SEG, st, win, true, true, 0, my_off, my_len, rec, rounds_w);
            last_redo = qq;
            redo++;
            if (qq + 1 < nseg) {  // the successor, if it started elsewhere
                const int s1 = lane < T ? ld_sc1(a.S + (qq + 1) * T + lane) : 0;
                if (__ballot(lane < T && s1 != new_end)) {
                    if (i < 63) bm |= 1ull << (i + 1);
                    else carry = 1;
                }
            }
        }
    }
    if (lane == 0) {
        st_sc1(&a.ctr->chain_fallback, redo);
        atomicAdd(&a.ctr->chain_rounds, rounds_w);
    }
    return true;
}

// In-launch neighbour passes of round 0 (T <= 64 ints per hand-off), following
// the write-through protocol of MI355X_MICROARCH.md (inter-workgroup
// visibility): sc1 stores, drained, then an sc1 flag store by one lane; the
// reader polls the flag (relaxed, agent scope) and reads the state with sc1
// loads.  Waits are bounded (CHAIN_WAIT_US of wall clock): a timed-out wait
// skips that pass and is counted (chain_timeouts); it costs time, never
// correctness, since the segment then reports itself unchecked.
constexpr long long CHAIN_WAIT_US = 500;
constexpr int CHAIN_MAX_PASSES = 8;

__device__ __forceinline__ void publish_state(int *dst, int *flag, unsigned int epoch, int v, int T) {
    if (threadIdx.x < T) st_sc1(dst + threadIdx.x, v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) st_sc1(flag, (int)epoch);
}

__device__ __forceinline__ bool wait_flag(const int *flag, unsigned int epoch) {
    int ok = 0;
    if (threadIdx.x == 0) {
        const long long t0 = wall_clock64(), limit = CHAIN_WAIT_US * 100;  // 100 MHz constant clock
        while (true) {
            if (ld_sc1(flag) == (int)epoch) {
                ok = 1;
                break;
            }
            if (wall_clock64() - t0 > limit) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return __builtin_amdgcn_readfirstlane(ok) != 0;
}

struct ChainPass {
    int *E;              // [CHAIN_MAX_PASSES][nseg][T] end state of segment s after pass k
    int *flags;          // [CHAIN_MAX_PASSES][nseg] == epoch once E[k][s] is published
    unsigned int epoch;  // per batch, never 0
    int passes;          // in-launch passes, 1 .. CHAIN_MAX_PASSES (1: round 0 alone)
};

// Round k >= 1: a segment re-solves when its start differs from the estimate
// of its exact start, seeded with its previous choices.  mode 0 (neighbour):
// the estimate is the predecessor's end from the previous launch -- right as
// soon as the predecessor was, and absorbing start errors where multi-type
// requests level the list heads (few types); mode 1 (prefix): the sum of all
// earlier deltas -- passes a start error that no choice depends on straight
// through (many types, rare multi-type competition).  A launch that re-solved
// nothing proves every start equal to its predecessor's end: the fixed point.
template <int TB>
__global__ __launch_bounds__(64) void k_chainr(ChainArgs a, int round, int final, int mode, int prefix_next) {
    if (*a.clean) return;
    extern __shared__ unsigned int win[];
    const int lane = threadIdx.x, T = a.T, s = blockIdx.x, g = s / a.gs;
    if constexpr (TB <= 8) win[TB * (SEG + a.warm) + lane] = ~0u;  // seg_solve_small's sentinel row
    const bool tl = lane < T;
    const int my_off = lane <= T ? a.candoff[lane] : 0, my_len = tl ? a.candlen[lane] : 0;
    int sv = tl ? a.Sp[s * T + lane] : 0;
    int dv = tl ? a.Dp[s * T + lane] : 0;
    int xv = 0;
    if (mode == 0) xv = (tl && s > 0) ? a.Sp[(s - 1) * T + lane] + a.Dp[(s - 1) * T + lane] : 0;
    else xv = tl ? a.GO[g * T + lane] + a.LP[s * T + lane] : 0;
    int rounds = 0, solved = 0;
    if (__ballot(tl && xv != sv)) {
        int rec;
        const int end = seg_solve<TB>(a, s, s * SEG, xv, win, true, true, 0, my_off, my_len, rec, rounds);
        solved = 1;
        sv = xv;
        dv = end - xv;
    }
    // a re-solved segment may now be inconsistent with a predecessor re-solved alongside it
    chain_arrive<TB>(a, s, sv, dv, solved, solved, rounds, round, 0, final != 0, prefix_next != 0, win);
}

// ---------------------------------------------------------------- finalize + park
// Every request: pin its unit and write TA_RESERVE_RESP (adlb.c:1210-1224), or
// NO_CURR_WORK (1311-1316).  Requests that park are counted into a 64-bit
// arrival ticket (parked << 32 | 1 per workgroup); the workgroup that arrives
// last appends them to rq in arrival order and chooses their RFR donors
// (1238-1310).  Response words [10], [11] of a parked request are written only
// by that last workgroup, so no two workgroups store the same bytes.
// The RFR donors of a batch's parked Reserves (wave 0 of k_finalize's last
// workgroup), in FIFO order: the same choices as rfr_select per Reserve
// (adlb.c:1280-1308, 3487-3534), with the donor state held by the wave
// instead of re-read from memory per Reserve -- lane i holds server i's qlen,
// RFR-outstanding flag and maximum prio over types, its qmstat row sits in
// LDS, and the tq in LDS; 64 Reserves at a time have their rank's current
// rfr_to_rank and their type vector in registers.  Returns the first FIFO
// position left without a donor check (every later one has none).
constexpr int DONOR_TQ_LDS = 256;  // tq entries the fast path stages
__device__ int park_donors_fast(const DonorCtx &c, const int *__restrict__ reqs, const int *rq_req, int n0, int np,
                                int *resp, int *s_hi, int *s_tq, int *s_tv) {
    const int lane = threadIdx.x & 63, S = c.S, T = c.T;
    for (int q = lane; q < S * T; q += 64) s_hi[q] = c.qm_hi[q];
    for (int q = lane; q < 4 * c.n_tq; q += 64) s_tq[q] = c.tq[q];
    const int ut = lane < T ? c.utypes[lane] : INT_MIN;
    const int srv = c.master + lane;
    const bool mine = lane < S;
    int qlen = mine ? c.qm_qlen[lane] : 0;
    int rfo = (mine && srv < c.num_world) ? ld_agent(c.rfr_out + srv) : 1;
    __builtin_amdgcn_wave_barrier();
    int rowmax = LOWEST;
    if (mine)
        for (int t = 0; t < T; t++) rowmax = max(rowmax, s_hi[lane * T + t]);
    const bool self = srv == c.my_world;
    auto eligible = [&]() { return mine && !self && !rfo && qlen > 0; };
    auto any_open = [&]() { return c.n_tq > 0 || __ballot(eligible() && rowmax > LOWEST) != 0ull; };
    // find_cand from the staged state (wave-uniform): tq first, then the argmax over servers
    auto cand_of = [&](int rank, int wt) -> int {
        for (int base = 0; base < c.n_tq; base += 64) {
            const int k = base + lane;
            bool hit = false;
            int sv = -1;
            if (k < c.n_tq) {
                hit = s_tq[4 * k] == rank && (wt == -1 || wt == s_tq[4 * k + 1]);
                sv = s_tq[4 * k + 2];
            }
            const unsigned long long b = __ballot(hit);
            if (b) return __shfl(sv, __ffsll((long long)b) - 1, 64);
        }
        int ti = -1;
        if (wt >= 0) {
            const unsigned long long b = __ballot(lane < T && ut == wt);
            if (!b) return -1;  // undeclared type
            ti = __ffsll((long long)b) - 1;
        }
        unsigned long long key = 0;
        if (eligible()) {
            const int v = wt < 0 ? rowmax : s_hi[lane * T + ti];
            if (v > LOWEST)
                key = ((unsigned long long)((unsigned int)v ^ 0x80000000u) << 32) | (0xffffffffull - (unsigned int)lane);
        }
        key = wave_max_u64(key);
        return key ? c.master + (int)(0xffffffffu - (unsigned int)(key & 0xffffffffu)) : -1;
    };
    int k = n0;
    bool open = any_open();
    for (int k0 = n0; k0 < n0 + np && open; k0 += 64) {
        // the next 64 parked Reserves: request index, rank, its rfr_to_rank, type vector
        __builtin_amdgcn_s_waitcnt(0);  // the last batch's rfr stores have reached L2 before these loads
        const int kk = k0 + lane;
        const bool in = kk < n0 + np;
        const int j = in ? rq_req[kk] : 0;
        const int *rr = reqs + (long long)ADLBQ_RESERVE_INTS * j;
        const int rank = in ? rr[0] : -1;
#pragma unroll
        for (int e = 0; e < NREQ; e++) s_tv[lane * NREQ + e] = in ? rr[2 + e] : -2;
        int rtr = (in && rank >= 0 && rank < c.A) ? ld_agent(c.rfr_to_rank + rank) : 0;
        const int kn = min(64, n0 + np - k0);
        __builtin_amdgcn_wave_barrier();  // one wave owns s_tv: its LDS ops complete in order
        for (int i = 0; i < kn && open; i++, k++) {
            const int rk = __builtin_amdgcn_readlane(rank, i), jj = __builtin_amdgcn_readlane(j, i);
            int cand = -1;
            if (rk >= 0 && rk < c.A && __builtin_amdgcn_readlane(rtr, i) < 0) {
                for (int e = 0; e < NREQ; e++) {
                    const int wt = s_tv[i * NREQ + e];
                    if (wt < -1) break;
                    cand = cand_of(rk, wt);
                    if (cand >= 0) break;
                }
                if (cand >= 0) {  // rfr_to_rank[rank] = cand, rfr_out[cand] = 1 (adlb.c:1300-1304)
                    if (lane == 0) {
                        st_agent(c.rfr_to_rank + rk, cand);
                        if (cand < c.num_world) st_agent(c.rfr_out + cand, 1);
                    }
                    if (mine && srv == cand) rfo = 1;
                    if (rank == rk) rtr = cand;  // this rank's later Reserves see the RFR outstanding
                }
            }
            if (lane == 0) resp[(long long)ADLBQ_RESP_INTS * jj + 11] = cand;
            if (cand >= 0 && c.n_tq == 0) open = any_open();
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    return k;
}

__device__ void park_tail(const DonorCtx &c, int donors, const int *__restrict__ reqs, int R,
                          const unsigned long long *pmask, int *rq_rank, int *rq_types, int *rq_live, int *rq_req,
                          int *rq_seq, DevCounters *ctr, int *resp) {
    __shared__ int wsum[16];
    __shared__ int s_n0, s_total, s_stop, s_seq0;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nth = blockDim.x;
    // the parked requests are the set bits of the per-wave ballots every
    // workgroup published (pmask[j >> 6]); thread tid takes a contiguous run
    // of words so that rq order is request order
    const int nw = (R + 63) / 64, per = (nw + nth - 1) / nth, w0 = min(nw, tid * per), w1 = min(nw, w0 + per);
    constexpr int MAXW = 8;  // per <= 8 words held in registers (R <= 131072 at 256 threads)
    unsigned long long bits[MAXW];
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < MAXW; q++) {
        bits[q] = w0 + q < w1 ? __hip_atomic_load(pmask + w0 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        cnt += __popcll(bits[q]);
    }
    for (int q = w0 + MAXW; q < w1; q++)  // larger batches: the rest straight from memory
        cnt += __popcll(__hip_atomic_load(pmask + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    int x = cnt;  // block exclusive scan of cnt
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    if (tid == 0) {
        s_n0 = ctr->rq_n;
        s_seq0 = ctr->rq_next;
    }
    __syncthreads();
    int wpre = 0;
    for (int q = 0; q < w; q++) wpre += wsum[q];
    if (tid == nth - 1) s_total = wpre + x;
    int pos = s_n0 + wpre + x - cnt;
    for (int q = w0; q < w1; q++) {
        unsigned long long b = q - w0 < MAXW ? bits[q - w0]
                                             : __hip_atomic_load(pmask + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // read for the last time: zero again for the next batch (its waves write only non-zero words)
        if (b) __hip_atomic_store(const_cast<unsigned long long *>(pmask) + q, 0ull, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        for (; b; b &= b - 1) {
            const int jj = q * 64 + __ffsll((long long)b) - 1;
            const int *rq = reqs + (long long)ADLBQ_RESERVE_INTS * jj;
            rq_rank[pos] = rq[0];
            for (int k = 0; k < NREQ; k++) rq_types[(long long)pos * NREQ + k] = rq[2 + k];
            rq_live[pos] = 1;
            rq_req[pos] = jj;
            const int seq = s_seq0 + (pos - s_n0) + 1;  // next_rqseqno++ (adlb.c:1244)
            rq_seq[pos] = seq;
            resp[(long long)ADLBQ_RESP_INTS * jj + 10] = seq;
            pos++;
        }
    }
    __threadfence();
    __syncthreads();
    const int n0 = s_n0, np = s_total;
    // the RFR donors in FIFO order (rfr_out / rfr_to_rank chain them); once no
    // server can be a donor any more (each RFR sets rfr_out), the rest get -1
    // in parallel
    __shared__ int s_hi[ADLBQ_MAX_TYPES * 64], s_tq[4 * DONOR_TQ_LDS], s_tv[64 * NREQ];
    if (w == 0 && donors && c.S <= 64 && c.T <= ADLBQ_MAX_TYPES && c.n_tq <= DONOR_TQ_LDS) {
        const int k = park_donors_fast(c, reqs, rq_req, n0, np, resp, s_hi, s_tq, s_tv);
        if (lane == 0) s_stop = k;
    } else if (w == 0) {
        bool open = donors && (c.n_tq > 0 || any_donor(c));
        int k = n0;
        for (; k < n0 + np && open; k++) {
            const int j = rq_req[k];
            const int *rr = reqs + (long long)ADLBQ_RESERVE_INTS * j;
            const int rank = rr[0];
            int cand = -1;
            if (rank >= 0 && rank < c.A && ld_agent(c.rfr_to_rank + rank) < 0)
                cand = rfr_select(c, rank, rr + 2);
            if (lane == 0) resp[(long long)ADLBQ_RESP_INTS * j + 11] = cand;
            if (cand >= 0 && c.n_tq == 0) open = any_donor(c);
        }
        if (lane == 0) s_stop = k;
    }
    __syncthreads();
    for (int k = s_stop + tid; k < n0 + np; k += nth) resp[(long long)ADLBQ_RESP_INTS * rq_req[k] + 11] = -1;
    if (tid == 0) {
        ctr->rq_n = n0 + np;
        ctr->rq_next += np;
        ctr->rq_live += np;
        bytes_add(ctr, BYTES_RQ * np);  // rq_node_create per parked Reserve (adlb.c:1244-1276)
        if (ctr->rq_live > ctr->rq_hwm) ctr->rq_hwm = ctr->rq_live;
        ctr->n_parked_last = np;
    }
}

struct FinArgs {
    const int *reqs;
    int R;
    const int *tmatch, *umatch, *cslot;
    uint32_t *meta;
    int *pin;
    int my_world;
    int *resp;
    DevCounters *ctr;
    DonorCtx dc;
    int donors;
    int *rq_rank, *rq_types, *rq_live, *rq_req, *rq_seq, *dem;
    int T;
    DevCounters *snap;
    unsigned long long snap_tag;
    long long *anchor, *anchor_next;
    unsigned long long *pmask;
    long long *gcut, *gcut_next;
    const int4 *rrec;
    const int *needsort;
    int *sortfail;
    int2 *mslot;  // [R] out: (slot, wqseqno) request j was given, or -1 (adlbq_unreserve_resp_device reads it back)
    const int2 *rh;  // [R] (rank, hang) as prep_block copied them: 8 B per request instead of a 72 B record stride
    int flat;        // grids up to this size arrive at one counter ("fin_flat"), larger ones by 8 groups
    int snap_diag;   // diagnostic ("fin_snap_diag"): the snapshot's host stores not drained before the tag
    int resp16;      // resp is 16-byte aligned (every row then is: 48 B each)
};

// k_rank gave up waiting for an in-launch candidate sort: the lists may be
// out of order, so the batch is answered ADLB_ERROR (nothing pinned, nothing
// parked) instead of with possibly wrong matches
__device__ __forceinline__ bool fin_failed(const FinArgs &f) {
    return __hip_atomic_load(f.sortfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// A chosen unit's bucket position must lie inside the open bucket's page list:
// every gathered position does.  One that does not is counted and fails the
// whole batch (k_finalize answers ADLB_ERROR, pins and parks nothing) instead of
// indexing past the list.  (The r05 fault on this path)
__device__ __forceinline__ bool pos_in_list(unsigned int pos, int npages, DevCounters *ctr, int *fail) {
    if ((int)(pos >> PAGE_SHIFT) < npages) return true;
    atomicAdd(&ctr->bound_faults, 1);
    __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
}

// Request j (j < R): pin its unit and write its response (rk, tm, um: its
// rh, tmatch and umatch entries, loaded by finalize_body).  A request that
// parks (no unit, hang) leaves words [10], [11] to the park tail.  Every
// writer of umatch gives a unit (cslot) with it: um >= 0 means slot >= 0.
__device__ __forceinline__ void fin_request(const FinArgs &f, int j, bool failed, int2 rk, int tm, int um) {
    const int rank = rk.x, hang = failed ? 0 : rk.y;
    const int slot = failed ? -1 : tm >= 0 ? tm : (um >= 0 ? f.cslot[um] : -1);
    int o[ADLBQ_RESP_INTS] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -1, -1};
    if (failed) {
        o[0] = -1;  // ADLB_ERROR
    } else if (slot >= 0) {
        f.pin[slot] = rank;  // adlb.c:1210-1212
        if (rank >= 0) __hip_atomic_fetch_or(f.meta + slot, M_PINNED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int4 c0 = f.rrec[2ll * slot], c1 = f.rrec[2ll * slot + 1];  // one 32 B record
        o[0] = 1;
        o[1] = c1.z;
        o[2] = c1.w;
        o[3] = c0.y;
        o[4] = c0.x;
        o[5] = c0.z;
        o[6] = f.my_world;
        o[7] = c0.w;
        o[8] = c1.x;
        o[9] = c1.y;
    } else if (!hang) {
        o[0] = -2;  // NO_CURR_WORK
    }
    f.mslot[j] = make_int2(slot, o[5]);
    const bool parks = slot < 0 && hang;
    int *out = f.resp + (long long)ADLBQ_RESP_INTS * j;
    if (f.resp16) {  // 16-byte aligned rows: three (or two and a half) vector stores instead of twelve
        int4 *o4 = reinterpret_cast<int4 *>(out);
        o4[0] = make_int4(o[0], o[1], o[2], o[3]);
        o4[1] = make_int4(o[4], o[5], o[6], o[7]);
        if (!parks) o4[2] = make_int4(o[8], o[9], -1, -1);
        else *reinterpret_cast<int2 *>(out + 8) = make_int2(o[8], o[9]);  // [10], [11]: the park tail
        return;
    }
#pragma unroll
    for (int i = 0; i < 10; i++) out[i] = o[i];
    if (!parks) {
        out[10] = -1;
        out[11] = -1;
    }
}

// Two-level arrival of workgroup bid of nb (8 groups, then one top counter)
// keeps every counter's atomics to about nb / 8; a count rides in the high
// half.  One thread; returns (parked in the batch << 32) | 1 for the last.
// fin_arrive in two halves: the first atomic (issue), then what its result decides (finish)
__device__ __forceinline__ unsigned long long fin_arrive_issue(const FinArgs &f, int parked, unsigned int nb,
                                                               unsigned int bid) {
    // an index the compiler must treat as per-lane: its wave-level atomic optimisation (one lane's
    // atomic, the result broadcast with readfirstlane) would wait for the result right here
    int z = 0;
    asm volatile("" : "+v"(z));
    unsigned long long *c = nb <= (unsigned int)f.flat ? &f.ctr->fin_top : &f.ctr->fin_group[bid & 7u];
    return atomicAdd(c + z, ((unsigned long long)parked << 32) | 1ull);
}
__device__ __forceinline__ unsigned long long fin_arrive_finish(const FinArgs &f, int parked, unsigned int nb,
                                                                unsigned int bid, unsigned long long v) {
    if (nb <= (unsigned int)f.flat)
        return (unsigned int)v == nb - 1u ? ((((v >> 32) + (unsigned long long)parked) << 32) | 1ull) : 0ull;
    const unsigned int g = bid & 7u, ng = (nb - g + 7u) / 8u, ngroups = min(nb, 8u);
    if ((unsigned int)v == ng - 1u) {
        const unsigned long long tg = (v >> 32) + (unsigned long long)parked;
        const unsigned long long top = atomicAdd(&f.ctr->fin_top, (tg << 32) | 1ull);
        if ((unsigned int)top == ngroups - 1u) return (((top >> 32) + tg) << 32) | 1ull;
    }
    return 0ull;
}
__device__ __forceinline__ unsigned long long fin_arrive(const FinArgs &f, int parked, unsigned int nb,
                                                         unsigned int bid) {
    if (nb <= (unsigned int)f.flat) {  // a small grid: one counter, one returning atomic per workgroup
        const unsigned long long top = atomicAdd(&f.ctr->fin_top, ((unsigned long long)parked << 32) | 1ull);
        return (unsigned int)top == nb - 1u ? ((((top >> 32) + (unsigned long long)parked) << 32) | 1ull) : 0ull;
    }
    const unsigned int g = bid & 7u, ng = (nb - g + 7u) / 8u, ngroups = min(nb, 8u);
    unsigned long long v = atomicAdd(&f.ctr->fin_group[g], ((unsigned long long)parked << 32) | 1ull);
    if ((unsigned int)v == ng - 1u) {
        const unsigned long long tg = (v >> 32) + (unsigned long long)parked;
        const unsigned long long top = atomicAdd(&f.ctr->fin_top, (tg << 32) | 1ull);
        if ((unsigned int)top == ngroups - 1u) return (((top >> 32) + tg) << 32) | 1ull;
    }
    return 0ull;
}

// The last workgroup of the batch (every thread of it): anchors and cuts for
// the next scan, the parked Reserves, counters, then the counter snapshot.
__device__ __forceinline__ void fin_tail(const FinArgs &f, int total, bool failed) {
    const int T = f.T;
    if ((int)threadIdx.x < T) {
        f.dem[threadIdx.x] = 0;  // prep_block of the next batch accumulates into it
        const long long a = f.anchor_next[threadIdx.x];
        if (a != LLONG_MIN) {  // lower the anchor to the live maximum k_thresholds saw
            f.anchor[threadIdx.x] = a;
            f.anchor_next[threadIdx.x] = LLONG_MIN;
        }
        const long long g = f.gcut_next[threadIdx.x];
        if (g != LLONG_MIN) {  // the next scan's pass-1 guess
            f.gcut[threadIdx.x] = g;
            f.gcut_next[threadIdx.x] = LLONG_MIN;
        }
    }
    int nsl = 0;  // every type's sort flag at once (one thread's loop waited for each load in turn)
    for (int t = threadIdx.x; t < T; t += blockDim.x) nsl |= f.needsort[t];
    if (total > 0)
        park_tail(f.dc, f.donors, f.reqs, f.R, f.pmask, f.rq_rank, f.rq_types, f.rq_live, f.rq_req, f.rq_seq, f.ctr,
                  f.resp);
    const int ns = __syncthreads_or(nsl != 0);
    if (threadIdx.x == 0) {
        DevCounters *ctr = f.ctr;
        if (failed) {
            ctr->batch_failed += 1;
            __hip_atomic_store(f.sortfail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // per batch
        }
        if (total == 0) ctr->n_parked_last = 0;
        ctr->needsort_last = ns ? 1 : 0;  // the host launches the segmented sort while this holds
        for (int g = 0; g < 8; g++) ctr->fin_group[g] = 0;
        ctr->fin_top = 0;
    }
    if (threadIdx.x < 64) {
        // mapped host memory: every field (sc1 loads: fields other XCDs' waves stored in this
        // launch when the finalize rides in the chain), then the tag the host waits for
        static_assert(sizeof(DevCounters) % 4 == 0, "DevCounters copies as ints");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int *src = reinterpret_cast<const int *>(f.ctr);
        int *dst = reinterpret_cast<int *>(f.snap);
        constexpr int NW = (int)(sizeof(DevCounters) / 4), NR = (NW + 63) / 64;
        int v[NR];  // every load in flight before the first store
#pragma unroll
        for (int q = 0; q < NR; q++) v[q] = threadIdx.x + 64 * q < NW ? ld_sc1(src + threadIdx.x + 64 * q) : 0;
#pragma unroll
        for (int q = 0; q < NR; q++)
            if (threadIdx.x + 64 * q < NW) dst[threadIdx.x + 64 * q] = v[q];
        if (f.snap_diag) {  // timing diagnostic only: no drain, no release (a torn snapshot may land)
            if (threadIdx.x == 0) __hip_atomic_store(&f.snap->snap_tag, f.snap_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // the tag's system-scope release store orders the wave's drained snapshot stores before it
        if (threadIdx.x == 0)
            __hip_atomic_store(&f.snap->snap_tag, f.snap_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Which requests park is known from tmatch / umatch alone: the park mask is
// published and the workgroup arrives first, then the units are pinned and the
// responses written (their loads and stores overlap the arrival, and the last
// workgroup's tail -- which reads only the park mask -- overlaps theirs).
__device__ __forceinline__ void finalize_body(FinArgs f, const int bid_, const int nbk_) {
    __shared__ int s_parked;
    __shared__ unsigned long long s_ticket;
    const int j = bid_ * blockDim.x + threadIdx.x;
    if (threadIdx.x == 0) s_parked = 0;
    // the request's rows first (unconditional, clamped; the past-the-end lanes' values replaced after),
    // then the batch's failure flag: loaded first, it was waited for before these were issued
    const int jc = j < f.R ? j : 0;
    int2 rk = f.rh[jc];
    int tm = f.tmatch[jc], um = f.umatch[jc];
    const bool failed = fin_failed(f);
    unsigned int in = j < f.R ? 1u : 0u;
    asm volatile("" : "+v"(in));  // opaque to the optimiser (no select sunk into a branch around the loads)
    if (!in) rk = make_int2(-1, 0), tm = -1, um = -1;
    __syncthreads();
    if (j < f.R) {
        const bool parks = !failed && rk.y && tm < 0 && um < 0;
        const unsigned long long pb = __ballot(parks);
        if ((threadIdx.x & 63) == 0 && pb) {
            // published for the last workgroup's park (write-through, drained before the arrival below);
            // a wave with nothing parked writes nothing: park_tail zeroes the words it read, so every word
            // is zero at the start of a batch
            __hip_atomic_store(f.pmask + (j >> 6), pb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicAdd(&s_parked, __popcll(pb));
            __builtin_amdgcn_s_waitcnt(0);  // this wave's store has landed before the block arrives
        }
    }
    __syncthreads();
    // the arrival's first atomic goes out, the request's loads and stores follow, and its result is
    // looked at only after them (the two used to run one after the other in wave 0)
    unsigned long long v;  // read by thread 0 only (no value on the other lanes: nothing to merge at the join)
    const int parked = s_parked;
    if (threadIdx.x == 0) v = fin_arrive_issue(f, parked, nbk_, bid_);
    if (j < f.R) fin_request(f, j, failed, rk, tm, um);
    if (threadIdx.x == 0) s_ticket = fin_arrive_finish(f, parked, nbk_, bid_, v);
    __syncthreads();
    if (!(s_ticket & 1ull)) return;
    fin_tail(f, (int)(s_ticket >> 32), failed);
}

__global__ __launch_bounds__(256) void k_finalize(FinArgs f) {
    finalize_body(f, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------- one Reserve against a large open bucket
// A batch of one Reserve (T <= 8, no targeted units, an open bucket too large
// for k_reserve_small) in one launch instead of the seven of the pipeline.
// At most 256 workgroups step through the bucket's page pairs in bucket order
// (256 threads, 32 units each per pair, all loads in flight) and find each
// type's best available unit by (prio desc, bucket position asc) --
// wq_find_hi_prio's order (xq.c:190-217), the pipeline's key -- folding each
// pair's minima into per-type global ones (agent-scope atomic min).  A
// workgroup stops once every type the Reserve names has its best unit so far
// at the type's anchor (the upper bound of its available priorities) before
// its next pair: nothing later can come first.  On a queue whose top
// priority is common that is within the first round of pairs; with a stale
// anchor the whole bucket is read, as before.  The last workgroup to arrive
// prepares the request (prep_block), takes the best head among its types, and
// finalizes it as k_finalize would (pin, response, park, counters, snapshot).
struct OneArgs {
    PrepArgs pa;
    const int *pages; int npages, tail_fill;
    int pg0;                   // >= 0: the open pages are pg0, pg0 + 1, ... (no page-table read before the loads)
    const int *prio; const uint32_t *meta; const int *pbase, *pwide;
    int T;
    unsigned long long *part;  // [8] per-type best key over the workgroups (atomic min; ~0 between launches)
    int *arrive;               // [9] arrival counters: eight groups, then the top (the last workgroup resets them)
    int *umatch, *cslot;
    FinArgs f;
    int inject;  // test only: the choice is told a position past the page list
    const uint32_t *zero;  // 16 KB of zeros: the meta read for a group past the open pages
};
template <int TB>
__global__ __launch_bounds__(256, 2) void k_reserve_one(OneArgs a) {  // at most 256 workgroups (one_grid)
    static_assert(TB <= 8, "T <= 8");
    __shared__ unsigned long long smin[4][8];
    __shared__ unsigned long long s_want;
    __shared__ long long s_anc[8];
    __shared__ int s_last, s_skip;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int npairs = (a.npages + 1) / 2;
    unsigned long long *const gbest = a.part;  // [8] per-type best key over the workgroups (atomic min)
    // wave 0: the Reserve's types (a superset of prep_block's mask: every type whose value a slot
    // names, every type for a -1) and the anchors (upper bounds of the available priorities)
    if (w == 0) {
        const int v = a.pa.reqs[2 + (lane < NREQ ? lane : 0)];
        const int ut = a.pa.utypes[lane < a.T ? lane : 0];
        const long long an = a.f.anchor[lane < a.T ? lane : 0];
        const bool wild = __ballot(lane < NREQ && v == -1) != 0ull;
        unsigned long long want = 0ull;
#pragma unroll
        for (int q = 0; q < NREQ; q++) want |= __ballot(lane < a.T && ut == __shfl(v, q, 64));
        if (wild) want = (1ull << a.T) - 1;
        if (lane == 0) s_want = want;
        if (lane < 8) s_anc[lane] = lane < a.T ? an : LLONG_MAX;
    }
    __syncthreads();
    const unsigned long long want = s_want;
    // Page pairs in bucket order, gridDim.x workgroups at a time.  A pair is skipped (and so every later
    // one of this workgroup) once each wanted type's best unit so far sits at its anchor's priority
    // before the pair: no unit of the pair can come first (prio desc, then bucket position asc).
    for (int pair = blockIdx.x; pair < npairs; pair += gridDim.x) {
        if (w == 0) {
            bool open_t = false;
            if (lane < TB && ((want >> lane) & 1ull)) {
                const unsigned long long gb = (unsigned long long)__hip_atomic_load(
                    (long long *)(gbest + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const long long an = s_anc[lane];
                const bool at_anchor = an >= (long long)INT_MIN && an <= (long long)INT_MAX &&
                                       (unsigned int)(gb >> 32) == ~((unsigned int)(int)an ^ 0x80000000u);
                open_t = !(gb != ~0ull && at_anchor && (unsigned int)gb < ((unsigned int)(2 * pair) << PAGE_SHIFT));
            }
            const unsigned long long ob = __ballot(open_t);
            if (lane == 0) s_skip = ob == 0ull;
        }
        __syncthreads();
        if (s_skip) break;
        unsigned long long kmin[TB];
#pragma unroll
        for (int u = 0; u < TB; u++) kmin[u] = ~0ull;
        {
            // groups of 4 units: the pair's two pages hold 2 x 1024; thread tid takes g = tid + 256 i
            uint4 mv[8];
            int4 pv[8];
            int pb[2], wide[2], pg[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int p = 2 * pair + h;
                pg[h] = p >= a.npages ? -1 : a.pg0 >= 0 ? a.pg0 + p : a.pages[p];
                pb[h] = pg[h] >= 0 ? a.pbase[pg[h]] : 0;
                wide[h] = pg[h] >= 0 ? a.pwide[pg[h]] : 0;
            }
            // unconditional meta loads, a group past the open pages reading zeros (nothing LIVE): a load
            // inside a per-lane branch made the compiler wait for each before the next, and a mask per
            // group cost the registers of a fifth wave per SIMD; the prio column only on a wide page
            // (h = i / 4 is uniform: one branch per page)
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int g = tid + 256 * i, h = g >> 10, gi = g & 1023, p = 2 * pair + h;
                const int fill = p == a.npages - 1 ? a.tail_fill : PAGE;
                const bool ok = pg[h] >= 0 && gi * 4 < fill;
                const uint32_t *src = ok ? a.meta + ((long long)pg[h] << PAGE_SHIFT) : a.zero;
                mv[i] = reinterpret_cast<const uint4 *>(src)[gi];
                pv[i] = make_int4(0, 0, 0, 0);
            }
#pragma unroll
            for (int h = 0; h < 2; h++) {
                if (pg[h] >= 0 && wide[h]) {
                    const long long base = (long long)pg[h] << PAGE_SHIFT;
#pragma unroll
                    for (int i = 4 * h; i < 4 * h + 4; i++) {
                        const int gi = (tid + 256 * i) & 1023;
                        pv[i] = reinterpret_cast<const int4 *>(a.prio + base)[gi];  // masked through mv below
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int g = tid + 256 * i, h = g >> 10, gi = g & 1023, p = 2 * pair + h;
                const uint32_t mm[4] = {mv[i].x, mv[i].y, mv[i].z, mv[i].w};
                const int pw[4] = {pv[i].x, pv[i].y, pv[i].z, pv[i].w};
#ifdef ADLBQ_ONE_MEMONLY  // timing diagnostic only (wrong results): the loads without the comparisons
                kmin[0] ^= (unsigned long long)(mm[0] ^ mm[1] ^ mm[2] ^ mm[3] ^ pw[0]);
                continue;
#endif
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int pr = wide[h] ? pw[q] : pb[h] + (int)(mm[q] >> M_OFF_SHIFT);
                    if ((mm[q] & (M_LIVE | M_PINNED)) != M_LIVE || pr <= LOWEST) continue;
                    const int t = (int)(mm[q] & M_TYPE);
                    const unsigned long long key = ((unsigned long long)(~((unsigned int)pr ^ 0x80000000u)) << 32) |
                                                   ((unsigned long long)(unsigned int)p << PAGE_SHIFT) |
                                                   (unsigned long long)(gi * 4 + q);
#pragma unroll
                    for (int u = 0; u < TB; u++)  // only the types the Reserve names (a uniform test)
                        if (((want >> u) & 1ull) && t == u) kmin[u] = min(kmin[u], key);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < TB; u++) {
            if (!((want >> u) & 1ull)) continue;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) kmin[u] = min(kmin[u], (unsigned long long)__shfl_xor((long long)kmin[u], o, 64));
            if (lane == 0) smin[w][u] = kmin[u];
        }
        __syncthreads();
        if (tid < TB && ((want >> tid) & 1ull)) {  // the pair's minima into the per-type global ones (agent scope)
            const unsigned long long m = min(min(smin[0][tid], smin[1][tid]), min(smin[2][tid], smin[3][tid]));
            if (m != ~0ull) __hip_atomic_fetch_min(gbest + tid, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    if (tid == 0) {  // two-level arrival: eight group counters, then the top one (a.arrive[8])
        // The minima go out as sc1 (agent-scope) stores drained by vmcnt(0) before the arrival, and the
        // last workgroup reads them with sc1 (agent-scope atomic) loads: MI355X_MICROARCH.md's valid
        // hand-off form without a release / acquire pair.  An acq_rel arrival cost every workgroup an
        // L2 write-back and invalidate (~10 us on the one-Reserve latency, measured).
        const unsigned int nb = gridDim.x, g = blockIdx.x & 7u, ng = (nb - g + 7u) / 8u, ngroups = min(nb, 8u);
        int last = 0;
        if ((unsigned int)__hip_atomic_fetch_add(a.arrive + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ng - 1u)
            last = (unsigned int)__hip_atomic_fetch_add(a.arrive + 8, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   ngroups - 1u;
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    if (tid <= 8) a.arrive[tid] = 0;  // for the next launch (kernel boundary in between)
#ifdef ADLBQ_ONE_DIAG  // timing diagnostic only (wrong results): the scan and the arrival alone
    return;
#endif
    // ---- the last workgroup: the request, every workgroup's minima, the choice, its finalize
    prep_block<TB>(a.pa, 0);
    // the per-type minima every workgroup folded in (agent-scope atomic loads; every workgroup has
    // arrived), then reset for the next launch
    unsigned long long gm = ~0ull;
    if (tid < TB) {
        gm = (unsigned long long)__hip_atomic_load((long long *)(gbest + tid), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gbest + tid, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // a wanted type's best unit is its highest available priority: the anchor comes down to it (after
        // an early stop it is the anchor already), so the next one-Reserve batch can stop early again
        // instead of reading the whole bucket behind a stale anchor
        if (((want >> tid) & 1ull) && gm != ~0ull) {
            const long long pr = (long long)(int)(~(unsigned int)(gm >> 32) ^ 0x80000000u);
            if (pr < a.f.anchor[tid]) a.f.anchor[tid] = pr;
        }
    }
    __syncthreads();  // prep_block's outputs, and smin free again
    if (tid < TB) smin[0][tid] = gm, smin[1][tid] = ~0ull, smin[2][tid] = ~0ull, smin[3][tid] = ~0ull;
    __syncthreads();
    const FinArgs &f = a.f;
    if (tid == 0) {
        const unsigned long long m = a.pa.mask[0];
        unsigned long long best = ~0ull;
#pragma unroll
        for (int u = 0; u < TB; u++) {
            const unsigned long long k = min(min(smin[0][u], smin[1][u]), min(smin[2][u], smin[3][u]));
            if (u < a.T && ((m >> u) & 1ull)) best = min(best, k);
        }
        int um = -1;
        bool bad = false;
        if (best != ~0ull) {
            const int p = a.inject ? a.npages : (int)((best >> PAGE_SHIFT) & 0xfffffu), sl = (int)(best & (PAGE - 1));
            if (pos_in_list((unsigned int)p << PAGE_SHIFT, a.npages, f.ctr, f.sortfail)) {
                a.cslot[0] = (a.pages[p] << PAGE_SHIFT) | sl;
                um = 0;
            } else {
                bad = true;  // answered ADLB_ERROR below; fin_tail resets the flag
            }
        }
        a.umatch[0] = um;
        const int2 rk = f.rh[0];
        const bool parks = !bad && rk.y && um < 0;
        if (parks) __hip_atomic_store(f.pmask, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // zero otherwise
        fin_request(f, 0, bad, rk, -1, um);
        s_last = (parks ? 1 : 0) | (bad ? 2 : 0);
    }
    __syncthreads();
    fin_tail(f, s_last & 1, (s_last & 2) != 0);
}

// Round 0: every segment from its level guess (lane t = type t's head), then
// passes 2 .. P in the same launch: segment s waits for segment s-1's end of
// the previous pass and re-solves (seeded) only if it differs from its own
// start; finally each segment checks its start against its predecessor's last
// end.  A launch in which every check holds is the fixed point.
template <int TB>
__device__ __forceinline__ void chain0_body(ChainArgs a, ChainPass cp, int prefix_next, int final, const int bid_,
                                            const int nbk_) {
    extern __shared__ unsigned int win[];
    const int lane = threadIdx.x, T = a.T, s = bid_, nseg = a.nseg, P = cp.passes;
    chain_stamp(a, s, 0);
    if (s == 0 && lane == 0) *a.clean = 0;
    if constexpr (TB <= 8) win[TB * (SEG + a.warm) + lane] = ~0u;  // seg_solve_small's sentinel row
    int rounds = 0;
    const int jb = max(0, s * SEG - a.warm);  // a.warm is a multiple of SEG
    // the type masks of [jb, segment end) in flight with the guess's loads (T <= 8: staged in LDS)
    constexpr int NRB = TB <= 8 ? (SEG + CHAIN_WARM) / 64 : 1;
    unsigned long long mk[NRB];
    int tm[NRB];
    const int j1 = min(a.R, s * SEG + SEG);
    if constexpr (TB <= 8) {
        // unconditional loads (clamped index, masked after with masks opaque to the optimiser): a load
        // under a per-lane condition was issued only after the one before had returned
        unsigned int okm = 0u;
#pragma unroll
        for (int i = 0; i < NRB; i++) {
            const int j = jb + i * 64 + lane;
            okm |= (j < j1 ? 1u : 0u) << i;
            mk[i] = a.mask[j < j1 ? j : 0];
            tm[i] = a.tmatch[j < j1 ? j : 0];
        }
        asm volatile("" : "+v"(okm));
#pragma unroll
        for (int i = 0; i < NRB; i++) {
            const unsigned int b = (okm >> i) & 1u;
            mk[i] &= 0ull - (unsigned long long)b;
            tm[i] &= 0 - (int)b;
        }
    }
    // lane t: type t's list offset and length (lane T: the total), all loads of the prologue in flight together
    unsigned int lm = (lane <= T ? 1u : 0u) | (lane < T ? 2u : 0u);
    int my_off = a.candoff[lane <= T ? lane : 0], my_len = a.candlen[lane < T ? lane : 0];
    asm volatile("" : "+v"(lm));
    my_off &= 0 - (int)(lm & 1u);
    my_len &= 0 - (int)((lm >> 1) & 1u);
    // J from the prefix k_thresholds left, unless k_rank changed seg_cnt since (a type with no candidate)
    const int jpv = a.jpref != nullptr ? a.jpref[jb >> 6] : 0;
    const bool use_jp = a.jpref != nullptr && __ballot(lane < T && my_len == 0) == 0ull;
    if (a.rdone != nullptr) {
        // k_rank's blocks ride in this launch (k_rank_chain0).  They write what the chain reads (ranks, level
        // rows, seg_cnt) only when k_select_open did not rank the candidates, a list needs sorting or a type
        // has no candidate at all -- the conditions of rank_body's own early return; then wait for every
        // rank block's arrival (release there, acquire here: MI355X_MICROARCH.md, inter-workgroup visibility)
        const int ns = lane < T ? a.needsort[lane] : 0;
        const bool slow = ld_sc1(&a.ctr->rank_fast) == 0 || __ballot(ns == 1 && my_len > 1) != 0ull ||
                          __ballot(lane < T && my_len == 0) != 0ull;
        if (slow) {
            if (lane == 0) {
                while (__hip_atomic_load(a.rdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.rtarget)
                    __builtin_amdgcn_s_sleep(2);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_wave_barrier();
            __syncthreads();
        }
    }
    int J = 0;  // requests before jb that take an untargeted unit
    if (use_jp) {
        J = jpv;
    } else {
        const int nq = jb >> 6;
        int cv[16];
#pragma unroll
        for (int u = 0; u < 16; u++) cv[u] = u * 64 + lane < nq ? a.seg_cnt[u * 64 + lane] : 0;
#pragma unroll
        for (int u = 0; u < 16; u++) J += cv[u];
        for (int q = 1024 + lane; q < nq; q += 64) J += a.seg_cnt[q];  // batches above 65,536 Reserves
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) J += __shfl_xor(J, o, 64);
    }
    int guess;
    if (a.lv != nullptr) {  // T <= 8: the level state at J is k_rank's row J (every head at one level)
        const int G = __builtin_amdgcn_readlane(my_off, T);
        // the row at the sampled rank below J, the rest spread in proportion to the list lengths
        const int Js = J & ~(LV_STEP - 1);
        // ranks [Js, J): one type byte per lane, counted per type (LV_STEP == 64)
        const int tt = (Js + lane < J && Js + lane < G) ? (int)a.rtype[Js + lane] : 255;
        int extra = 0;
#pragma unroll
        for (int q = 0; q < (TB <= 8 ? TB : 8); q++) {
            const int c = __popcll(__ballot(tt == q));
            if (lane == q) extra = c;
        }
        guess = lane >= T || J == 0 ? 0
                : J >= G            ? my_len
                                    : min(my_len, (Js ? a.lv[(long long)(Js / LV_STEP) * T + lane] : 0) + extra);
    } else {
        guess = level_guess<(TB <= 8 ? TB : 8)>(a, J);
    }
    if constexpr (TB <= 8) {
        unsigned long long *smk = staged_masks<TB>(a, win);
#pragma unroll
        for (int i = 0; i < NRB; i++)
            if (jb + i * 64 < j1) smk[i * 64 + lane] = tm[i] < 0 ? mk[i] : 0ull;
    }
    chain_stamp(a, s, 1);
    int start;
    int end = seg_solve<TB>(a, s, jb, guess, win, false, TB > 8, 0, my_off, my_len, start, rounds);
    chain_stamp(a, s, 2);
    int solves = 0, timeouts = 0;
    auto E = [&](int k, int q) { return cp.E + ((long long)k * nseg + q) * T; };
    auto F = [&](int k, int q) { return cp.flags + (long long)k * nseg + q; };
    publish_state(E(0, s), F(0, s), cp.epoch, end, T);
    for (int k = 1; k < P; k++) {
        if (s > 0) {
            if (wait_flag(F(k - 1, s - 1), cp.epoch)) {
                const int pe = lane < T ? ld_sc1(E(k - 1, s - 1) + lane) : 0;
                if (__ballot(lane < T && pe != start)) {
                    int rec;
                    __builtin_amdgcn_wave_barrier();  // win is refilled
                    end = seg_solve<TB>(a, s, s * SEG, pe, win, true, TB > 8, s * SEG - jb, my_off, my_len, rec, rounds);
                    start = pe;
                    solves++;
                }
            } else {
                timeouts++;
            }
        }
        publish_state(E(k, s), F(k, s), cp.epoch, end, T);
    }
    chain_stamp(a, s, 3);
    // own check: the final start against the predecessor's final end
    int bad = 0;
    if (s > 0) {
        if (wait_flag(F(P - 1, s - 1), cp.epoch)) {
            const int pe = lane < T ? ld_sc1(E(P - 1, s - 1) + lane) : 0;
            bad = __ballot(lane < T && pe != start) ? 1 : 0;
        } else {
            timeouts++;
            bad = 1;  // unknown: a later round or the walk looks
        }
    }
    if (timeouts && lane == 0) atomicAdd(&a.ctr->chain_timeouts, timeouts);
    chain_stamp(a, s, 4);
    chain_arrive<TB>(a, s, start, end - start, solves, bad, rounds, 0, P, final != 0, prefix_next != 0, win);
    chain_stamp(a, s, 5);
}

template <int TB>
__global__ __launch_bounds__(64) void k_chain0(ChainArgs a, ChainPass cp, int prefix_next, int final) {
    chain0_body<TB>(a, cp, prefix_next, final, blockIdx.x, gridDim.x);
}

// k_rank and round 0 of the chain as one launch (T <= 8): blocks [0, rg) are
// k_rank's (64 threads each), the rest the chain's segments.  In the usual case
// (k_select_open ranked the candidates) the rank blocks have nothing the chain
// reads and the segments never wait; otherwise each segment waits for every
// rank block's arrival.  The segments cannot hold back a rank block: each CU
// has room for a rank block beside a segment, whatever the dispatch order.
template <int TB>
__global__ __launch_bounds__(64) void k_rank_chain0(RankArgs ra, int rg, ChainArgs a, ChainPass cp, int prefix_next,
                                                    int final) {
    if ((int)blockIdx.x < rg) {
        // whether the chain will wait for these blocks (its own test, read before rank_body changes any
        // flag: k_select_open did not rank the candidates, or a type has none): only then is there
        // anything to write back before the arrival (the release fence writes back the XCD's L2)
        const int lane = threadIdx.x;
        const int len = ra.candlen[lane < ra.T ? lane : 0];
        const bool slow = ld_sc1(&ra.ctr->rank_fast) == 0 || __ballot(lane < ra.T && len == 0) != 0ull;
        rank_body<64>(ra, blockIdx.x, rg);
        __syncthreads();
        if (threadIdx.x == 0) {  // one wave: its stores drained, written back, then the arrival
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (slow) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            atomicAdd(const_cast<unsigned long long *>(a.rdone), 1ull);
        }
        return;
    }
    chain0_body<TB>(a, cp, prefix_next, final, (int)blockIdx.x - rg, (int)gridDim.x - rg);
}

// ---------------------------------------------------------------- one launch per kernel for a group of handles
// adlbq_reserve_group_device: the reserve batches of several handles (a GPU
// process's server shards) go as ONE launch per pipeline kernel, grid.y =
// handle, each handle's arguments in a device table (launch_reserve records
// them instead of launching: GroupRec).  Blocks past a handle's own grid
// return at once; every body gets its handle's block index and grid size.
struct GPrep { PrepArgs pa; int nprep; HistArgs ha; int grid; };
struct GThr {
    unsigned int *zcs; long long zn; int T; const int *dem; unsigned int *csum; int nchunks;
    int *theta, *need, *candlen, *needsort, *binoff; unsigned int *coltot; int *type_cnt;
    const long long *anchor; long long *anchor_next, *gcut_next; int guess; int grid; const long long *gcut;
};
struct GSel {
    const int *pages; int npages, tail_fill; const int *prio; const uint32_t *meta; const int *seqa; int T;
    const long long *anchor; const int *theta, *need, *binoff; const unsigned int *csum; const unsigned short *gh;
    const int *candlen; int *candoff_out; unsigned long long *ckey; int *cslot; const long long *gcut;
    const unsigned int *spec; const int *specn, *pbase, *pwide; DevCounters *ctr; unsigned int *crank; int *lv;
    unsigned char *rtype; int R; int grid;
};
struct GRank { RankArgs ra; int grid; };
struct GChain { ChainArgs a; ChainPass cp; int prefix_next, final; int grid; };
struct GFin { FinArgs f; int grid; };

enum : int { GK_PREP = 1, GK_THR = 2, GK_SEL = 4, GK_RANK = 8, GK_CHAIN = 16, GK_FIN = 32 };
struct GroupRec {
    int kinds = 0;  // GK_* recorded
    int tb = 0;     // the TB of the templated kernels (4 or 8)
    GPrep prep; GThr thr; GSel sel; GRank rank; GChain chain; GFin fin;
    size_t lds_prep = 0, lds_sel = 0, lds_chain = 0;
    bool selw = false;  // pass 2 with one wave per page (k_select_wave), else four (k_select_open)
    size_t lds_sel_open = 0;  // k_select_open's LDS for this handle (a group of mixed shapes takes it)
};

template <int TB>
__global__ __launch_bounds__(256, hist_waves(TB) > 1 ? 5 : 1) void k_prep_hist_g(const GPrep *__restrict__ t) {
    const GPrep &g = t[blockIdx.y];
    if ((int)blockIdx.x >= g.grid) return;
    prep_hist_body<TB>(g.pa, g.nprep, g.ha, blockIdx.x);
}
__global__ __launch_bounds__(TH_THREADS) void k_thresholds_g(const GThr *__restrict__ t) {
    const GThr &g = t[blockIdx.y];
    if ((int)blockIdx.x >= g.grid) return;
    thresholds_body(g.zcs, g.zn, g.T, g.dem, g.csum, g.nchunks, g.theta, g.need, g.candlen, g.needsort, g.binoff,
                    g.coltot, g.type_cnt, g.anchor, g.anchor_next, g.gcut_next, g.guess, g.gcut, blockIdx.x, g.grid);
}
template <int TB>
__global__ __launch_bounds__(256) void k_select_open_g(const GSel *__restrict__ t) {
    const GSel &g = t[blockIdx.y];
    if ((int)blockIdx.x >= g.grid) return;
    select_open_body<TB>(g.pages, g.npages, g.tail_fill, g.prio, g.meta, g.seqa, g.T, g.anchor, g.theta, g.need,
                         g.binoff, g.csum, g.gh, g.candlen, g.candoff_out, g.ckey, g.cslot, g.gcut, g.spec, g.specn,
                         g.pbase, g.pwide, g.ctr, g.crank, g.lv, g.rtype, g.R, blockIdx.x, g.grid);
}
// the group twin of k_select_wave (T <= 8): one wave per page, blockIdx.y = shard
template <int TB>
__global__ __launch_bounds__(64) void k_select_wave_g(const GSel *__restrict__ t) {
    const GSel &g = t[blockIdx.y];
    if ((int)blockIdx.x >= g.npages) return;  // whole workgroups return together
    select_wave_body<TB>(g.pages, g.npages, g.tail_fill, g.prio, g.meta, g.T, g.anchor, g.theta, g.need, g.binoff,
                         g.csum, g.gh, g.candlen, g.candoff_out, g.ckey, g.cslot, g.gcut, g.spec, g.specn, g.pbase,
                         g.pwide, g.ctr, g.crank, g.lv, g.rtype, g.R, nullptr, blockIdx.x);
}
__global__ __launch_bounds__(RANK_TILE) void k_rank_g(const GRank *__restrict__ t) {
    const GRank &g = t[blockIdx.y];
    if ((int)blockIdx.x >= g.grid) return;
    rank_body<RANK_TILE>(g.ra, blockIdx.x, g.grid);
}
template <int TB>
__global__ __launch_bounds__(64) void k_chain0_g(const GChain *__restrict__ t) {
    const GChain &g = t[blockIdx.y];
    if ((int)blockIdx.x >= g.grid) return;
    chain0_body<TB>(g.a, g.cp, g.prefix_next, g.final, blockIdx.x, g.grid);
}
__global__ __launch_bounds__(256) void k_finalize_g(const GFin *__restrict__ t) {
    const GFin &g = t[blockIdx.y];
    if ((int)blockIdx.x >= g.grid) return;
    finalize_body(g.f, blockIdx.x, g.grid);
}

// ---------------------------------------------------------------- steal export
// The k best available units of every type for the cross-shard merge
// (SURVEY §8(e)): the two passes above with demand k for every type, then the
// first min(k, candlen) entries of each candidate list (preference order) as
// records {prio, wqseqno, work_type, len, answer_rank, common_len,
// common_server, common_seqno} -- the fields SS_RFR_RESP carries
// (adlb.c:1828-1840).  Block t gathers type t; the blocks also do what k_rank
// and k_finalize do after a batch's scan: zero the chunk sums, reset the
// demand, apply the anchors the thresholds found.
__global__ void k_export_begin(int *dem, int T, int k) {
    if ((int)threadIdx.x < T) dem[threadIdx.x] = k;
}

__global__ __launch_bounds__(256) void k_export_gather(int T, int k, const int *__restrict__ candoff,
                                                       const int *__restrict__ candlen, const int *__restrict__ cslot,
                                                       const int *__restrict__ prio, const int *__restrict__ seqa,
                                                       const int4 *__restrict__ cold0, const int4 *__restrict__ cold1,
                                                       int *__restrict__ recs, int *__restrict__ nrec,
                                                       long long *__restrict__ navail,
                                                       const unsigned int *__restrict__ coltot, int scanned,
                                                       unsigned int *csum, long long ncsum, int *dem,
                                                       long long *anchor, long long *anchor_next) {
    const int t = blockIdx.x;
    if (threadIdx.x < 64) {  // available units of type t: its column totals (k_thresholds)
        unsigned long long a = scanned ? coltot[t * NB + threadIdx.x] : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (threadIdx.x == 0) navail[t] = (long long)a;
    }
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < ncsum;
         i += (long long)gridDim.x * blockDim.x)
        csum[i] = 0;
    const int n = min(k, candlen[t]), off = candoff[t];
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int slot = cslot[off + i];
        const int4 c0 = cold0[slot], c1 = cold1[slot];
        int4 *r = reinterpret_cast<int4 *>(recs + ((long long)t * k + i) * 8);
        r[0] = make_int4(prio[slot], seqa[slot], c1.z, c0.y);
        r[1] = make_int4(c0.x, c0.w, c1.x, c1.y);
    }
    if (threadIdx.x == 0) nrec[t] = n;
    if (t == 0)
        for (int u = threadIdx.x; u < T; u += blockDim.x) {
            dem[u] = 0;
            const long long a = anchor_next[u];
            if (a != LLONG_MIN) {
                anchor[u] = a;
                anchor_next[u] = LLONG_MIN;
            }
        }
}

// ================================================================ host side
namespace adlbq {

int ensure_req_capacity(adlbq_server *h, int n) {
    if (n <= h->cap_req) return ADLBQ_OK;
    int nc = std::max(n, std::max(1024, h->cap_req * 2));
    AQ_HIP(hipStreamSynchronize(h->stream));
    void *ps[] = {h->d_mask, h->d_tmatch, h->d_umatch, h->d_mslot, h->d_rh, h->d_reqbuf, h->d_respbuf,
                  h->d_seg_cnt, h->d_chS, h->d_chD, h->d_chLP, h->d_chGT, h->d_chGO, h->d_chclean, h->d_cht,
                  h->d_chcnt, h->d_chE, h->d_chflag, h->d_pmask, h->d_lv, h->d_rtype, h->d_jpref};
    for (void *p : ps)
        if (p) AQ_HIP(hipFree(p));
    AQ_HIP(hipMalloc((void **)&h->d_mask, sizeof(unsigned long long) * nc));
    AQ_HIP(hipMalloc((void **)&h->d_jpref, sizeof(int) * ((nc + 63) / 64 + 1)));
    AQ_HIP(hipMalloc((void **)&h->d_tmatch, sizeof(int) * nc));
    AQ_HIP(hipMalloc((void **)&h->d_umatch, sizeof(int) * nc));
    AQ_HIP(hipMalloc((void **)&h->d_mslot, sizeof(int2) * nc));
    AQ_HIP(hipMalloc((void **)&h->d_rh, sizeof(int2) * nc));
    AQ_HIP(hipMemsetAsync(h->d_mslot, 0xff, sizeof(int2) * nc, h->stream));
    AQ_HIP(hipMalloc((void **)&h->d_reqbuf, sizeof(int) * ADLBQ_RESERVE_INTS * (size_t)nc));
    AQ_HIP(hipMalloc((void **)&h->d_respbuf, sizeof(int) * ADLBQ_RESP_INTS * (size_t)nc));
    const size_t nseg = (size_t)(nc + SEG - 1) / SEG, T1 = (size_t)std::max(h->T, 1);
    AQ_HIP(hipMalloc((void **)&h->d_seg_cnt, sizeof(int) * ((nc + 63) / 64)));
    AQ_HIP(hipMalloc((void **)&h->d_pmask, sizeof(unsigned long long) * ((nc + 63) / 64)));
    AQ_HIP(hipMemsetAsync(h->d_pmask, 0, sizeof(unsigned long long) * ((nc + 63) / 64), h->stream));  // see k_finalize
    AQ_HIP(hipMalloc((void **)&h->d_chS, sizeof(int) * 2 * nseg * T1));  // two buffers: launch parity
    AQ_HIP(hipMalloc((void **)&h->d_chD, sizeof(int) * 2 * nseg * T1));
    AQ_HIP(hipMalloc((void **)&h->d_chLP, sizeof(int) * nseg * T1));
    AQ_HIP(hipMalloc((void **)&h->d_chE, sizeof(int) * CHAIN_MAX_PASSES * nseg * T1));
    // [CHAIN_MAX_PASSES][nseg] hand-off flags
    AQ_HIP(hipMalloc((void **)&h->d_chflag, sizeof(int) * (CHAIN_MAX_PASSES + 1) * nseg));
    AQ_HIP(hipMemsetAsync(h->d_chflag, 0, sizeof(int) * (CHAIN_MAX_PASSES + 1) * nseg, h->stream));  // epochs start at 1
    AQ_HIP(hipMalloc((void **)&h->d_chGT, sizeof(int) * CH_GROUPS * T1));
    AQ_HIP(hipMalloc((void **)&h->d_chGO, sizeof(int) * CH_GROUPS * T1));
    AQ_HIP(hipMalloc((void **)&h->d_chclean, sizeof(int) * 2));  // [1]: the fused finalize's epoch flag
    AQ_HIP(hipMemsetAsync(h->d_chclean, 0, sizeof(int) * 2, h->stream));
    AQ_HIP(hipMalloc((void **)&h->d_cht, (size_t)nc));
    AQ_HIP(hipMalloc((void **)&h->d_chcnt, sizeof(unsigned long long) * (CH_GROUPS + 2)));  // + k_rank_chain0's
    // the last arriver of every chain launch re-zeroes them
    AQ_HIP(hipMemsetAsync(h->d_chcnt, 0, sizeof(unsigned long long) * (CH_GROUPS + 2), h->stream));
    h->rank_arrivals = 0;  // k_rank_chain0's counter starts again
    AQ_HIP(hipMalloc((void **)&h->d_lv, sizeof(int) * 8 * (size_t)nc));
    AQ_HIP(hipMalloc((void **)&h->d_rtype, (size_t)nc + 64));
    h->cap_req = nc;
    return ADLBQ_OK;
}

// diagnostic ("kernel_stamps"): the stamp rows of pass 1 (which 0) or pass 2 (1) of the next batch, or nullptr
static unsigned long long *kst_for(adlbq_server *h, int n, int which) {
    if (!h->kstamps || n <= 0) return nullptr;
    if (n > h->cap_kst) {
        (void)hipStreamSynchronize(h->stream);
        if (h->d_kst) (void)hipFree(h->d_kst);
        h->cap_kst = n;
        if (hipMalloc((void **)&h->d_kst, sizeof(unsigned long long) * 8 * n) != hipSuccess) {
            h->d_kst = nullptr;
            h->cap_kst = 0;
            return nullptr;
        }
    }
    h->n_kst = n;
    return h->d_kst + (size_t)which * 4 * n;
}

static int ensure_scan_capacity(adlbq_server *h, int npages) {
    const long long C = (long long)std::max(h->T, 1) * NB;
    const long long need_gh = (long long)npages * C, nchunks = (npages + CHUNK - 1) / CHUNK;
    const long long need_cs = (std::max(1ll, nchunks) + th_tiles((int)std::max(1ll, nchunks))) * C,
                    need_cand = (long long)npages * PAGE;
    if (need_gh > h->cap_gh || need_cs > h->cap_csum || need_cand > h->cap_cand || (long long)npages * 4 > h->cap_spec)
        AQ_HIP(hipStreamSynchronize(h->stream));
    if (need_gh > h->cap_gh) {
        if (h->d_gh) AQ_HIP(hipFree(h->d_gh));
        h->cap_gh = std::max(need_gh, 2 * h->cap_gh);
        AQ_HIP(hipMalloc((void **)&h->d_gh, sizeof(unsigned short) * h->cap_gh));

    }
    if (need_cs > h->cap_csum) {
        if (h->d_csum) AQ_HIP(hipFree(h->d_csum));
        h->cap_csum = std::max(need_cs, 2 * h->cap_csum);
        // two buffers used by the scans in turn: a scan's pass 1 zeroes the one the previous scan used
        AQ_HIP(hipMalloc((void **)&h->d_csum, sizeof(unsigned int) * 2 * h->cap_csum));
        AQ_HIP(hipMemsetAsync(h->d_csum, 0, sizeof(unsigned int) * 2 * h->cap_csum, h->stream));
        h->csum_used[0] = h->csum_used[1] = 0;
    }
    if ((long long)npages * 4 > h->cap_spec) {
        if (h->d_spec) AQ_HIP(hipFree(h->d_spec));
        if (h->d_specn) AQ_HIP(hipFree(h->d_specn));
        h->cap_spec = std::max((long long)npages * 4, 2 * h->cap_spec);
        AQ_HIP(hipMalloc((void **)&h->d_spec, sizeof(unsigned int) * SPEC_CAP * h->cap_spec));
        AQ_HIP(hipMalloc((void **)&h->d_specn, sizeof(int) * h->cap_spec));
    }
    if (need_cand > h->cap_cand) {
        void *ps[] = {h->d_ckey, h->d_ckey2, h->d_cslot, h->d_cslot2, h->d_crank};
        for (void *p : ps)
            if (p) AQ_HIP(hipFree(p));
        h->cap_cand = std::max(need_cand, 2 * h->cap_cand);
        AQ_HIP(hipMalloc((void **)&h->d_ckey, sizeof(unsigned long long) * h->cap_cand));
        AQ_HIP(hipMalloc((void **)&h->d_ckey2, sizeof(unsigned long long) * h->cap_cand));
        AQ_HIP(hipMalloc((void **)&h->d_cslot, sizeof(int) * h->cap_cand));
        AQ_HIP(hipMalloc((void **)&h->d_cslot2, sizeof(int) * h->cap_cand));
        AQ_HIP(hipMalloc((void **)&h->d_crank, sizeof(unsigned int) * h->cap_cand));
    }
    return ADLBQ_OK;
}

// Both passes over the open bucket for the current demand (d_dem): per-type
// candidate lists in preference order at d_candoff / d_candlen / d_cslot.
// A reserve batch's request preparation (pa, nprep workgroups) rides in the
// first launch.
static int launch_scan(adlbq_server *h, const PrepArgs &pa, int nprep, bool sort, int R) {
    const int T = h->T, C = T * NB;
    const int np = (int)h->open.pages.size();
    hipStream_t s = h->stream;
    hipEvent_t ev;
    const bool scan = np > 0 && T > 0;
    auto lt0 = std::chrono::steady_clock::now();
    auto lsec = [&](const char *name) {  // host time per launch of the scan ("hacc:ls_*")
        const auto now = std::chrono::steady_clock::now();
        h->hacc[name] += std::chrono::duration_cast<std::chrono::nanoseconds>(now - lt0).count();
        lt0 = now;
    };
    // the open bucket's pages in one run of ids (one bulk Put): pass 1 computes the page id
    int pg0 = np > 0 ? h->open.pages[0] : -1;
    for (int i = 1; i < np && pg0 >= 0; i++)
        if (h->open.pages[(size_t)i] != pg0 + i) pg0 = -1;
    const int par = h->csum_par;
    unsigned int *csum = h->d_csum + (long long)par * h->cap_csum, *zcs = h->d_csum + (long long)(par ^ 1) * h->cap_csum;
    HistArgs ha{h->d_open_pages, np, h->open.tail_fill, h->d_prio, h->d_meta, T, h->d_anchor, h->d_gh, csum,
                h->d_gcut, h->d_spec, h->d_specn, h->d_pbase, h->d_pwide, zcs, h->csum_used[par ^ 1], pg0};
    ha.kst = kst_for(h, np, 0);
    ha.all_narrow = h->open_all_narrow ? 1 : 0;
    if (scan) {  // this scan's buffer; the other one is clean once pass 1 has run
        const int nch = (np + CHUNK - 1) / CHUNK;
        h->csum_used[par] = (long long)(nch + th_tiles(nch)) * C;  // the chunk sums and the tile area
        h->csum_used[par ^ 1] = 0;
        h->csum_par = par ^ 1;
    }
    const int pp = hist_pp(T <= 8 ? 8 : 64), npb = (np + pp - 1) / pp;  // pages per pass-1 workgroup
    const int grid = nprep + (scan ? npb : 0);
    if (grid > 0) {
        // pass 1: the histogram copies, then the four waves' speculative lists
        const int lds = (int)std::max(nprep > 0 ? (size_t)PREP_LDS : 0,
                                      scan ? sizeof(unsigned int) * pp * hist_page_words(C, T <= 8) : 0);
        stage_begin(h, "hist", &ev);
        auto kph = T <= 4 ? k_prep_hist<4> : T <= 8 ? k_prep_hist<8> : k_prep_hist<64>;
        if (h->split_prep && nprep > 0 && scan) {  // diagnostic: the two roles as two launches
            kph<<<nprep, 256, lds, s>>>(pa, nprep, ha);
            kph<<<npb, 256, lds, s>>>(pa, 0, ha);
        } else if (h->grec) {  // adlbq_reserve_group_device: recorded, launched with the group's
            h->grec->kinds |= GK_PREP;
            h->grec->tb = T <= 4 ? 4 : 8;
            h->grec->prep = GPrep{pa, nprep, ha, grid};
            h->grec->lds_prep = (size_t)lds;
        } else {
            lsec("ls_pre");
            kph<<<grid, 256, lds, s>>>(pa, nprep, ha);
        }
        stage_end(h, "hist", ev);
        lsec("ls_hist");
    }
    if (scan) {
        const int nchunks = (np + CHUNK - 1) / CHUNK;
        if (h->grec) {
            h->grec->kinds |= GK_THR;
            h->grec->thr = GThr{zcs, ha.zn, T, h->d_dem, csum, nchunks, h->d_theta, h->d_need, h->d_candlen,
                                h->d_needsort, h->d_binoff, h->d_coltot, h->d_type_cnt, h->d_anchor, h->d_anchor_next,
                                h->d_gcut_next, nprep > 0 ? 1 : 0, th_tiles(nchunks) * T, h->d_gcut};
        } else {
            stage_begin(h, "thresholds", &ev);
            // plus one workgroup: the prefix of seg_cnt for the chain (prep_block wrote it in this batch)
            const bool jp = nprep > 0 && T <= 8;
            k_thresholds<<<th_tiles(nchunks) * T + (jp ? 1 : 0), TH_THREADS, 0, s>>>(
                zcs, ha.zn, T, h->d_dem, csum, nchunks, h->d_theta, h->d_need, h->d_candlen, h->d_needsort,
                h->d_binoff, h->d_coltot, h->d_type_cnt, h->d_anchor, h->d_anchor_next, h->d_gcut_next,
                nprep > 0 ? 1 : 0, h->d_gcut, h->d_seg_cnt, (R + 63) / 64, jp ? h->d_jpref : nullptr);
            h->jpref_ok = jp;
            stage_end(h, "thresholds", ev);
            lsec("ls_thr");
        }
        stage_begin(h, "select", &ev);
        auto sel = T <= 4 ? k_select_open<4> : T <= 8 ? k_select_open<8> : k_select_open<64>;
        if (h->grec) {
            h->grec->kinds |= GK_SEL;
            h->grec->sel = GSel{h->d_open_pages, np, h->open.tail_fill, h->d_prio, h->d_meta, h->d_seq, T, h->d_anchor,
                                h->d_theta, h->d_need, h->d_binoff, csum, h->d_gh, h->d_candlen, h->d_candoff,
                                h->d_ckey, h->d_cslot, h->d_gcut, h->d_spec, h->d_specn, h->d_pbase, h->d_pwide,
                                h->d_ctr, (sort || !h->rank_in_select) ? nullptr : h->d_crank,
                                (!sort && T <= 8) ? h->d_lv : nullptr, h->d_rtype, R, np};
            h->grec->selw = T <= 8 && h->select_wave;
            h->grec->lds_sel_open = sizeof(unsigned int) * (4 * C + 4 * 1024);
            h->grec->lds_sel = h->grec->selw ? sizeof(unsigned int) * (C + 1024) : sizeof(unsigned int) * (4 * C + 4 * 1024);
        } else if (T <= 8 && h->select_wave) {
            auto selw = T <= 4 ? k_select_wave<4> : k_select_wave<8>;
            selw<<<np, 64, sizeof(unsigned int) * (C + 1024), s>>>(
                h->d_open_pages, np, h->open.tail_fill, h->d_prio, h->d_meta, T, h->d_anchor, h->d_theta, h->d_need,
                h->d_binoff, csum, h->d_gh, h->d_candlen, h->d_candoff, h->d_ckey, h->d_cslot, h->d_gcut, h->d_spec,
                h->d_specn, h->d_pbase, h->d_pwide, h->d_ctr, (sort || !h->rank_in_select) ? nullptr : h->d_crank,
                !sort ? h->d_lv : nullptr, h->d_rtype, R, kst_for(h, np, 1));
        } else
        sel<<<np, 256, sizeof(unsigned int) * (4 * C + 4 * 1024), s>>>(
            h->d_open_pages, np, h->open.tail_fill, h->d_prio, h->d_meta, h->d_seq, T, h->d_anchor, h->d_theta,
            h->d_need, h->d_binoff, csum, h->d_gh, h->d_candlen, h->d_candoff, h->d_ckey, h->d_cslot,
            h->d_gcut, h->d_spec, h->d_specn, h->d_pbase, h->d_pwide, h->d_ctr,
            (sort || !h->rank_in_select) ? nullptr : h->d_crank, (!sort && T <= 8) ? h->d_lv : nullptr, h->d_rtype, R,
            kst_for(h, np, 1));
        stage_end(h, "select", ev);
        lsec("ls_sel");
        if (sort) {  // a reserve batch sorts inside k_rank
            stage_begin(h, "sort", &ev);
            k_sort_types<<<T, 1024, 0, s>>>(h->d_needsort, h->d_candoff, h->d_candlen, h->d_ckey, h->d_cslot,
                                            h->d_ckey2, h->d_cslot2);
            stage_end(h, "sort", ev);
        }
    } else {
        AQ_HIP(hipMemsetAsync(h->d_candlen, 0, sizeof(int) * std::max(T, 1), s));
        AQ_HIP(hipMemsetAsync(h->d_candoff, 0, sizeof(int) * (std::max(T, 1) + 1), s));
    }
    return ADLBQ_OK;
}

// The targeted units' sorted index (k_targeted_idx), rebuilt after targeted
// Puts: keys/vals over every slot of every rank-bucket page (holes sort last),
// one stable radix sort, then the (bucket, type) ranges.
static int tindex_ranges(adlbq_server *h, int nb) {
    hipStream_t s = h->stream;
    const int G = nb * 64;
    if (G > 0)
        k_tindex_bounds<<<(G + 255) / 256, 256, 0, s>>>(h->d_tkeys, (int)h->tidx_n, G, h->d_tstart, h->d_tend);
    AQ_HIP(hipGetLastError());
    h->tidx_groups = G;
    return ADLBQ_OK;
}

// Stable merge of two sorted key runs with their values: entry i of a lands at
// i + |{b < key}|, entry j of b at j + |{a <= key}|.
__global__ __launch_bounds__(256) void k_merge_sorted(const unsigned long long *__restrict__ ak,
                                                      const int *__restrict__ av, long long na,
                                                      const unsigned long long *__restrict__ bk,
                                                      const int *__restrict__ bv, long long nb,
                                                      unsigned long long *__restrict__ ok, int *__restrict__ ov) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= na + nb) return;
    const bool from_a = i < na;
    const unsigned long long key = from_a ? ak[i] : bk[i - na];
    const int val = from_a ? av[i] : bv[i - na];
    const unsigned long long *o = from_a ? bk : ak;
    long long lo = 0, hi = from_a ? nb : na;
    while (lo < hi) {  // a: first b >= key; b: first a > key
        const long long mid = (lo + hi) >> 1;
        const unsigned long long x = o[mid];
        if (from_a ? x < key : x <= key) lo = mid + 1;
        else hi = mid;
    }
    const long long pos = (from_a ? i : i - na) + lo;
    ok[pos] = key;
    ov[pos] = val;
}

__global__ __launch_bounds__(256) void k_copy_kv(const unsigned long long *__restrict__ sk,
                                                 const int *__restrict__ sv, long long m,
                                                 unsigned long long *__restrict__ dk, int *__restrict__ dv) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) {
        dk[i] = sk[i];
        dv[i] = sv[i];
    }
}

static int ensure_tindex(adlbq_server *h) {
    if (!h->tindex_dirty) return ADLBQ_OK;
    hipStream_t s = h->stream;
    const int nb = (int)h->bucket_ranks.size();
    int npg = 0;
    for (int k = 0; k < nb; k++) npg += (int)h->rankb[k].pages.size();
    const long long n = (long long)npg * PAGE;
    if (n > h->cap_tidx) {
        AQ_HIP(hipStreamSynchronize(s));
        void *ps[] = {h->d_tkeys, h->d_tkeys2, h->d_tvals, h->d_tvals2};
        for (void *p : ps)
            if (p) AQ_HIP(hipFree(p));
        h->cap_tidx = std::max(n, 2 * h->cap_tidx);
        AQ_HIP(hipMalloc((void **)&h->d_tkeys, sizeof(unsigned long long) * h->cap_tidx));
        AQ_HIP(hipMalloc((void **)&h->d_tkeys2, sizeof(unsigned long long) * h->cap_tidx));
        AQ_HIP(hipMalloc((void **)&h->d_tvals, sizeof(int) * h->cap_tidx));
        AQ_HIP(hipMalloc((void **)&h->d_tvals2, sizeof(int) * h->cap_tidx));
        h->tidx_valid = false;  // the sorted entries were in the freed arrays
    }
    if ((long long)nb * 64 > h->cap_trange) {
        AQ_HIP(hipStreamSynchronize(s));
        if (h->d_tstart) AQ_HIP(hipFree(h->d_tstart));
        if (h->d_tend) AQ_HIP(hipFree(h->d_tend));
        h->cap_trange = std::max((long long)nb * 64, 2 * h->cap_trange);
        AQ_HIP(hipMalloc((void **)&h->d_tstart, sizeof(int) * h->cap_trange));
        AQ_HIP(hipMalloc((void **)&h->d_tend, sizeof(int) * h->cap_trange));
        h->tidx_groups = 0;  // the bounds were in the freed arrays
    }
    const long long m = (long long)h->tnew_keys.size();
    // incremental: the new units' keys (sorted on the host, ties kept in Put order) merged into the
    // delta index, or into the sorted main index -- old entries first on equal keys, as their
    // bucket positions are lower
    if (h->tidx_valid && m > 0 && h->tidx_n + h->tdel_n + m <= h->cap_tidx && m * 4 <= h->tidx_n + 4096) {
        if (m > h->cap_tnew) {
            AQ_HIP(hipStreamSynchronize(s));
            if (h->d_tnewk) AQ_HIP(hipFree(h->d_tnewk));
            if (h->d_tnewv) AQ_HIP(hipFree(h->d_tnewv));
            h->cap_tnew = std::max(m, 2 * h->cap_tnew);
            AQ_HIP(hipMalloc((void **)&h->d_tnewk, sizeof(unsigned long long) * h->cap_tnew));
            AQ_HIP(hipMalloc((void **)&h->d_tnewv, sizeof(int) * h->cap_tnew));
        }
        auto tq0 = std::chrono::steady_clock::now();
        auto tsec = [&](const char *name) {
            const auto now = std::chrono::steady_clock::now();
            h->hacc[name] += std::chrono::duration_cast<std::chrono::nanoseconds>(now - tq0).count();
            tq0 = now;
        };
        h->hacc["ti_keys"] += m;
        const auto &K = h->tnew_keys;
        // stable LSD radix sort of the new keys' indices, 8-bit digits, only the digits the
        // keys differ in (a comparison sort of ~1,600 keys cost ~48 us of the config-4 step)
        std::vector<int> ord((size_t)m), ord2((size_t)m);
        for (long long i = 0; i < m; i++) ord[(size_t)i] = (int)i;
        {
            unsigned long long vor = 0, vand = ~0ull;
            for (long long i = 0; i < m; i++) {
                vor |= K[(size_t)i];
                vand &= K[(size_t)i];
            }
            const unsigned long long vary = vor ^ vand;
            for (int sh = 0; sh < 64; sh += 8) {
                if (((vary >> sh) & 0xffull) == 0) continue;
                int cnt[257] = {0};
                for (long long i = 0; i < m; i++) cnt[((K[(size_t)ord[(size_t)i]] >> sh) & 0xff) + 1]++;
                for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
                for (long long i = 0; i < m; i++) {
                    const int x = ord[(size_t)i];
                    ord2[(size_t)cnt[(K[(size_t)x] >> sh) & 0xff]++] = x;
                }
                ord.swap(ord2);
            }
        }
        tsec("ti_sort");
        // pinned host staging, two buffers used in turn: a buffer is rewritten only once the
        // copy of two merges ago has run (its event), so the host never waits for the last one
        const int sl = h->tnew_slot;
        h->tnew_slot ^= 1;
        const auto w0 = std::chrono::steady_clock::now();
        if (h->tnew_ev[sl]) AQ_HIP(hipEventSynchronize(h->tnew_ev[sl]));
        else AQ_HIP(hipEventCreateWithFlags(&h->tnew_ev[sl], hipEventDisableTiming));
        h->hacc["tindex_wait"] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
        tsec("ti_wait");
        if (m > h->cap_htnew[sl]) {
            if (h->h_tnewk[sl]) AQ_HIP(hipHostFree(h->h_tnewk[sl]));
            if (h->h_tnewv[sl]) AQ_HIP(hipHostFree(h->h_tnewv[sl]));
            // generous from the start: a pinned reallocation costs milliseconds and synchronises
            h->cap_htnew[sl] = std::max<long long>({m, 2 * h->cap_htnew[sl], 1ll << 16});
            AQ_HIP(hipHostMalloc((void **)&h->h_tnewk[sl], sizeof(unsigned long long) * h->cap_htnew[sl], hipHostMallocDefault));
            AQ_HIP(hipHostMalloc((void **)&h->h_tnewv[sl], sizeof(int) * h->cap_htnew[sl], hipHostMallocDefault));
        }
        tsec("ti_alloc");
        for (long long i = 0; i < m; i++) {
            h->h_tnewk[sl][i] = K[(size_t)ord[(size_t)i]];
            h->h_tnewv[sl][i] = h->tnew_vals[(size_t)ord[(size_t)i]];
        }
        tsec("ti_fill");
        // read straight from the pinned buffers by a kernel: a small hipMemcpyAsync from host
        // memory waited for the stream's earlier work (~0.45 ms per config-4 Put batch)
        unsigned long long *dk = nullptr;
        int *dv = nullptr;
        AQ_HIP(hipHostGetDevicePointer((void **)&dk, h->h_tnewk[sl], 0));
        AQ_HIP(hipHostGetDevicePointer((void **)&dv, h->h_tnewv[sl], 0));
        tsec("ti_devptr");
        k_copy_kv<<<(unsigned int)((m + 255) / 256), 256, 0, s>>>(dk, dv, m, h->d_tnewk, h->d_tnewv);
        AQ_HIP(hipGetLastError());
        tsec("ti_launch");
        AQ_HIP(hipEventRecord(h->tnew_ev[sl], s));
        h->tnew_keys.clear();
        h->tnew_vals.clear();
        tsec("ti_stage");
        const int G = nb * 64;
        int rc;
        // sorted runs a, b merged into (ok, ov), stable (a's entries first on equal keys):
        // every entry finds its output position by one binary search in the other run
        auto merge_into = [&](const unsigned long long *ak, const int *av, long long na, const unsigned long long *bk,
                              const int *bv, long long nbk, unsigned long long *ok, int *ov) -> int {
            const long long tot = na + nbk;
            if (tot > 0)
                k_merge_sorted<<<(unsigned int)((tot + 255) / 256), 256, 0, s>>>(ak, av, na, bk, bv, nbk, ok, ov);
            AQ_HIP(hipGetLastError());
            return ADLBQ_OK;
        };
        // the main index's bounds after m2 sorted keys (nk) joined it (m2 = 0: new groups only)
        auto shift_main = [&](const unsigned long long *nk, long long m2, long long n_old) -> int {
            if (h->tidx_groups > 0 && h->tidx_groups <= (long long)G) {
                k_tindex_shift<<<(G + 255) / 256, 256, 0, s>>>(nk, (int)m2, (int)h->tidx_groups, (int)n_old, G,
                                                              h->d_tstart, h->d_tend);
                AQ_HIP(hipGetLastError());
                h->tidx_groups = G;
                return ADLBQ_OK;
            }
            return tindex_ranges(h, nb);
        };
        if (h->tdel_max > 0 && h->tdel_n + m <= h->tdel_max && (h->tdel_n == 0 || h->tdel_max <= h->cap_del)) {
            // into the delta index (the main index stays where it is: no 8M-entry move per Put batch)
            if (h->tdel_max > h->cap_del || (long long)G > h->cap_drange) {
                AQ_HIP(hipStreamSynchronize(s));
                if (h->tdel_max > h->cap_del) {
                    void *ps[] = {h->d_dkeys, h->d_dkeys2, h->d_dvals, h->d_dvals2};
                    for (void *p : ps)
                        if (p) AQ_HIP(hipFree(p));
                    h->cap_del = h->tdel_max;
                    AQ_HIP(hipMalloc((void **)&h->d_dkeys, sizeof(unsigned long long) * h->cap_del));
                    AQ_HIP(hipMalloc((void **)&h->d_dkeys2, sizeof(unsigned long long) * h->cap_del));
                    AQ_HIP(hipMalloc((void **)&h->d_dvals, sizeof(int) * h->cap_del));
                    AQ_HIP(hipMalloc((void **)&h->d_dvals2, sizeof(int) * h->cap_del));
                }
                if ((long long)G > h->cap_drange) {
                    if (h->d_dstart) AQ_HIP(hipFree(h->d_dstart));
                    if (h->d_dend) AQ_HIP(hipFree(h->d_dend));
                    h->cap_drange = std::max((long long)G, 2 * h->cap_drange);
                    AQ_HIP(hipMalloc((void **)&h->d_dstart, sizeof(int) * h->cap_drange));
                    AQ_HIP(hipMalloc((void **)&h->d_dend, sizeof(int) * h->cap_drange));
                }
            }
            if (h->tdel_n == 0) {
                AQ_HIP(hipMemcpyAsync(h->d_dkeys, h->d_tnewk, sizeof(unsigned long long) * m, hipMemcpyDeviceToDevice, s));
                AQ_HIP(hipMemcpyAsync(h->d_dvals, h->d_tnewv, sizeof(int) * m, hipMemcpyDeviceToDevice, s));
            } else {
                if ((rc = merge_into(h->d_dkeys, h->d_dvals, h->tdel_n, h->d_tnewk, h->d_tnewv, m, h->d_dkeys2,
                                     h->d_dvals2)))
                    return rc;
                std::swap(h->d_dkeys, h->d_dkeys2);
                std::swap(h->d_dvals, h->d_dvals2);
            }
            h->tdel_n += m;
            if (h->tidx_groups != (long long)G && (rc = shift_main(h->d_tnewk, 0, h->tidx_n))) return rc;  // new buckets
            k_tindex_bounds<<<(G + 255) / 256, 256, 0, s>>>(h->d_dkeys, (int)h->tdel_n, G, h->d_dstart, h->d_dend);
            AQ_HIP(hipGetLastError());
            tsec("ti_delta");
            h->tidx_delta_merges++;
            h->tindex_dirty = false;
            return ADLBQ_OK;
        }
        if (h->tdel_n > 0) {  // fold the delta into the main index first
            if ((rc = merge_into(h->d_tkeys, h->d_tvals, h->tidx_n, h->d_dkeys, h->d_dvals, h->tdel_n, h->d_tkeys2,
                                 h->d_tvals2)))
                return rc;
            std::swap(h->d_tkeys, h->d_tkeys2);
            std::swap(h->d_tvals, h->d_tvals2);
            const long long n_old = h->tidx_n;
            h->tidx_n += h->tdel_n;
            if ((rc = shift_main(h->d_dkeys, h->tdel_n, n_old))) return rc;
            h->tdel_n = 0;
            h->tidx_folds++;
        }
        if ((rc = merge_into(h->d_tkeys, h->d_tvals, h->tidx_n, h->d_tnewk, h->d_tnewv, m, h->d_tkeys2, h->d_tvals2)))
            return rc;
        std::swap(h->d_tkeys, h->d_tkeys2);
        std::swap(h->d_tvals, h->d_tvals2);
        const long long n_old = h->tidx_n;
        h->tidx_n += m;
        h->tidx_merges++;
        if ((rc = shift_main(h->d_tnewk, m, n_old))) return rc;
        h->tindex_dirty = false;
        return ADLBQ_OK;
    }
    // full build: keys over every slot of every rank-bucket page (holes sort last), one stable sort
    const size_t tmp = rsx_temp_bytes(n);
    if (tmp > h->cap_tsort) {
        AQ_HIP(hipStreamSynchronize(s));
        if (h->d_tsort) AQ_HIP(hipFree(h->d_tsort));
        h->cap_tsort = std::max(tmp, 2 * h->cap_tsort);
        AQ_HIP(hipMalloc(&h->d_tsort, h->cap_tsort));
    }
    long long filled = 0;
    for (int k = 0; k < nb; k++)
        if (!h->rankb[k].pages.empty()) filled += (long long)(h->rankb[k].pages.size() - 1) * PAGE + h->rankb[k].tail_fill;
    if (npg > 0) {
        k_tindex_keys<<<npg, 256, 0, s>>>(h->d_rank_pstart, h->d_rank_pages, h->d_rank_fill, nb, h->d_prio, h->d_meta,
                                          h->d_tkeys, h->d_tvals);
        const int rs = rsx_sort_pairs(h->d_tsort, h->cap_tsort, h->d_tkeys, h->d_tkeys2, h->d_tvals, h->d_tvals2, n, 0,
                                      TIDX_KEY_BITS, false, s);
        if (rs) return rs;
        std::swap(h->d_tkeys, h->d_tkeys2);  // keep the sorted arrays in d_tkeys / d_tvals
        std::swap(h->d_tvals, h->d_tvals2);
    }
    h->tidx_n = filled;  // the holes sorted past the filled slots
    h->tdel_n = 0;       // every targeted unit is in the main index again
    h->tidx_valid = true;
    h->tidx_rebuilds++;
    h->tnew_keys.clear();
    h->tnew_vals.clear();
    int rc;
    if ((rc = tindex_ranges(h, nb))) return rc;
    h->tindex_dirty = false;
    return ADLBQ_OK;
}

// The ranges sorted by launch_segsort, passed by value.
struct SegList {
    int n;
    int type[ADLBQ_MAX_TYPES], beg[ADLBQ_MAX_TYPES], end[ADLBQ_MAX_TYPES];
};

// the sorted ranges back into the candidate lists; needsort 2 = sorted
__global__ __launch_bounds__(256) void k_segsort_back(SegList sl, const unsigned long long *__restrict__ k2,
                                                      const int *__restrict__ s2, unsigned long long *key, int *slot,
                                                      int *needsort) {
    const int q = blockIdx.y;
    if (q >= sl.n) return;
    const int b = sl.beg[q], e = sl.end[q];
    for (int i = b + blockIdx.x * blockDim.x + threadIdx.x; i < e; i += gridDim.x * blockDim.x) {
        key[i] = k2[i];
        slot[i] = s2[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) needsort[sl.type[q]] = 2;
}

// short list from + blockIdx.x sorted by one workgroup (sort_type: LDS bitonic
// blocks, then merges through key2 / slot2), then copied to key2 / slot2, where
// k_segsort_back takes every sorted list from
__global__ __launch_bounds__(1024) void k_segsort_short(SegList sl, int from, unsigned long long *key, int *slot,
                                                        unsigned long long *key2, int *slot2) {
    __shared__ unsigned long long sk[SORT_BLK];
    __shared__ int ss[SORT_BLK];
    const int q = from + blockIdx.x, b = sl.beg[q], n = sl.end[q] - b;
    sort_type(b, n, key, slot, key2, slot2, sk, ss);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        key2[b + i] = key[b + i];
        slot2[b + i] = slot[b + i];
    }
}

// Per-type OR / AND of the candidate keys (kb[t] = OR, kb[64 + t] = AND): the
// bits a list's keys differ in (the sync-free radix sort's plan, k_sort_plan).
__global__ __launch_bounds__(256) void k_keybits(const int *__restrict__ candoff, const int *__restrict__ candlen,
                                                 const unsigned long long *__restrict__ key,
                                                 unsigned long long *kb) {
    const int t = blockIdx.y, b = candoff[t], e = b + candlen[t];
    unsigned long long o = 0, a = ~0ull;
    for (int i = b + blockIdx.x * blockDim.x + threadIdx.x; i < e; i += gridDim.x * blockDim.x) {
        const unsigned long long k = key[i];
        o |= k;
        a &= k;
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        o |= __shfl_xor(o, d, 64);
        a &= __shfl_xor(a, d, 64);
    }
    if ((threadIdx.x & 63) == 0 && a != ~0ull) {
        atomicOr(&kb[t], o);
        atomicAnd(&kb[ADLBQ_MAX_TYPES + t], a);
    }
}

constexpr int LIST_SHIFT = 58;  // a list whose keys vary at or above this bit cannot be planned

// A read-back sort's figures for the next batch's sync-free radix sort
// (launch_segsort_radix): candidates in all, lowest key bit any list varies
// in, highest prio-field bit.
__global__ void k_sort_plan(int T, const int *__restrict__ candoff, const int *__restrict__ candlen,
                            const int *__restrict__ needsort, const unsigned long long *__restrict__ kb, int g_bound,
                            int lo_hint, int *plan, DevCounters *ctr) {
    const int t = threadIdx.x;
    const bool has = t < T && candlen[t] > 0;
    const unsigned long long diff = has ? (kb[t] ^ kb[ADLBQ_MAX_TYPES + t]) : 0ull;
    const bool bad_top = (diff >> LIST_SHIFT) != 0ull;
    int lo = diff ? __ffsll((long long)diff) - 1 : 64;
    const bool wants = t < T && needsort[t] == 1 && candlen[t] > 1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) lo = min(lo, __shfl_xor(lo, o, 64));
    const bool ok = __ballot(bad_top) == 0ull, nsort = __ballot(wants) != 0ull;
    unsigned int up = (unsigned int)(diff >> 32);  // prio-field bits this list varies in
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) up |= __shfl_xor(up, o, 64);
    if (t == 0) {
        const int G = candoff[T];
        ctr->plan_phi = up ? 31 - __clz(up) : -1;
        lo = min(lo, LIST_SHIFT);
        plan[0] = (ok && nsort && G <= g_bound && lo >= lo_hint) ? 1 : 0;
        plan[1] = G;
        if (g_bound > 0 && nsort && !plan[0]) ctr->plan_missed += 1;
        ctr->plan_g = G;
        ctr->plan_lo = ok ? lo : 0;
    }
}

// ---------------------------------------------------------------- list-stable radix sort
// The candidate lists leave k_select_open in (column, bucket position) order,
// and a list's columns cover descending, disjoint prio ranges: entries of equal
// prio are already in key order.  Sorting every list STABLY by prio,
// descending, therefore yields the full key order.  Sort key (32 bits): the
// list index above the low pb bits of ~(key >> 32); the prio-field bits at and
// above pb must be constant inside each list (checked on the device: per-list
// OR / AND of the field).  LSD radix sort, 8-bit digits, RS_TILE entries per
// 1024-thread workgroup, two launches per digit: count (per-tile digit counts)
// and scatter (each tile sums the counts of the tiles before it and of the
// smaller digits itself, then ranks its entries stably, a wave per 256).  The
// payload moves once: k_rs_keys copies the lists aside (ckey3 / cslot3) and
// the last scatter writes them back in order.  If the plan does not hold
// (more candidates than planned, a list varying at or above pb, or nothing to
// sort) every launch after k_rs_keys returns at once and k_rank sorts
// in-launch (needsort stays 1): a stale plan costs time, never results.
constexpr int RS_TILE = 4096, RS_THREADS = 1024, RS_WAVES = RS_THREADS / 64;
constexpr int RS_WAVE_ITEMS = RS_TILE / RS_WAVES, RS_STEPS = RS_WAVE_ITEMS / 64;  // 4 steps of 64 per wave
constexpr int RS_PARTS = RS_THREADS / 256;  // threads per digit in the tile-prefix sums

struct RsArgs {
    int T, pb, g_bound, nblk;
    const int *candoff, *candlen;
    int *needsort;
    unsigned int *acc;       // [64] OR, [64] AND of each list's prio field (this batch)
    unsigned int *acc_next;  // the other parity: reset here for the next batch
    int *cnt;                // [nblk][256] digit counts per tile
    DevCounters *ctr;
};

// does the plan hold for this batch
__device__ __forceinline__ bool rs_plan_ok(const RsArgs &a, int *G_out, unsigned int *U_out, bool *want_out) {
    unsigned int U = 0;
    bool want = false;
    for (int t = 0; t < a.T; t++) {
        if (a.candlen[t] > 0) U |= a.acc[t] ^ a.acc[64 + t];
        want |= a.needsort[t] == 1 && a.candlen[t] > 1;
    }
    const int G = a.candoff[a.T];
    if (G_out) *G_out = G;
    if (U_out) *U_out = U;
    if (want_out) *want_out = want;
    return want && G <= a.g_bound && (a.pb >= 32 || (U >> a.pb) == 0u);
}

__global__ __launch_bounds__(256) void k_rs_keys(RsArgs a, const unsigned long long *__restrict__ ckey,
                                                 const int *__restrict__ cslot, unsigned long long *__restrict__ ckey3,
                                                 int *__restrict__ cslot3, unsigned int *__restrict__ K,
                                                 unsigned int *__restrict__ I) {
    __shared__ int soff[ADLBQ_MAX_TYPES + 1];
    __shared__ unsigned int sor[ADLBQ_MAX_TYPES], sand[ADLBQ_MAX_TYPES];
    const int T = a.T;
    for (int t = threadIdx.x; t <= T; t += blockDim.x) soff[t] = a.candoff[t];
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        sor[t] = 0u;
        sand[t] = ~0u;
        if (blockIdx.x == 0) {  // the next batch accumulates into the other parity
            a.acc_next[t] = 0u;
            a.acc_next[64 + t] = ~0u;
        }
    }
    __syncthreads();
    const int G = min(soff[T], a.g_bound);
    const unsigned int pmask = a.pb >= 32 ? ~0u : ((1u << a.pb) - 1u);
    for (int i0 = blockIdx.x * blockDim.x; i0 < G; i0 += gridDim.x * blockDim.x) {
        const int i = i0 + threadIdx.x;
        int t = 0;
        unsigned int pf = 0;
        if (i < G) {
            int lo = 0, hi = T - 1;  // the last list starting at or before i
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (soff[mid] <= i) lo = mid;
                else hi = mid - 1;
            }
            t = lo;
            const unsigned long long k = ckey[i];
            const int sl = cslot[i];
            ckey3[i] = k;
            cslot3[i] = sl;
            pf = (unsigned int)(k >> 32);
            K[i] = ((unsigned int)t << a.pb) | (~pf & pmask);
            I[i] = (unsigned int)i;
        }
        // per-list OR / AND: one LDS update per wave when the wave lies in one list
        const bool valid = i < G;
        const int t0 = __shfl(t, 0, 64);
        const bool uni = __ballot(valid && t != t0) == 0ull, any = __ballot(valid) != 0ull;
        if (uni) {
            unsigned int o = valid ? pf : 0u, n = valid ? pf : ~0u;
#pragma unroll
            for (int d = 32; d > 0; d >>= 1) {
                o |= __shfl_xor(o, d, 64);
                n &= __shfl_xor(n, d, 64);
            }
            if ((threadIdx.x & 63) == 0 && any) {
                atomicOr(&sor[t0], o);
                atomicAnd(&sand[t0], n);
            }
        } else if (valid) {
            atomicOr(&sor[t], pf);
            atomicAnd(&sand[t], pf);
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += blockDim.x)
        if (sand[t] != ~0u || sor[t] != 0u) {
            atomicOr(&a.acc[t], sor[t]);
            atomicAnd(&a.acc[64 + t], sand[t]);
        }
}

// lanes of this wave with the same 8-bit digit (valid lanes only)
__device__ __forceinline__ unsigned long long rs_peers(unsigned int d, bool valid) {
    unsigned long long m = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
        const unsigned long long bb = __ballot((d >> b) & 1u);
        m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    return m;
}

__global__ __launch_bounds__(RS_THREADS) void k_rs_count(RsArgs a, int pass, const unsigned int *__restrict__ K) {
    __shared__ unsigned int sc[256];
    __shared__ int s_ok, s_G;
    if (threadIdx.x == 0) {
        int G = 0;
        s_ok = rs_plan_ok(a, &G, nullptr, nullptr);
        s_G = G;
    }
    if (threadIdx.x < 256) sc[threadIdx.x] = 0u;
    __syncthreads();
    if (!s_ok) return;
    const int G = s_G, b = blockIdx.x, sh = 8 * pass, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int st = 0; st < RS_STEPS; st++) {
        const int i = b * RS_TILE + w * RS_WAVE_ITEMS + st * 64 + lane;
        const bool valid = i < G;
        const unsigned int d = valid ? (K[i] >> sh) & 255u : 0u;
        const unsigned long long pe = rs_peers(d, valid);
        if (valid && (pe & lt) == 0ull) atomicAdd(&sc[d], (unsigned int)__popcll(pe));
    }
    __syncthreads();
    if (threadIdx.x < 256) a.cnt[(long long)b * 256 + threadIdx.x] = (int)sc[threadIdx.x];
}

__global__ __launch_bounds__(RS_THREADS) void k_rs_scatter(RsArgs a, int pass, int last,
                                                           const unsigned int *__restrict__ K,
                                                           const unsigned int *__restrict__ I,
                                                           unsigned int *__restrict__ Ko, unsigned int *__restrict__ Io,
                                                           const unsigned long long *__restrict__ ckey3,
                                                           const int *__restrict__ cslot3, unsigned long long *ckey,
                                                           int *cslot) {
    __shared__ unsigned int wc[RS_WAVES][256];
    __shared__ unsigned int spre[RS_PARTS][256], stot[RS_PARTS][256];
    __shared__ unsigned int wsum[4];
    __shared__ int s_ok, s_G;
    const int b = blockIdx.x, sh = 8 * pass, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        int G = 0;
        unsigned int U = 0;
        bool want = false;
        const bool ok = rs_plan_ok(a, &G, &U, &want);
        if (last && b == 0) {  // this batch's figures, for the next batch's plan
            if (want && !ok) a.ctr->plan_missed += 1;
            a.ctr->plan_g = G;
            a.ctr->plan_phi = U ? 31 - __clz(U) : -1;
            a.ctr->plan_lo = 0;
        }
        s_ok = ok;
        s_G = G;
    }
    __syncthreads();
    if (!s_ok) return;
    const int G = s_G;
    {  // counts of digit d in the tiles before this one, and in all tiles
        const int d = threadIdx.x & 255, q = threadIdx.x >> 8;
        unsigned int pre = 0, tot = 0;
        for (int bb = q; bb < a.nblk; bb += RS_PARTS) {
            const unsigned int v = (unsigned int)a.cnt[(long long)bb * 256 + d];
            tot += v;
            pre += bb < b ? v : 0u;
        }
        spre[q][d] = pre;
        stot[q][d] = tot;
    }
    for (int q = 0; q < RS_WAVES; q++)
        if (threadIdx.x < 256) wc[q][threadIdx.x] = 0u;
    __syncthreads();
    if (threadIdx.x < 256) {  // exclusive scan of the digit totals: this tile's start per digit
        const int d = threadIdx.x;
        unsigned int tot = 0, pre = 0;
#pragma unroll
        for (int q = 0; q < RS_PARTS; q++) {
            tot += stot[q][d];
            pre += spre[q][d];
        }
        unsigned int x = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[w] = x;
        spre[0][d] = x - tot + pre;  // wave-local exclusive prefix + earlier tiles (waves added below)
    }
    __syncthreads();
    unsigned int key[RS_STEPS], idx[RS_STEPS], pos[RS_STEPS];
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int st = 0; st < RS_STEPS; st++) {
        const int i = b * RS_TILE + w * RS_WAVE_ITEMS + st * 64 + lane;
        const bool valid = i < G;
        key[st] = valid ? K[i] : 0u;
        idx[st] = valid ? I[i] : 0xffffffffu;
    }
#pragma unroll
    for (int st = 0; st < RS_STEPS; st++) {
        const bool valid = idx[st] != 0xffffffffu;
        const unsigned int d = (key[st] >> sh) & 255u;
        const unsigned long long pe = rs_peers(d, valid);
        const unsigned int before = wc[w][d];
        pos[st] = before + (unsigned int)__popcll(pe & lt);
        __builtin_amdgcn_wave_barrier();
        if (valid && (pe & lt) == 0ull) wc[w][d] = before + (unsigned int)__popcll(pe);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    if (threadIdx.x < 256) {  // per digit: the tile's global start plus the counts of the earlier waves
        const int d = threadIdx.x;
        unsigned int run = spre[0][d];
        for (int q = 0; q < (d >> 6); q++) run += wsum[q];
        for (int q = 0; q < RS_WAVES; q++) {
            const unsigned int c = wc[q][d];
            wc[q][d] = run;
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int st = 0; st < RS_STEPS; st++) {
        if (idx[st] == 0xffffffffu) continue;
        const unsigned int d = (key[st] >> sh) & 255u;
        const unsigned int dst = wc[w][d] + pos[st];
        if (!last) {
            Ko[dst] = key[st];
            Io[dst] = idx[st];
        } else {
            ckey[dst] = ckey3[idx[st]];
            cslot[dst] = cslot3[idx[st]];
        }
    }
    if (last && b == 0)
        for (int t = threadIdx.x; t < a.T; t += blockDim.x)
            if (a.needsort[t] == 1) a.needsort[t] = 2;
}

// the sync-free plan as the list-stable radix sort; false (not done) when no
// plan has landed or the keys would not fit 32 bits
static int launch_segsort_radix(adlbq_server *h, bool *done) {
    *done = false;
    int g_last = 0, lo_last = 0, phi_last = -1;
    if (!plan_hint(h, &g_last, &lo_last, &phi_last)) return ADLBQ_OK;
    const int T = h->T;
    if (T < 1 || T > ADLBQ_MAX_TYPES) return ADLBQ_OK;
    const int tb = T > 1 ? 32 - __builtin_clz((unsigned int)(T - 1)) : 0;
    int pb = std::max(1, std::min(31, phi_last + 3));  // two bits of margin above the last batch's
    const int passes = (tb + pb + 7) / 8;
    pb = std::min(31, passes * 8 - tb);  // the last digit's spare bits widen the margin for free
    if (tb + pb > 32 || pb <= phi_last) return ADLBQ_OK;
    hipStream_t s = h->stream;
    const long long gb = std::min<long long>(h->cap_cand, (long long)g_last + g_last / 4 + 4096);
    const int nblk = (int)((gb + RS_TILE - 1) / RS_TILE);
    if (gb > h->cap_c3 || 4 * gb > h->cap_rs || 256ll * nblk > h->cap_rs_cnt) {
        AQ_HIP(hipStreamSynchronize(s));
        if (gb > h->cap_c3) {
            if (h->d_ckey3) AQ_HIP(hipFree(h->d_ckey3));
            if (h->d_cslot3) AQ_HIP(hipFree(h->d_cslot3));
            h->cap_c3 = std::min(std::max(gb, h->cap_cand / 4), h->cap_cand);
            AQ_HIP(hipMalloc((void **)&h->d_ckey3, sizeof(unsigned long long) * h->cap_c3));
            AQ_HIP(hipMalloc((void **)&h->d_cslot3, sizeof(int) * h->cap_c3));
        }
        if (4 * gb > h->cap_rs) {
            if (h->d_rs) AQ_HIP(hipFree(h->d_rs));
            h->cap_rs = 4 * std::max(gb, h->cap_cand / 4);
            AQ_HIP(hipMalloc((void **)&h->d_rs, sizeof(unsigned int) * h->cap_rs));
        }
        if (256ll * nblk > h->cap_rs_cnt) {
            if (h->d_rs_cnt) AQ_HIP(hipFree(h->d_rs_cnt));
            h->cap_rs_cnt = 256ll * std::max<long long>(nblk, (h->cap_cand / 4 + RS_TILE - 1) / RS_TILE);
            AQ_HIP(hipMalloc((void **)&h->d_rs_cnt, sizeof(int) * h->cap_rs_cnt));
        }
    }
    if (!h->d_rs_acc) {  // two parities of [64] OR, [64] AND
        AQ_HIP(hipMalloc((void **)&h->d_rs_acc, sizeof(unsigned int) * 256));
        for (int q = 0; q < 2; q++) {
            AQ_HIP(hipMemsetAsync(h->d_rs_acc + 128 * q, 0, sizeof(unsigned int) * 64, s));
            AQ_HIP(hipMemsetAsync(h->d_rs_acc + 128 * q + 64, 0xff, sizeof(unsigned int) * 64, s));
        }
    }
    h->rs_parity ^= 1;
    const RsArgs ra{T, pb, (int)gb, nblk, h->d_candoff, h->d_candlen, h->d_needsort,
                    h->d_rs_acc + 128 * h->rs_parity, h->d_rs_acc + 128 * (h->rs_parity ^ 1), h->d_rs_cnt, h->d_ctr};
    unsigned int *K0 = h->d_rs, *I0 = h->d_rs + gb, *K1 = h->d_rs + 2 * gb, *I1 = h->d_rs + 3 * gb;
    k_rs_keys<<<(int)std::min<long long>(1024, (gb + 255) / 256), 256, 0, s>>>(ra, h->d_ckey, h->d_cslot, h->d_ckey3,
                                                                          h->d_cslot3, K0, I0);
    for (int p = 0; p < passes; p++) {
        const bool last = p == passes - 1;
        k_rs_count<<<nblk, RS_THREADS, 0, s>>>(ra, p, K0);
        k_rs_scatter<<<nblk, RS_THREADS, 0, s>>>(ra, p, last ? 1 : 0, K0, I0, K1, I1, h->d_ckey3, h->d_cslot3,
                                                 h->d_ckey, h->d_cslot);
        std::swap(K0, K1);
        std::swap(I0, I1);
    }
    AQ_HIP(hipGetLastError());
    h->n_sort_radix++;
    *done = true;
    return ADLBQ_OK;
}

// The lists of multi-priority thresholds sorted after a read-back of their
// bounds (no plan from a landed batch yet): each long list by a device-wide
// radix sort of its own, the short ones one workgroup each.  The keys' varying
// bits are recorded (k_keybits, k_sort_plan) for the next batch's sync-free
// radix sort.
constexpr int SEGSORT_WIDE = 16384;  // a list this long or longer gets a device-wide sort of its own

static int launch_segsort(adlbq_server *h) {
    const int T = h->T;
    hipStream_t s = h->stream;
    if (!h->d_kb) AQ_HIP(hipMalloc((void **)&h->d_kb, sizeof(unsigned long long) * 2 * ADLBQ_MAX_TYPES));
    const int kgx = 16;  // blocks per list of the key pass
    AQ_HIP(hipMemsetAsync(h->d_kb, 0, sizeof(unsigned long long) * ADLBQ_MAX_TYPES, s));
    AQ_HIP(hipMemsetAsync(h->d_kb + ADLBQ_MAX_TYPES, 0xff, sizeof(unsigned long long) * ADLBQ_MAX_TYPES, s));
    k_keybits<<<dim3(kgx, T), 256, 0, s>>>(h->d_candoff, h->d_candlen, h->d_ckey, h->d_kb);
    if (!h->d_plan) AQ_HIP(hipMalloc((void **)&h->d_plan, sizeof(int) * 4));
    k_sort_plan<<<1, 64, 0, s>>>(T, h->d_candoff, h->d_candlen, h->d_needsort, h->d_kb, 0, 64, h->d_plan, h->d_ctr);
    AQ_HIP(hipGetLastError());
    std::vector<int> hb(3 * (size_t)T + 1);
    AQ_HIP(hipMemcpyAsync(hb.data(), h->d_candoff, sizeof(int) * (T + 1), hipMemcpyDeviceToHost, s));
    AQ_HIP(hipMemcpyAsync(hb.data() + T + 1, h->d_candlen, sizeof(int) * T, hipMemcpyDeviceToHost, s));
    AQ_HIP(hipMemcpyAsync(hb.data() + 2 * T + 1, h->d_needsort, sizeof(int) * T, hipMemcpyDeviceToHost, s));
    AQ_HIP(hipStreamSynchronize(s));
    // wide lists first, then the short ones
    SegList sl{};
    int maxlen = 0, nwide = 0;
    for (int pass = 0; pass < 2; pass++)
        for (int t = 0; t < T; t++) {
            const int off = hb[t], len = hb[T + 1 + t], ns = hb[2 * T + 1 + t];
            if (ns != 1 || len < 2 || (len >= SEGSORT_WIDE) != (pass == 0)) continue;
            sl.type[sl.n] = t;
            sl.beg[sl.n] = off;
            sl.end[sl.n] = off + len;
            sl.n++;
            nwide += pass == 0;
            maxlen = std::max(maxlen, len);
        }
    if (sl.n == 0) return ADLBQ_OK;
    h->n_segsort += nwide;
    const int nshort = sl.n - nwide;
    if (nwide > 0) {
        const size_t tmp = rsx_temp_bytes(maxlen);
        if (tmp > h->cap_ssort) {
            if (h->d_ssort) AQ_HIP(hipFree(h->d_ssort));
            h->cap_ssort = std::max(tmp, 2 * h->cap_ssort);
            AQ_HIP(hipMalloc(&h->d_ssort, h->cap_ssort));
        }
    }
    int rc;
    for (int q = 0; q < nwide; q++) {  // a device-wide sort of its own per long list
        const int b = sl.beg[q], len = sl.end[q] - b;
        if ((rc = rsx_sort_pairs(h->d_ssort, h->cap_ssort, h->d_ckey + b, h->d_ckey2 + b, h->d_cslot + b,
                                 h->d_cslot2 + b, len, 0, 64, true, s)))
            return rc;
    }
    if (nshort > 0)  // one workgroup per short list
        k_segsort_short<<<nshort, 1024, 0, s>>>(sl, nwide, h->d_ckey, h->d_cslot, h->d_ckey2, h->d_cslot2);
    const int gx = std::min((maxlen + 255) / 256, 256);
    k_segsort_back<<<dim3(gx, sl.n), 256, 0, s>>>(sl, h->d_ckey2, h->d_cslot2, h->d_ckey, h->d_cslot, h->d_needsort);
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

// k_finalize's arguments for a batch
static FinArgs fin_args(adlbq_server *h, int R, const int *d_reqs, int *d_resp, DevCounters *snap) {
    return FinArgs{d_reqs, R, h->d_tmatch, h->d_umatch, h->d_cslot, h->d_meta, h->d_pin, h->my_world, d_resp,
                   h->d_ctr, donor_ctx(h), (h->S > 1 || !h->tq.empty()) ? 1 : 0, h->d_rq_rank, h->d_rq_types,
                   h->d_rq_live, h->d_rq_req, h->d_rq_seq, h->d_dem, h->T, snap, h->snap_tag[h->snap_next],
                   h->d_anchor, h->d_anchor_next, h->d_pmask, h->d_gcut, h->d_gcut_next, h->d_rrec, h->d_needsort,
                   h->d_rank_sync + ADLBQ_MAX_TYPES + 1, h->d_mslot, h->d_rh, h->fin_flat, h->fin_snap_diag,
                   ((uintptr_t)d_resp & 15) == 0 ? 1 : 0};
}

// the host side of a batch in flight: its snapshot slot, counts, upper bounds
static void batch_launched(adlbq_server *h, int R, int export_k, const int *d_reqs) {
    h->last_reqs = d_reqs;  // its d_rh rows describe these requests (adlbq_unreserve_resp_device)
    h->last_R = R;
    // its k_finalize (fin_request) writes d_mslot; a batch with targeted units in the queue is not trusted
    // (k_thresholds' anchor bound covers the open bucket's units only)
    h->mslot_epoch = h->live_targeted == 0 ? h->mut_epoch : ~0ull;
    h->batch_export_k = export_k;
    h->batch_export_R = R;
    h->launched_reserves += R;
    h->snap_at[h->snap_next] = h->launched_reserves;
    h->snap_next = (h->snap_next + 1) % adlbq_server::NSNAP;
    h->hint_stamp++;  // a new snapshot slot is in flight: look again next time
    h->ctr_stale = true;
    h->rq_n_upper += R;
    h->rq_next_upper += R;
}

// ---------------------------------------------------------------- small queues: one workgroup
// An open bucket of at most SMALL_UNITS units and a batch of at most
// SMALL_R Reserves: the request preparation (unless a targeted phase needs it
// first), then the whole untargeted choice in one workgroup -- the available
// units gathered and sorted by (type, prio desc, position asc) in LDS, then
// the serial dictatorship in request order on one wave (lane t holds type t's
// list head; a Reserve takes the least head among its types), the same rule
// as xq.c:190-247 / adlb.c:1199-1317 that the batch pipeline evaluates in
// parallel.  Writes umatch / cslot for k_finalize (cslot[j] = request j's unit).
constexpr int SMALL_UNITS = 4 * PAGE, SMALL_R = 1024;  // 140 KB of LDS

struct SmallArgs {
    PrepArgs pa;
    int prep;  // 1: prepare the requests here (no targeted phase)
    const int *pages;
    int npages, tail_fill;
    const int *prio;
    const uint32_t *meta;
    int T, R;
    int *umatch, *cslot, *needsort;
    const int *tmatch;
    const unsigned long long *mask;
    DevCounters *ctr;
    int *sortfail;  // set: k_finalize answers the batch ADLB_ERROR (a choice outside the page list)
    int inject;     // test only: the first choice is told a position past the page list
};


// sort key, ascending = better within a type: type (7 bits), prio descending, position ascending
__device__ __forceinline__ unsigned long long small_key(int t, int pr, unsigned int pos) {
    return ((unsigned long long)t << 56) | ((unsigned long long)(~((unsigned int)pr ^ 0x80000000u)) << 24) |
           (unsigned long long)pos;
}

constexpr int SMALL_THREADS = 1024;

template <int TB>
__global__ __launch_bounds__(SMALL_THREADS) void k_reserve_small(SmallArgs a) {
    extern __shared__ unsigned long long skey[];  // [m] keys, then R masks, then R targeted flags
    __shared__ int s_n, s_start[ADLBQ_MAX_TYPES], s_end[ADLBQ_MAX_TYPES];
    const int tid = threadIdx.x, lane = tid & 63, T = a.T, R = a.R;
    if (a.prep) {
        const int nprep = (R + PREP_BLOCK - 1) / PREP_BLOCK;
        for (int b = 0; b < nprep; b++) {
            prep_block<TB>(a.pa, b);
            __syncthreads();
        }
    }
    if (tid == 0) s_n = 0;
    if (tid < ADLBQ_MAX_TYPES) s_start[tid] = s_end[tid] = 0;
    if (tid < T) a.needsort[tid] = 0;  // k_finalize reports needsort_last from it
    __syncthreads();
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    // the available units, appended in any order (they are sorted next); every load in flight first
    const int nslots = a.npages > 0 ? (a.npages - 1) * PAGE + a.tail_fill : 0;
    constexpr int GPT = SMALL_UNITS / SMALL_THREADS;
    uint32_t gm[GPT];
    int gp[GPT];
#pragma unroll
    for (int g = 0; g < GPT; g++) gm[g] = 0u, gp[g] = LOWEST;
    if (nslots > 0) {
        // unconditional loads (slot 0 of page 0 past the end, masked after): loads inside a branch were
        // issued one unit at a time.  Two rounds: the page ids, then every unit's meta and prio.
        int pgs[GPT];
#pragma unroll
        for (int g = 0; g < GPT; g++) {
            const int i = g * SMALL_THREADS + tid;
            pgs[g] = a.pages[(i < nslots ? i : 0) >> PAGE_SHIFT];
        }
#pragma unroll
        for (int g = 0; g < GPT; g++) {
            const int i = g * SMALL_THREADS + tid;
            const long long slot = ((long long)pgs[g] << PAGE_SHIFT) | (i < nslots ? (i & (PAGE - 1)) : 0);
            const uint32_t m = a.meta[slot];
            const int pr = a.prio[slot];
            unsigned int km = i < nslots ? ~0u : 0u;  // opaque: a select would be sunk into a branch
            asm volatile("" : "+v"(km));
            gm[g] = m & km;  // 0: not LIVE
            gp[g] = pr;
        }
    }
    unsigned long long gk[GPT];  // this thread's units' keys, ~0 when not available
#pragma unroll
    for (int g = 0; g < GPT; g++) {
        const int i = g * SMALL_THREADS + tid;
        const bool av = (gm[g] & (M_LIVE | M_PINNED)) == M_LIVE && gp[g] > LOWEST;
        gk[g] = av ? small_key((int)(gm[g] & M_TYPE), gp[g], (unsigned int)i) : ~0ull;
    }
    unsigned long long *smask = skey + SMALL_UNITS;
    int *stm = reinterpret_cast<int *>(smask + SMALL_R);
    for (int j = tid; j < R; j += SMALL_THREADS) {  // written by this launch's prep or earlier kernels: sc1 loads
        stm[j] = __hip_atomic_load(a.tmatch + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        smask[j] = __hip_atomic_load(a.mask + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int g = 0; g < GPT; g++) {
        const bool av = gk[g] != ~0ull;
        const unsigned long long b = __ballot(av);
        int base = 0;
        if (lane == 0 && b) base = atomicAdd(&s_n, __popcll(b));
        base = __shfl(base, 0, 64);
        if (av) skey[base + mbcnt64(b)] = gk[g];
    }
    __syncthreads();
    const int n = s_n;
    int mpow = 1;
    while (mpow < n) mpow <<= 1;
    for (int i = n + tid; i < mpow; i += SMALL_THREADS) skey[i] = ~0ull;
    __syncthreads();
    // bitonic sort, ascending
    for (int k = 2; k <= mpow; k <<= 1) {
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int i = tid; i < mpow; i += SMALL_THREADS) {
                const int x = i ^ jj;
                if (x > i) {
                    const unsigned long long u = skey[i], v = skey[x];
                    const bool up = (i & k) == 0;
                    if ((u > v) == up) {
                        skey[i] = v;
                        skey[x] = u;
                    }
                }
            }
            __syncthreads();
        }
    }
    // each type's run
    for (int i = tid; i < n; i += SMALL_THREADS) {
        const int t = (int)(skey[i] >> 56);
        if (i == 0 || (int)(skey[i - 1] >> 56) != t) s_start[t] = i;
        if (i == n - 1 || (int)(skey[i + 1] >> 56) != t) s_end[t] = i + 1;
    }
    __syncthreads();
    if (tid >= 64) return;
    const unsigned long long t_sorted = __builtin_amdgcn_s_memrealtime();
    constexpr unsigned long long KM = (1ull << 56) - 1;  // key without the type field
    auto uni = [](unsigned long long x) {  // a wave-uniform value into scalar registers
        return ((unsigned long long)(unsigned int)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
               (unsigned long long)(unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)x);
    };
    if constexpr (TB <= 8) {
        // T <= 8: every type's head, and the two after it (loads in flight), held uniformly: a
        // Reserve is a few scalar compares, no cross-lane step
        unsigned long long c0[TB], c1[TB], c2[TB];
        int hp[TB], he[TB];
#pragma unroll
        for (int q = 0; q < TB; q++) {
            hp[q] = q < T ? s_start[q] : 0;
            he[q] = q < T ? s_end[q] : 0;
            c0[q] = hp[q] < he[q] ? uni(skey[hp[q]]) : ~0ull;
            c1[q] = hp[q] + 1 < he[q] ? uni(skey[hp[q] + 1]) : ~0ull;
            c2[q] = hp[q] + 2 < he[q] ? uni(skey[hp[q] + 2]) : ~0ull;
        }
        unsigned long long mreg = 0ull;  // lane l: request j0 + l's mask (0: matched in the targeted phase)
        int um_l = -1, cs_l = -1;         // lane l: request j0 + l's results, stored once per 64
        unsigned int live = 0u;           // types whose list is not exhausted (uniform)
#pragma unroll
        for (int q = 0; q < TB; q++) live |= c0[q] != ~0ull ? (1u << q) : 0u;
        int j = 0;
        for (; j < R && live; j++) {
            if ((j & 63) == 0) {
                const int jl = j + lane;
                mreg = jl < R && stm[jl] < 0 ? smask[jl] : 0ull;
                um_l = -1;
                cs_l = -1;
            }
            const unsigned long long mk =
                ((unsigned long long)(unsigned int)__builtin_amdgcn_readlane((int)(mreg >> 32), j & 63) << 32) |
                (unsigned long long)(unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)mreg, j & 63);
            unsigned long long best = ~0ull;
            int bq = -1;
            if (mk & live) {
#pragma unroll
                for (int q = 0; q < TB; q++)
                    if (((mk >> q) & 1ull) && c0[q] != ~0ull && (c0[q] & KM) < best) {
                        best = c0[q] & KM;
                        bq = q;
                    }
            }
            if (bq >= 0) {
#pragma unroll
                for (int q = 0; q < TB; q++)
                    if (q == bq) {
                        hp[q]++;
                        c0[q] = c1[q];
                        c1[q] = c2[q];
                        c2[q] = hp[q] + 2 < he[q] ? uni(skey[hp[q] + 2]) : ~0ull;
                        if (c0[q] == ~0ull) live &= ~(1u << q);
                    }
                const unsigned int pos =
                    (a.inject && j == 0) ? (unsigned int)a.npages << PAGE_SHIFT : (unsigned int)(best & 0xffffffu);
                if ((j & 63) == lane && pos_in_list(pos, a.npages, a.ctr, a.sortfail)) {
                    cs_l = (a.pages[pos >> PAGE_SHIFT] << PAGE_SHIFT) | (int)(pos & (PAGE - 1));
                    um_l = j;
                }
            }
            if ((j & 63) == 63 || j == R - 1 || !live) {  // this block of 64 Reserves' results
                const int jl = (j & ~63) + lane;
                if (jl <= j) {
                    a.umatch[jl] = um_l;
                    a.cslot[jl] = cs_l;
                }
            }
        }
        for (int jl = j + lane; jl < R; jl += 64) a.umatch[jl] = -1;  // every list exhausted: no unit left
        if (lane == 0) {  // diagnostic sums
            const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
            atomicAdd((unsigned long long *)&a.ctr->diag[0], (unsigned long long)n);
            atomicAdd((unsigned long long *)&a.ctr->diag[1], (unsigned long long)R);
            atomicAdd((unsigned long long *)&a.ctr->diag[2], t_sorted - t_start);
            atomicAdd((unsigned long long *)&a.ctr->diag[3], t_end - t_sorted);
            atomicAdd((unsigned long long *)&a.ctr->diag[4], 1ull);
        }
        return;
    }
    // the serial dictatorship: lane t = type t, its head and the one after (the next head in flight)
    const bool tl = lane < T;
    const int e = tl ? s_end[lane] : 0;
    int h = tl ? s_start[lane] : 0;
    unsigned long long cur = h < e ? skey[h] : ~0ull, nxt = h + 1 < e ? skey[h + 1] : ~0ull;
    int tp = 1;
    while (tp < T) tp <<= 1;
    unsigned long long mreg = 0ull;  // lane l: request j0 + l's mask (0: matched in the targeted phase)
    for (int j = 0; j < R; j++) {
        if ((j & 63) == 0) {
            const int jl = j + lane;
            mreg = jl < R && stm[jl] < 0 ? smask[jl] : 0ull;
        }
        const unsigned long long mk =
            ((unsigned long long)(unsigned int)__builtin_amdgcn_readlane((int)(mreg >> 32), j & 63) << 32) |
            (unsigned long long)(unsigned int)__builtin_amdgcn_readlane((int)(unsigned int)mreg, j & 63);
        // compared across types without the type field: prio descending, position ascending
        // (an exhausted list's head is ~0: no candidate)
        const unsigned long long c =
            (tl && cur != ~0ull && ((mk >> lane) & 1ull)) ? (cur & ((1ull << 56) - 1)) : ~0ull;
        unsigned long long best = c;
        for (int o = 1; o < tp; o <<= 1) best = min(best, (unsigned long long)__shfl_xor(best, o, 64));
        best = ((unsigned long long)(unsigned int)__builtin_amdgcn_readfirstlane((int)(best >> 32)) << 32) |
               (unsigned long long)(unsigned int)__builtin_amdgcn_readfirstlane((int)(unsigned int)best);  // lane 0's
        if (best != ~0ull) {
            const unsigned long long w = __ballot(tl && c == best);
            if (lane == __ffsll((long long)w) - 1) {
                h++;
                cur = nxt;
                nxt = h + 1 < e ? skey[h + 1] : ~0ull;
            }
            if (lane == 0) {
                const unsigned int pos =
                    (a.inject && j == 0) ? (unsigned int)a.npages << PAGE_SHIFT : (unsigned int)(best & 0xffffffu);
                const bool ok = pos_in_list(pos, a.npages, a.ctr, a.sortfail);
                a.cslot[j] = ok ? (a.pages[pos >> PAGE_SHIFT] << PAGE_SHIFT) | (int)(pos & (PAGE - 1)) : -1;
                a.umatch[j] = ok ? j : -1;
            }
        } else if (lane == 0) {
            a.umatch[j] = -1;
        }
    }
}

// More than ADLBQ_MAX_TYPES types: the sorted-runs choice (adlbq_wide.hip), then k_finalize.
static int launch_reserve_wide(adlbq_server *h, int R, const int *d_reqs, int *d_resp) {
    int rc;
    if ((rc = wide_choose(h, R, d_reqs))) return rc;
    DevCounters *const snap = h->d_snap + h->snap_next;
    h->snap_tag[h->snap_next] = ++h->snap_tags;
    __atomic_store_n(&h->h_snap[h->snap_next].snap_tag, 0ull, __ATOMIC_RELEASE);
    const FinArgs fa = fin_args(h, R, d_reqs, d_resp, snap);
    k_finalize<<<(R + 255) / 256, 256, 0, h->stream>>>(fa);
    AQ_HIP(hipGetLastError());
    batch_launched(h, R, 0, d_reqs);
    return ADLBQ_OK;
}

// The kernels a handle recorded (GroupRec), launched one by one on its own stream.
static int launch_recorded(adlbq_server *h, GroupRec &r) {
    hipStream_t s = h->stream;
    const bool t4 = r.tb == 4;
    if (r.kinds & GK_PREP) {
        auto kph = t4 ? k_prep_hist<4> : k_prep_hist<8>;
        kph<<<r.prep.grid, 256, r.lds_prep, s>>>(r.prep.pa, r.prep.nprep, r.prep.ha);
    }
    if (r.kinds & GK_THR) {
        const GThr &g = r.thr;
        k_thresholds<<<g.grid, TH_THREADS, 0, s>>>(g.zcs, g.zn, g.T, g.dem, g.csum, g.nchunks, g.theta, g.need,
                                                   g.candlen, g.needsort, g.binoff, g.coltot, g.type_cnt, g.anchor,
                                                   g.anchor_next, g.gcut_next, g.guess, g.gcut);
    }
    if ((r.kinds & GK_SEL) && r.selw) {
        const GSel &g = r.sel;
        auto selw = t4 ? k_select_wave<4> : k_select_wave<8>;
        selw<<<g.grid, 64, r.lds_sel, s>>>(g.pages, g.npages, g.tail_fill, g.prio, g.meta, g.T, g.anchor, g.theta,
                                            g.need, g.binoff, g.csum, g.gh, g.candlen, g.candoff_out, g.ckey, g.cslot,
                                            g.gcut, g.spec, g.specn, g.pbase, g.pwide, g.ctr, g.crank, g.lv, g.rtype,
                                            g.R, nullptr);
    } else if (r.kinds & GK_SEL) {
        const GSel &g = r.sel;
        auto sel = t4 ? k_select_open<4> : k_select_open<8>;
        sel<<<g.grid, 256, r.lds_sel, s>>>(g.pages, g.npages, g.tail_fill, g.prio, g.meta, g.seqa, g.T, g.anchor,
                                           g.theta, g.need, g.binoff, g.csum, g.gh, g.candlen, g.candoff_out, g.ckey,
                                           g.cslot, g.gcut, g.spec, g.specn, g.pbase, g.pwide, g.ctr, g.crank, g.lv,
                                           g.rtype, g.R, nullptr);
    }
    if (r.kinds & GK_RANK) k_rank<<<r.rank.grid, RANK_TILE, 0, s>>>(r.rank.ra);
    if (r.kinds & GK_CHAIN) {
        const GChain &g = r.chain;
        (t4 ? k_chain0<4> : k_chain0<8>)<<<g.grid, 64, r.lds_chain, s>>>(g.a, g.cp, g.prefix_next, g.final);
    }
    if (r.kinds & GK_FIN) k_finalize<<<r.fin.grid, 256, 0, s>>>(r.fin.f);
    r.kinds = 0;
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

int launch_reserve(adlbq_server *h, int R, const int *d_reqs, int *d_resp) {
    int rc;
    const auto host_t0 = std::chrono::steady_clock::now();
    h->mut_epoch++;   // pins units (and may fail before writing d_mslot)
    h->hint_stamp++;  // landed-snapshot hints are looked up once for this launch
    h->reserve_batches++;
    using hclk = std::chrono::steady_clock;
    auto hsec = [&](const char *name, hclk::time_point &t) {  // always-on host section timer
        const auto now = hclk::now();
        h->hacc[name] += std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
        t = now;
    };
    auto ht = host_t0;
    if ((rc = ensure_req_capacity(h, R))) return rc;
    hsec("req_cap", ht);
    recycle_apply(h);
    maybe_compact_rq(h);
    if ((rc = sync_tables(h))) return rc;
    if ((rc = recycle_launch(h))) return rc;
    hsec("tables", ht);
    if ((rc = ensure_rq_capacity(h, R))) return rc;
    hsec("rq_cap", ht);
    if (h->T > ADLBQ_MAX_TYPES) return launch_reserve_wide(h, R, d_reqs, d_resp);
    const int T = h->T;
    const int np = (int)h->open.pages.size();
    if ((rc = ensure_scan_capacity(h, std::max(np, 1)))) return rc;
    hsec("scan_cap", ht);
    hipStream_t s = h->stream;
    hipEvent_t ev;

    PrepArgs pa{d_reqs, R, h->d_utypes, T, h->d_mask, h->d_dem, h->d_seg_cnt, h->d_ctr, h->d_tmatch,
                nullptr, 0, nullptr, nullptr, 0, h->export_extra, h->d_rh};
    const int nb = (int)h->bucket_ranks.size();
    const bool targeted = h->live_targeted > 0 && nb > 0;
    // small rank buckets and few Reserves per bucket (config 5's bound updates): each bucket's Reserves
    // scan its pages (k_targeted) -- no sorted index to keep up to date after every targeted Put
    bool tscan = targeted && nb < (1 << 20) && h->targeted_scan != 0;
    if (tscan && h->targeted_scan < 0) {
        tscan = (long long)R <= 4ll * nb;
        for (int k = 0; k < nb && tscan; k++) tscan = (int)h->rankb[k].pages.size() <= 1;
    }
    if (targeted && nb < (1 << 20) && !tscan) {  // per-bucket Reserve lists for k_targeted_idx
        const int tcap = std::min(TGT_REQ, std::max(64, 2 * ((R + nb - 1) / nb) + 64));
        if ((long long)nb > h->cap_tcnt || (long long)nb * tcap > h->cap_tlist) {
            AQ_HIP(hipStreamSynchronize(s));
            if ((long long)nb > h->cap_tcnt) {
                if (h->d_tcnt) AQ_HIP(hipFree(h->d_tcnt));
                h->cap_tcnt = std::max<long long>(nb, 2 * h->cap_tcnt);
                AQ_HIP(hipMalloc((void **)&h->d_tcnt, sizeof(int) * h->cap_tcnt));
                AQ_HIP(hipMemsetAsync(h->d_tcnt, 0, sizeof(int) * h->cap_tcnt, s));  // k_targeted_idx re-zeroes its own
            }
            if ((long long)nb * tcap > h->cap_tlist) {
                if (h->d_tlist) AQ_HIP(hipFree(h->d_tlist));
                h->cap_tlist = std::max<long long>((long long)nb * tcap, 2 * h->cap_tlist);
                AQ_HIP(hipMalloc((void **)&h->d_tlist, sizeof(int) * h->cap_tlist));
            }
        }
        h->tcap = tcap;
        pa.rank2b = h->d_rank2b;
        pa.A = h->A;
        pa.tcnt = h->d_tcnt;
        pa.tlist = h->d_tlist;
        pa.tcap = tcap;
    }
    host_stage_add(h, "pre", host_t0);
    const auto scan_t0 = std::chrono::steady_clock::now();
    // a small open bucket and batch: one workgroup chooses (k_reserve_small), no scan
    // one Reserve, no targeted units: one launch (k_reserve_one), whatever the bucket's size (k_reserve_small
    // sorts every live unit of its pages, ~260 us at 10K units)
    const bool one = !h->grec && T > 0 && T <= 8 && R == 1 && h->live_targeted == 0 && h->reserve_one && np > 0;
    const bool small = !one && !h->grec && T > 0 && R <= std::min(h->small_r, SMALL_R) && np <= h->small_pages &&
                       (long long)np * PAGE <= SMALL_UNITS;
    if (small) {
        if (targeted) {  // the targeted phase reads the prepared requests first
            const int nprep = (R + PREP_BLOCK - 1) / PREP_BLOCK;
            HistArgs none{};
            auto kph = T <= 4 ? k_prep_hist<4> : T <= 8 ? k_prep_hist<8> : k_prep_hist<64>;
            kph<<<nprep, 256, 0, s>>>(pa, nprep, none);
        }
    } else if (!one && (rc = launch_scan(h, pa, (R + PREP_BLOCK - 1) / PREP_BLOCK, false, R))) {
        return rc;
    }
    host_stage_add(h, "scan", scan_t0);
    auto hl = hclk::now();
    h->hacc["l_scan"] += std::chrono::duration_cast<std::chrono::nanoseconds>(hl - scan_t0).count();
    h->last_scan_units = h->live_units - h->live_targeted;

    // a group member whose batch needs a launch between the recorded ones (the targeted index, a
    // read-back sort) launches what it recorded on its own stream and leaves the group
    auto leave_group = [&]() -> int {
        if (!h->grec) return ADLBQ_OK;
        const int r2 = launch_recorded(h, *h->grec);
        h->grec = nullptr;
        return r2;
    };
    if (targeted) {
        if ((rc = leave_group())) return rc;
        const auto ti_t0 = std::chrono::steady_clock::now();
        if (tscan) {  // the index is not kept meanwhile: the next indexed batch rebuilds it in full
            h->tnew_keys.clear();
            h->tnew_vals.clear();
            h->tidx_valid = false;
            h->tindex_dirty = true;
            h->tscan_batches++;
        } else if (nb < (1 << 20) && (rc = ensure_tindex(h))) {
            return rc;
        }
        host_stage_add(h, "tindex", ti_t0);
        auto tt = ti_t0;
        hsec("tindex", tt);
        stage_begin(h, "targeted", &ev);
        if (nb < (1 << 20) && !tscan)
            k_targeted_idx<<<nb, 256, 0, s>>>(h->d_bucket_ranks, h->d_rank_pstart, h->d_rank_pages, h->d_tkeys,
                                              h->d_tvals, h->d_tstart, h->d_tend,
                                              TDelta{h->d_dkeys, h->d_dvals, h->d_dstart, h->d_dend, (int)h->tdel_n},
                                              T, h->d_meta, h->d_mask, d_reqs, R,
                                              h->d_tmatch, h->d_seg_cnt, h->d_tcnt, h->d_tlist, h->tcap,
                                              h->targeted_diag);
        else
            k_targeted<<<nb, 256, 0, s>>>(h->d_bucket_ranks, h->d_rank_pstart, h->d_rank_pages, h->d_rank_fill,
                                          h->d_prio, h->d_meta, h->d_mask, d_reqs, R, h->d_tmatch, h->d_seg_cnt);
        stage_end(h, "targeted", ev);
    }
    if (one) {
        // page pairs, at most 256 workgroups at a time (they step through the pairs in bucket order and
        // stop once every wanted type's best unit is known: k_reserve_one); fewer stop sooner on a queue
        // whose best units sit at the anchors, more read a whole bucket faster (profiles/r06_variants.txt)
        const int grid = std::min((np + 1) / 2, h->one_grid > 0 ? h->one_grid : 256);
        if (grid > h->cap_onepart) {
            AQ_HIP(hipStreamSynchronize(s));
            if (h->d_onepart) AQ_HIP(hipFree(h->d_onepart));
            h->cap_onepart = std::max(grid, 2 * h->cap_onepart);
            // [16] arrival counters (ints), then [grid][8] per-type minima, then 16 KB of zeros (the
            // meta k_reserve_one reads past the open pages: nothing LIVE, no mask register needed)
            const size_t zoff = (size_t)8 * (h->cap_onepart + 2);
            AQ_HIP(hipMalloc((void **)&h->d_onepart, sizeof(unsigned long long) * (zoff + 2048)));
            AQ_HIP(hipMemsetAsync(h->d_onepart, 0, sizeof(unsigned long long) * 16, s));
            AQ_HIP(hipMemsetAsync(h->d_onepart + 16, 0xff, sizeof(unsigned long long) * 8, s));  // per-type best: none
            AQ_HIP(hipMemsetAsync(h->d_onepart + zoff, 0, sizeof(unsigned long long) * 2048, s));
        }
        DevCounters *const snap = h->d_snap + h->snap_next;
        h->snap_tag[h->snap_next] = ++h->snap_tags;
        __atomic_store_n(&h->h_snap[h->snap_next].snap_tag, 0ull, __ATOMIC_RELEASE);
        int pg0 = h->open.pages[0];
        for (int i = 1; i < np && pg0 >= 0; i++)
            if (h->open.pages[(size_t)i] != pg0 + i) pg0 = -1;
        const OneArgs oa{pa, h->d_open_pages, np, h->open.tail_fill, pg0, h->d_prio, h->d_meta, h->d_pbase, h->d_pwide, T,
                         h->d_onepart + 16, reinterpret_cast<int *>(h->d_onepart), h->d_umatch, h->d_cslot,
                         fin_args(h, R, d_reqs, d_resp, snap), h->bound_inject,
                         reinterpret_cast<const uint32_t *>(h->d_onepart + (size_t)8 * (h->cap_onepart + 2))};
        h->bound_inject = 0;
        stage_begin(h, "one", &ev);
        if (T <= 4) k_reserve_one<4><<<grid, 256, 0, s>>>(oa);
        else k_reserve_one<8><<<grid, 256, 0, s>>>(oa);
        stage_end(h, "one", ev);
        h->one_batches++;
        AQ_HIP(hipGetLastError());
        batch_launched(h, R, 0, d_reqs);  // no candidate lists for a steal export to reuse
        return ADLBQ_OK;
    }
    if (small) {
        // what the kernel assumes: the page list it reads is the one uploaded, candidates fit d_cslot
        if (h->tables_dirty || h->pinfo_dirty || (long long)R > h->cap_cand)
            return fail(ADLBQ_ERR_DEVICE, "k_reserve_small: stale page tables or candidate buffers (internal)");
        const SmallArgs sa{pa, targeted ? 0 : 1, h->d_open_pages, np, h->open.tail_fill, h->d_prio, h->d_meta, T, R,
                           h->d_umatch, h->d_cslot, h->d_needsort, h->d_tmatch, h->d_mask, h->d_ctr,
                           h->d_rank_sync + ADLBQ_MAX_TYPES + 1, h->bound_inject};
        h->bound_inject = 0;
        const size_t lds = sizeof(unsigned long long) * (SMALL_UNITS + SMALL_R) + sizeof(int) * SMALL_R;
        stage_begin(h, "small", &ev);
        if (T <= 4) k_reserve_small<4><<<1, SMALL_THREADS, lds, s>>>(sa);
        else if (T <= 8) k_reserve_small<8><<<1, SMALL_THREADS, lds, s>>>(sa);
        else k_reserve_small<64><<<1, SMALL_THREADS, lds, s>>>(sa);
        stage_end(h, "small", ev);
        h->small_batches++;
        DevCounters *const snap = h->d_snap + h->snap_next;
        h->snap_tag[h->snap_next] = ++h->snap_tags;
        __atomic_store_n(&h->h_snap[h->snap_next].snap_tag, 0ull, __ATOMIC_RELEASE);
        const FinArgs fa = fin_args(h, R, d_reqs, d_resp, snap);
        stage_begin(h, "finalize", &ev);
        k_finalize<<<(R + 255) / 256, 256, 0, s>>>(fa);
        stage_end(h, "finalize", ev);
        AQ_HIP(hipGetLastError());
        batch_launched(h, R, 0, d_reqs);  // no candidate lists for a steal export to reuse
        return ADLBQ_OK;
    }
    auto st0 = hclk::now();
    // 8 < T <= 64: every list sorted and ranked by one binning of the keys (k_rank's tile work skipped)
    const bool kr = np > 0 && T > RANK_FAST_T && T <= ADLBQ_MAX_TYPES && h->keyrank && keyrank_hint(h);
    if (kr) {
        if ((rc = leave_group())) return rc;
        stage_begin(h, "sort", &ev);
        if ((rc = launch_keyrank(h, R))) return rc;
        stage_end(h, "sort", ev);
    } else if (np > 0 && T > 0 && sort_hint(h)) {
        if ((rc = leave_group())) return rc;
        stage_begin(h, "sort", &ev);
        bool planned = false;
        if ((rc = launch_segsort_radix(h, &planned))) return rc;
        if (!planned && (rc = launch_segsort(h))) return rc;
        stage_end(h, "sort", ev);
    }
    hsec("sort", st0);
    RankArgs rka{};
    // k_rank rides in the chain's launch (k_rank_chain0) for T <= 8 outside a group
    const bool fuse_rc = np > 0 && T > 0 && T <= 8 && !h->grec && h->fuse_rank_chain;
    int rg_fused = 0;
    if (np > 0 && T > 0) {
        if (++h->rank_epoch == 0) h->rank_epoch = 1;
        const RankSort rs{h->d_needsort, h->d_ckey2, h->d_cslot, h->d_cslot2, h->d_rank_sync, h->rank_epoch,
                          h->sort_fail_test};
        // chunk sums: zeroed by the next scan
        rka = RankArgs{T, h->d_candoff, h->d_candlen, h->d_ckey, h->d_crank, nullptr, 0, h->d_mask, h->d_tmatch, R,
                       h->d_seg_cnt, rs, LevelRows{T <= 8 ? h->d_lv : nullptr, R, h->d_rtype}, h->d_ctr};
        {
            stage_begin(h, "rank", &ev);
            // a small grid when the last landed batch was ranked in k_select_open (every loop is
            // grid-strided: any grid is correct, the hint only sizes it)
            // otherwise one workgroup per tile of the candidates a batch can list at most (the
            // demand plus the export depth per type): 1,280 workgroups cost ~20 us on small lists
            const long long tiles = ((long long)R * std::min(T, NREQ) + (long long)T * h->export_extra + RANK_TILE - 1) /
                                    RANK_TILE;
            // (keyrank: k_rank's tiles run only when the batch failed over)
            const int rgrid = h->rank_grid ? h->rank_grid
                              : kr           ? 64
                              : (T <= RANK_FAST_T && rank_hint(h)) ? 4
                                                                    : (int)std::min(1280ll, std::max(8ll, tiles));
            if (h->grec) {
                h->grec->kinds |= GK_RANK;
                h->grec->rank = GRank{rka, rgrid};
            } else if (fuse_rc) {
                // 64-thread blocks: as many threads as rgrid blocks of RANK_TILE (16 on a rank hint: its
                // blocks then only check, the chain does not wait for them)
                rg_fused = h->rank_grid ? h->rank_grid : rank_hint(h) ? 16 : rgrid * (RANK_TILE / 64);
            } else {
                k_rank<<<rgrid, RANK_TILE, 0, s>>>(rka);
            }
            stage_end(h, "rank", ev);
        }
    }
    hsec("l_rank", hl);
    // k_finalize's arguments
    DevCounters *const snap = h->d_snap + h->snap_next;
    h->snap_tag[h->snap_next] = ++h->snap_tags;
    __atomic_store_n(&h->h_snap[h->snap_next].snap_tag, 0ull, __ATOMIC_RELEASE);  // not landed until k_finalize stores it
    const FinArgs fa = fin_args(h, R, d_reqs, d_resp, snap);
    stage_begin(h, "chain", &ev);
    {
        const int nseg = (R + SEG - 1) / SEG;
        // in-launch neighbour passes of round 0, then round launches (the last
        // launch walks in order whatever is still off the fixed point)
        const int P = h->chain_passes > 0 ? std::min(h->chain_passes, CHAIN_MAX_PASSES) : (T <= 8 ? 3 : 2);
        const int K = h->chain_rounds >= 0 ? h->chain_rounds : (T <= 8 ? 0 : 2);
        const int warm = T <= 8 ? (h->chain_warm >= 0 ? h->chain_warm : CHAIN_WARM) : 0;
        const int gs = (nseg + CH_GROUPS - 1) / CH_GROUPS;
        const long long nsT = (long long)nseg * std::max(T, 1);
        // round k's mode: bit k-1 of chain_modes (1 = prefix starts); default
        // prefix rounds (the neighbour passes already ran inside round 0)
        const long long modes = h->chain_modes != -1 ? h->chain_modes : ~0ll;
        if (++h->chain_epoch == 0) h->chain_epoch = 1;
        const ChainPass cp{h->d_chE, h->d_chflag, h->chain_epoch, P};
        ChainArgs ca{h->d_mask, h->d_tmatch, R, T, nseg, warm, gs, h->d_candoff, h->d_candlen, h->d_crank,
                     h->d_umatch, h->d_cht, h->d_seg_cnt, h->d_chS, h->d_chD, h->d_chS + nsT, h->d_chD + nsT,
                     h->d_chLP, h->d_chGT, h->d_chGO, h->d_chclean, h->d_chcnt, h->d_ctr,
                     (T <= 8 && np > 0) ? h->d_lv : nullptr, h->d_rtype, nullptr, nullptr, 0ull, h->d_needsort,
                     // the prefix of seg_cnt holds unless the targeted phase changed seg_cnt after k_thresholds
                     (h->jpref_ok && !targeted) ? h->d_jpref : nullptr};
        h->jpref_ok = false;
        if (rg_fused > 0) {
            ca.rdone = h->d_chcnt + CH_GROUPS + 1;
            ca.rtarget = (h->rank_arrivals += (unsigned long long)rg_fused);
        }
        if (h->chain_stamps) {
            if (nseg > h->cap_stamps) {
                AQ_HIP(hipStreamSynchronize(s));
                if (h->d_stamps) AQ_HIP(hipFree(h->d_stamps));
                h->cap_stamps = nseg;
                AQ_HIP(hipMalloc((void **)&h->d_stamps, sizeof(unsigned long long) * 16 * nseg));
            }
            AQ_HIP(hipMemsetAsync(h->d_stamps, 0, sizeof(unsigned long long) * 16 * nseg, s));
            ca.stamps = h->d_stamps;
            h->n_stamps = nseg;
        }
        auto flip = [&](int k) {  // launch k writes buffer k & 1 and reads the other
            ca.S = h->d_chS + (k & 1) * nsT;
            ca.D = h->d_chD + (k & 1) * nsT;
            ca.Sp = h->d_chS + ((k + 1) & 1) * nsT;
            ca.Dp = h->d_chD + ((k + 1) & 1) * nsT;
        };
        flip(0);
        size_t lds;
        // small variants: windows, sentinel row, staged masks (8 B) and seeds (1 B) per request
        if (T <= 4) lds = sizeof(unsigned int) * (4 * (SEG + warm) + 64) + 9 * (SEG + warm);
        else if (T <= 8) lds = sizeof(unsigned int) * (8 * (SEG + warm) + 64) + 9 * (SEG + warm);
        else lds = sizeof(unsigned int) * T * SEG + sizeof(TypeRec) * ADLBQ_MAX_TYPES;
        auto mode_of = [&](int k) { return (k >= 1 && k <= K) ? (int)(((unsigned long long)modes >> (k - 1)) & 1ull) : 0; };
        if (h->grec) {  // T <= 8, no round launches (group_eligible)
            h->grec->kinds |= GK_CHAIN;
            h->grec->chain = GChain{ca, cp, mode_of(1), K == 0 ? 1 : 0, nseg};
            h->grec->lds_chain = lds;
        } else if (rg_fused > 0) {
            auto krc = T <= 4 ? k_rank_chain0<4> : k_rank_chain0<8>;
            krc<<<rg_fused + nseg, 64, lds, s>>>(rka, rg_fused, ca, cp, mode_of(1), K == 0);
        } else if (T <= 4) k_chain0<4><<<nseg, 64, lds, s>>>(ca, cp, mode_of(1), K == 0);
        else if (T <= 8) k_chain0<8><<<nseg, 64, lds, s>>>(ca, cp, mode_of(1), K == 0);
        else k_chain0<64><<<nseg, 64, lds, s>>>(ca, cp, mode_of(1), K == 0);
        for (int k = 1; k <= K; k++) {
            flip(k);
            const int mode = mode_of(k), pn = mode_of(k + 1);
            if (T <= 4) k_chainr<4><<<nseg, 64, lds, s>>>(ca, k, k == K, mode, pn);
            else if (T <= 8) k_chainr<8><<<nseg, 64, lds, s>>>(ca, k, k == K, mode, pn);
            else k_chainr<64><<<nseg, 64, lds, s>>>(ca, k, k == K, mode, pn);
        }
    }
    stage_end(h, "chain", ev);
    hsec("l_chain", hl);
    stage_begin(h, "finalize", &ev);
    if (h->grec) {
        h->grec->kinds |= GK_FIN;
        h->grec->fin = GFin{fa, (R + 255) / 256};
    } else {
        k_finalize<<<(R + 255) / 256, 256, 0, s>>>(fa);
    }
    stage_end(h, "finalize", ev);
    hsec("l_fin", hl);
    // the lists hold export_extra more per type: a steal export right after this batch gathers them
    AQ_HIP(hipGetLastError());
    batch_launched(h, R, (np > 0 && T > 0) ? h->export_extra : 0, d_reqs);
    auto t_all = host_t0;
    hsec("total", t_all);
    return ADLBQ_OK;
}

// The export right after a reserve batch whose lists ran export_extra >= k
// deep beyond the demand: the ordered choice took a prefix of every list (its
// heads, in order), so the k best available units of type t are the list
// entries from h_t on, h_t = the batch's choices of type t (cht); the available
// count is the scan's column total less h_t.  Records as k_export_gather.
__device__ __forceinline__ int bytes_eq(unsigned int x, unsigned int t) {
    return ((x & 0xffu) == t) + (((x >> 8) & 0xffu) == t) + (((x >> 16) & 0xffu) == t) + ((x >> 24) == t);
}

// Grid (T, ceil(k / 256)): block (t, y) counts h_t itself (16 choice bytes per
// load, four loads in flight) and gathers records [256 y, 256 y + 256) of type t.
__device__ __forceinline__ void export_after_body(int T, int k, int R, const unsigned char *__restrict__ cht,
                                                  const int *__restrict__ candoff, const int *__restrict__ candlen,
                                                  const int *__restrict__ cslot, const int *__restrict__ prio,
                                                  const int *__restrict__ seqa, const int4 *__restrict__ cold0,
                                                  const int4 *__restrict__ cold1, int *__restrict__ recs,
                                                  int *__restrict__ nrec, long long *__restrict__ navail,
                                                  const unsigned int *__restrict__ coltot, const int t, const int y,
                                                  const int ny) {
    __shared__ int s_h[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned int ut = (unsigned int)t;
    const uint4 *cv = reinterpret_cast<const uint4 *>(cht);
    const int nv = R >> 4;
    int c = 0;
    for (int q0 = threadIdx.x; q0 < nv; q0 += 4 * blockDim.x) {
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int q = q0 + i * blockDim.x;
            v[i] = q < nv ? cv[q] : make_uint4(~0u, ~0u, ~0u, ~0u);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) c += bytes_eq(v[i].x, ut) + bytes_eq(v[i].y, ut) + bytes_eq(v[i].z, ut) + bytes_eq(v[i].w, ut);
    }
    for (int j = (nv << 4) + threadIdx.x; j < R; j += blockDim.x) c += cht[j] == t;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) s_h[w] = c;
    __syncthreads();
    const int ht = s_h[0] + s_h[1] + s_h[2] + s_h[3];
    if (y == 0 && threadIdx.x < 64) {
        unsigned long long a = coltot[t * NB + threadIdx.x];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
        if (threadIdx.x == 0) navail[t] = (long long)a - ht;
    }
    const int n = max(0, min(k, candlen[t] - ht)), off = candoff[t] + ht;
    for (int i = y * blockDim.x + threadIdx.x; i < n; i += ny * blockDim.x) {
        const int slot = cslot[off + i];
        const int4 c0 = cold0[slot], c1 = cold1[slot];
        int4 *r = reinterpret_cast<int4 *>(recs + ((long long)t * k + i) * 8);
        r[0] = make_int4(prio[slot], seqa[slot], c1.z, c0.y);
        r[1] = make_int4(c0.x, c0.w, c1.x, c1.y);
    }
    if (y == 0 && threadIdx.x == 0) nrec[t] = n;
}

__global__ __launch_bounds__(256) void k_export_after(int T, int k, int R, const unsigned char *__restrict__ cht,
                                                      const int *__restrict__ candoff, const int *__restrict__ candlen,
                                                      const int *__restrict__ cslot, const int *__restrict__ prio,
                                                      const int *__restrict__ seqa, const int4 *__restrict__ cold0,
                                                      const int4 *__restrict__ cold1, int *__restrict__ recs,
                                                      int *__restrict__ nrec, long long *__restrict__ navail,
                                                      const unsigned int *__restrict__ coltot) {
    export_after_body(T, k, R, cht, candoff, candlen, cslot, prio, seqa, cold0, cold1, recs, nrec, navail, coltot,
                      blockIdx.x, blockIdx.y, gridDim.y);
}

// adlbq_steal_group_export: the shards' k_export_after as one launch, grid (T, y, shard)
__global__ __launch_bounds__(256) void k_export_after_g(const ExportAfterGroup g) {
    const ExportAfterArgs &a = g.a[blockIdx.z];
    if ((int)blockIdx.x >= a.T) return;
    export_after_body(a.T, a.k, a.R, a.cht, a.candoff, a.candlen, a.cslot, a.prio, a.seqa, a.cold0, a.cold1, a.recs,
                      a.nrec, a.navail, a.coltot, blockIdx.x, blockIdx.y, gridDim.y);
}

bool export_after_args(adlbq_server *h, int k, int *d_recs, int *d_nrec, long long *d_navail, ExportAfterArgs *a) {
    if (h->batch_export_k < k || h->T < 1) return false;
    *a = ExportAfterArgs{h->T, k, h->batch_export_R, h->d_cht, h->d_candoff, h->d_candlen, h->d_cslot, h->d_prio,
                         h->d_seq, h->d_cold0, h->d_cold1, d_recs, d_nrec, d_navail, h->d_coltot};
    return true;
}

int launch_export_after_group(const ExportAfterGroup &g, int n, int k, int Tmax, hipStream_t s) {
    k_export_after_g<<<dim3(Tmax, std::min(8, std::max(1, (k + 255) / 256)), n), 256, 0, s>>>(g);
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}

// true (and the gather enqueued) when the last reserve batch's lists serve an export of depth k
bool launch_export_after(adlbq_server *h, int k, int *d_recs, int *d_nrec, long long *d_navail) {
    if (h->batch_export_k < k || h->T < 1) return false;
    k_export_after<<<dim3(h->T, std::min(8, std::max(1, (k + 255) / 256))), 256, 0, h->stream>>>(h->T, k, h->batch_export_R, h->d_cht, h->d_candoff, h->d_candlen,
                                                h->d_cslot, h->d_prio, h->d_seq, h->d_cold0, h->d_cold1, d_recs,
                                                d_nrec, d_navail, h->d_coltot);
    return true;
}

// recs8 [T][k][8] then nrec [T] land in d_out, navail [T] in d_navail (device)
int launch_export(adlbq_server *h, int k, int *d_out, long long *d_navail) {
    if (h->T > ADLBQ_MAX_TYPES) return fail(ADLBQ_ERR_UNSUPPORTED, "steal export: more than 64 work types");
    wq_changed(h);  // the export scan rebuilds the candidate lists
    int rc;
    if ((rc = sync_tables(h))) return rc;
    const int T = h->T;
    const int np = (int)h->open.pages.size();
    if ((rc = ensure_scan_capacity(h, std::max(np, 1)))) return rc;
    k_export_begin<<<1, 64, 0, h->stream>>>(h->d_dem, T, k);
    if ((rc = launch_scan(h, PrepArgs{}, 0, true, 0))) return rc;
    k_export_gather<<<T, 256, 0, h->stream>>>(T, k, h->d_candoff, h->d_candlen, h->d_cslot, h->d_prio, h->d_seq,
                                              h->d_cold0, h->d_cold1, d_out, d_out + (size_t)T * k * 8, d_navail,
                                              h->d_coltot, np > 0 ? 1 : 0, nullptr, 0, h->d_dem, h->d_anchor,
                                              h->d_anchor_next);
    AQ_HIP(hipGetLastError());
    return ADLBQ_OK;
}


// ---------------------------------------------------------------- group launch
// A batch that can be recorded whole: T <= 8 (the 4/8-wide kernels), a
// non-empty open bucket, no round launches after k_chain0, no diagnostics.
static bool group_eligible(const adlbq_server *h) {
    const int K = h->chain_rounds >= 0 ? h->chain_rounds : 0;
    return h->T > 0 && h->T <= 8 && !h->open.pages.empty() && K == 0 && !h->split_prep &&
           !h->chain_stamps;
}

static size_t gt_align(size_t b) { return (b + 255) & ~(size_t)255; }

// The recorded batches of handles m (same TB) as one launch per kernel on the
// first handle's stream, which first waits for every member's stream; every
// member's stream then waits for the last launch.
static int run_group(adlbq_server *const *hs, std::vector<GroupRec> &rec, const std::vector<int> &m) {
    adlbq_server *L = hs[m[0]];
    hipStream_t ls = L->stream;
    const int k = (int)m.size();
    int rc;
    if ((rc = group_join(hs, m))) return rc;
    const size_t o_thr = gt_align(sizeof(GPrep) * k), o_sel = o_thr + gt_align(sizeof(GThr) * k),
                 o_rank = o_sel + gt_align(sizeof(GSel) * k), o_chain = o_rank + gt_align(sizeof(GRank) * k),
                 o_fin = o_chain + gt_align(sizeof(GChain) * k), total = o_fin + gt_align(sizeof(GFin) * k);
    if (total > L->cap_gtab) {
        AQ_HIP(hipStreamSynchronize(ls));
        for (int sl = 0; sl < 2; sl++)
            if (L->h_gtab[sl]) AQ_HIP(hipHostFree(L->h_gtab[sl]));
        if (L->d_gtab) AQ_HIP(hipFree(L->d_gtab));
        L->cap_gtab = std::max<size_t>(total, 1 << 16);
        for (int sl = 0; sl < 2; sl++)
            AQ_HIP(hipHostMalloc((void **)&L->h_gtab[sl], L->cap_gtab, hipHostMallocDefault));
        AQ_HIP(hipMalloc((void **)&L->d_gtab, L->cap_gtab));
    }
    // pinned staging in turn: a buffer is refilled once the copy of two groups ago has run
    const int sl = L->gtab_slot;
    L->gtab_slot ^= 1;
    if (L->gtab_ev[sl]) AQ_HIP(hipEventSynchronize(L->gtab_ev[sl]));
    else AQ_HIP(hipEventCreateWithFlags(&L->gtab_ev[sl], hipEventDisableTiming));
    char *hb = L->h_gtab[sl];
    auto *tp = reinterpret_cast<GPrep *>(hb);
    auto *tt = reinterpret_cast<GThr *>(hb + o_thr);
    auto *ts = reinterpret_cast<GSel *>(hb + o_sel);
    auto *tr = reinterpret_cast<GRank *>(hb + o_rank);
    auto *tc = reinterpret_cast<GChain *>(hb + o_chain);
    auto *tf = reinterpret_cast<GFin *>(hb + o_fin);
    int gp = 0, gt = 0, gs = 0, gr = 0, gc = 0, gf = 0;
    bool all_selw = true;  // every member's pass 2 is one wave per page: k_select_wave_g
    size_t lp = 0, lsel = 0, lc = 0, lsel_o = 0;
    for (int j = 0; j < k; j++) {
        const GroupRec &r = rec[(size_t)m[(size_t)j]];
        tp[j] = r.prep;
        tt[j] = r.thr;
        ts[j] = r.sel;
        tr[j] = r.rank;
        tc[j] = r.chain;
        tf[j] = r.fin;
        if (!(r.kinds & GK_PREP)) tp[j].grid = 0;
        if (!(r.kinds & GK_THR)) tt[j].grid = 0;
        if (!(r.kinds & GK_SEL)) ts[j].grid = 0;
        if (!(r.kinds & GK_RANK)) tr[j].grid = 0;
        if (!(r.kinds & GK_CHAIN)) tc[j].grid = 0;
        if (!(r.kinds & GK_FIN)) tf[j].grid = 0;
        gp = std::max(gp, tp[j].grid);
        gt = std::max(gt, tt[j].grid);
        gs = std::max(gs, ts[j].grid);
        gr = std::max(gr, tr[j].grid);
        gc = std::max(gc, tc[j].grid);
        gf = std::max(gf, tf[j].grid);
        lp = std::max(lp, r.lds_prep);
        lsel = std::max(lsel, r.lds_sel);
        if ((r.kinds & GK_SEL) && !r.selw) all_selw = false;
        lsel_o = std::max(lsel_o, r.lds_sel_open);
        lc = std::max(lc, r.lds_chain);
    }
    char *d = L->d_gtab;
    AQ_HIP(hipMemcpyAsync(d, hb, total, hipMemcpyHostToDevice, ls));
    AQ_HIP(hipEventRecord(L->gtab_ev[sl], ls));
    const bool t4 = rec[(size_t)m[0]].tb == 4;
    if (gp) (t4 ? k_prep_hist_g<4> : k_prep_hist_g<8>)<<<dim3(gp, k), 256, lp, ls>>>(reinterpret_cast<const GPrep *>(d));
    if (gt) k_thresholds_g<<<dim3(gt, k), TH_THREADS, 0, ls>>>(reinterpret_cast<const GThr *>(d + o_thr));
    if (gs && all_selw)
        (t4 ? k_select_wave_g<4> : k_select_wave_g<8>)<<<dim3(gs, k), 64, lsel, ls>>>(reinterpret_cast<const GSel *>(d + o_sel));
    else if (gs)
        (t4 ? k_select_open_g<4> : k_select_open_g<8>)<<<dim3(gs, k), 256, lsel_o, ls>>>(
            reinterpret_cast<const GSel *>(d + o_sel));
    if (gr) k_rank_g<<<dim3(gr, k), RANK_TILE, 0, ls>>>(reinterpret_cast<const GRank *>(d + o_rank));
    if (gc) (t4 ? k_chain0_g<4> : k_chain0_g<8>)<<<dim3(gc, k), 64, lc, ls>>>(reinterpret_cast<const GChain *>(d + o_chain));
    if (gf) k_finalize_g<<<dim3(gf, k), 256, 0, ls>>>(reinterpret_cast<const GFin *>(d + o_fin));
    AQ_HIP(hipGetLastError());
    for (int j : m) rec[(size_t)j].kinds = 0;
    return group_release(hs, m);
}

// adlbq_reserve_group_device: every handle's batch recorded (or launched on its
// own stream when it cannot be), then the recorded ones grouped by TB.
int launch_group(adlbq_server *const *hs, int n, const int *const *d_reqs, int *const *d_resp, const int *counts) {
    std::vector<GroupRec> rec((size_t)n);
    std::vector<int> m4, m8;
    int rc;
    for (int i = 0; i < n; i++) {
        adlbq_server *h = hs[i];
        if (counts[i] <= 0) continue;
        const bool g = h->group_launch && group_eligible(h);
        h->grec = g ? &rec[(size_t)i] : nullptr;
        rc = launch_reserve(h, counts[i], d_reqs[i], d_resp[i]);
        h->grec = nullptr;
        if (rc) return rc;
        if (rec[(size_t)i].kinds) (rec[(size_t)i].tb == 4 ? m4 : m8).push_back(i);
    }
    for (auto *mm : {&m4, &m8}) {
        if (mm->size() == 1) rc = launch_recorded(hs[(*mm)[0]], rec[(size_t)(*mm)[0]]);
        else if (mm->size() > 1) rc = run_group(hs, rec, *mm);
        else rc = ADLBQ_OK;
        if (rc) return rc;
    }
    return ADLBQ_OK;
}
}  // namespace adlbq

extern "C" {

constexpr int RESERVE_ZC_MAX = 512;  // host-buffer batches up to this size go zero-copy

// The synchronous entry returns ADLBQ_ERR_DEVICE when k_finalize answered the
// batch ADLB_ERROR (a device-side wait gave up; nothing was pinned or parked).
static int batch_outcome(adlbq_server *h, int failed_before) {
    if (h->ctr.batch_failed != failed_before)
        return fail(ADLBQ_ERR_DEVICE, ("adlbq_reserve_batch: an in-launch candidate sort did not finish in time, "
                                       "or a choice lay outside the page list (stat bound_faults = " +
                                       std::to_string(h->ctr.bound_faults) +
                                       "); the batch was answered ADLB_ERROR and left the queues unchanged").c_str());
    return ADLBQ_OK;
}

int adlbq_reserve_batch(adlbq_server *h, int n, const int *reqs18, int *resp12) {
    if (!h || n < 0 || (n && (!reqs18 || !resp12))) return fail(ADLBQ_ERR_ARG, "adlbq_reserve_batch");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    int rc;
    if (h->ctr_stale && (rc = refresh_counters(h))) return rc;  // otherwise h->ctr is the last batch's own
    const int failed0 = h->ctr.batch_failed;
    if (n <= RESERVE_ZC_MAX) {  // a small batch: requests and replies through mapped pinned memory, no copies
        const size_t ni = (size_t)ADLBQ_RESERVE_INTS * n, no = (size_t)ADLBQ_RESP_INTS * n;
        if ((rc = ensure_zc(h, (long long)(ni + no)))) return rc;
        std::memcpy(h->h_zc, reqs18, sizeof(int) * ni);
        const long long one0 = h->one_batches;
        if ((rc = launch_reserve(h, n, h->d_zc, h->d_zc + ni))) return rc;
        // k_reserve_one: its one finishing wave stores the response, then the snapshot and last its
        // tag (system-scope release): the landed tag is the batch's end, no stream synchronisation
        if (h->one_batches == one0 || !wait_last_snapshot(h)) {
            if ((rc = sync_batch_counters(h))) return rc;  // synchronises
        }
        std::memcpy(resp12, h->h_zc + ni, sizeof(int) * no);
        return batch_outcome(h, failed0);
    }
    if ((rc = ensure_req_capacity(h, n))) return rc;
    AQ_HIP(hipMemcpyAsync(h->d_reqbuf, reqs18, sizeof(int) * ADLBQ_RESERVE_INTS * (size_t)n, hipMemcpyHostToDevice,
                          h->stream));
    if ((rc = launch_reserve(h, n, h->d_reqbuf, h->d_respbuf))) return rc;
    AQ_HIP(hipMemcpyAsync(resp12, h->d_respbuf, sizeof(int) * ADLBQ_RESP_INTS * (size_t)n, hipMemcpyDeviceToHost,
                          h->stream));
    if ((rc = sync_batch_counters(h))) return rc;
    return batch_outcome(h, failed0);
}

int adlbq_reserve_batch_device(adlbq_server *h, int n, const int *d_reqs18, int *d_resp12) {
    if (!h || n < 0 || (n && (!d_reqs18 || !d_resp12))) return fail(ADLBQ_ERR_ARG, "adlbq_reserve_batch_device");
    if (!n) return ADLBQ_OK;
    hipSetDevice(h->device);
    return launch_reserve(h, n, d_reqs18, d_resp12);
}


// One launch per pipeline kernel for the batches of n handles of one process
// (its server shards), each handle's stream ordered as if it had run its own.
int adlbq_reserve_group_device(adlbq_server *const *hs, int n, const int *const *d_reqs18, int *const *d_resp12,
                               const int *counts) {
    if (n < 0 || (n && (!hs || !d_reqs18 || !d_resp12 || !counts)))
        return fail(ADLBQ_ERR_ARG, "adlbq_reserve_group_device");
    for (int i = 0; i < n; i++) {
        if (!hs[i] || counts[i] < 0 || (counts[i] && (!d_reqs18[i] || !d_resp12[i])) ||
            hs[i]->device != hs[0]->device)
            return fail(ADLBQ_ERR_ARG, "adlbq_reserve_group_device: bad handle, count or pointer, or mixed devices");
        for (int j = 0; j < i; j++)
            if (hs[j] == hs[i]) return fail(ADLBQ_ERR_ARG, "adlbq_reserve_group_device: a handle appears twice");
    }
    if (!n) return ADLBQ_OK;
    hipSetDevice(hs[0]->device);
    return launch_group(hs, n, d_reqs18, d_resp12, counts);
}


}  // extern "C"
