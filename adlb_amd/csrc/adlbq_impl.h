// adlbq_impl.h -- internal state and device helpers of the MI355X ADLB queue engine.
//
// HBM layout (one handle = one ADLB server's queues):
//   * Work units live in fixed pages of PAGE slots.  Every page belongs to one
//     *bucket*: the open bucket (untargeted units, target_rank < 0) or the
//     bucket of one target app rank.  Within a bucket, pages are chained in
//     allocation order and slots are filled in order, so bucket order ==
//     wqseqno order (the reference's append order, xq.c:155-158).
//   * Per-slot structure of arrays: prio (i32), meta (u32: type index | LIVE |
//     PINNED), pin_rank (i32), wqseqno (i32), cold fields (2 x int4, read only
//     for matched units).  The matching scans read prio + meta = 8 B per unit;
//     type and target are implicit in (meta, bucket).
//   * Parked Reserves (rq) are indexed by rqseqno-1 (append-only, FIFO order).
#pragma once

#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <string>
#include <vector>
#include <unordered_map>

#include "adlbq.h"

struct GroupRec;  // adlbq_reserve.hip: a reserve batch's launches recorded for a group launch

namespace adlbq {

// the ordered choice (adlbq_reserve.hip): requests per segment (one wavefront)
// and the largest pass-1 warm-up replayed before a segment (T <= 8), a multiple of it
#ifndef ADLBQ_CHAIN_SEG
#define ADLBQ_CHAIN_SEG 256
#endif
#ifndef ADLBQ_CHAIN_WARM
#define ADLBQ_CHAIN_WARM 512
#endif
constexpr int SEG = ADLBQ_CHAIN_SEG;
constexpr int CHAIN_WARM = ADLBQ_CHAIN_WARM;
constexpr int PAGE_SHIFT = 12;
constexpr int PAGE = 1 << PAGE_SHIFT;       // 4096 slots per page
constexpr int SPEC_CAP = 128;              // pass-1 speculative candidates per wave quarter of a page
constexpr int NB = 64;                      // histogram bins per type (distance from anchor)
constexpr int NBX = 32;                     // bins [0, NBX) are exact (one priority value each)
constexpr int CHUNK = 8;                    // pages per prefix chunk in the open-bucket scan
constexpr int LOWEST = ADLBQ_LOWEST_PRIO;
constexpr uint32_t M_TYPE = 0xffu;
constexpr uint32_t M_LIVE = 1u << 8;
constexpr uint32_t M_PINNED = 1u << 9;
// bits 10..31: prio - page base, when the page is narrow (every unit's prio
// within 2^22 of the base): the scans then read 4 B per unit, not 8
constexpr int M_OFF_SHIFT = 10;
constexpr long long M_OFF_RANGE = 1ll << 22;
// More than ADLBQ_MAX_TYPES_WIDE (255) types (get_type_idx has no bound, adlb.c:3476-3485): such a
// server's pages are all wide (prio read from the prio column), so bits 10..31 carry the type
// index's bits above the low eight.  vw = the server has more than 255 types.
constexpr int VW_TYPES = ADLBQ_MAX_TYPES_WIDE;
__host__ __device__ __forceinline__ int meta_type(uint32_t m, int vw) {
    return (int)(m & M_TYPE) | (vw ? (int)(m >> M_OFF_SHIFT) << 8 : 0);
}
__host__ __device__ __forceinline__ uint32_t meta_of_type(int ti, int vw) {
    return vw ? ((uint32_t)ti & M_TYPE) | ((uint32_t)(ti >> 8) << M_OFF_SHIFT) : (uint32_t)ti;
}
constexpr int NREQ = ADLBQ_REQ_TYPES;
// the reference's allocation sizes (include/adlbq.h: ADLBQ_BYTES_*)
constexpr long long BYTES_WQ = ADLBQ_BYTES_WQ, BYTES_RQ = ADLBQ_BYTES_RQ, BYTES_TQ = ADLBQ_BYTES_TQ;


// device-side scalar counters shared by kernels and read back lazily by the host
struct DevCounters {
    unsigned long long fin_group[8];  // k_finalize arrivals per group: parked << 32 | workgroups
    unsigned long long fin_top;       // groups done: parked << 32 | groups (all reset by the last)
    int rq_n;          // rq slots used (slot k holds rqseqno rq_seq[k]; k_rq_reclaim compacts them)
    int rq_live;       // parked entries alive
    int rq_hwm;        // rq->max_count
    int rq_head;       // lowest rq slot that may be alive
    int n_parked_last; // parked by the last reserve batch
    int chain_rounds;  // Jacobi rounds of the last chain, all wavefronts (diagnostic)
    int chain_passes;      // segment passes of the last chain that recomputed something
    int chain_recomputed;  // segment solves over those passes
    int chain_fallback;    // segments the last chain launch's walk re-solved (0 at a fixed point)
    int chain_timeouts;    // bounded hand-off waits of round 0's neighbour passes that gave up (cumulative)
    int spec_page0;        // the last scan's page 0, wave 0 read pass 1's list (diagnostic)
    int needsort_last;     // the last reserve batch had a type whose threshold fell in a multi-prio bin
    int plan_g, plan_lo;   // the last candidate sort plan: candidates in all, lowest key bit any list varies in
    int plan_missed;       // sync-free sorts whose plan did not hold (k_rank sorted in-launch), cumulative
    int plan_phi;          // highest bit of the prio field any candidate list varies in (-1: none)
    int rank_fast;         // the last scan ranked its candidates in k_select_open (every threshold in an exact bin)
    int rank_covered;      // ... and every type had candidates (diagnostic)
    int kr_fail;           // batches whose keyrank failed over to k_rank (cumulative)
    int kr_why;            // the last keyrank failover: 1 more candidates than its buffers, 2 a bin over kr_bin_max
    int kr_maxbin;         // the largest digit bin of the last keyrank batch (diagnostic)
    int batch_failed;      // batches answered ADLB_ERROR because an in-launch candidate sort gave up (cumulative)
    int bound_faults;      // choices whose bucket position lay outside the page list (cumulative; the batch
                           // is answered ADLB_ERROR, never indexed past the list)
    int rq_next;           // rqseqnos handed out (next_rqseqno - 1, adlb.c:1244)
    int rq_reclaims;       // k_rq_reclaim compactions (cumulative)
    // the reference's curr_bytes_dmalloced / hwm_bytes_dmalloced (adlb.c:3419-3474) over the
    // structures this handle replaces, plus what the caller adds (adlbq_bytes_adjust)
    long long bytes, bytes_hwm;
    long long got, got_targeted;  // units removed by device-side Get batches (folded into the host counts)
    // diagnostic sums (stat "diag<k>"): k_reserve_small units gathered, Reserves, constant-clock
    // ticks to the sorted runs and of the serial choice, launches; k_put_match_blk staged rq
    // entries, ticks of the staging and of the matching
    long long diag[8];
    // in a batch snapshot (mapped host memory): the batch's tag, stored after every other
    // field has been written back; the host reads the snapshot once the tag matches
    unsigned long long snap_tag;
};

__device__ __forceinline__ void bytes_add(DevCounters *c, long long d) {  // one thread, in event order
    c->bytes += d;
    if (c->bytes > c->bytes_hwm) c->bytes_hwm = c->bytes;
}

struct Bucket {
    std::vector<int> pages;  // page ids in order
    int tail_fill = PAGE;    // slots used in the last page (PAGE when no page yet)
};

struct StageTimer {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    double total_ms = 0;
    long long launches = 0;
    long long host_ns = 0;  // host time spent issuing the stage (stage_begin .. stage_end)
};

}  // namespace adlbq

struct adlbq_server {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;

    int T = 0;
    std::vector<int> utypes;
    std::unordered_map<int, int> tindex;
    int A = 0, S = 1, my_idx = 0, my_world = 0, master = 0, num_world = 0;

    // ---- unit store
    int cap_pages = 0;   // allocated pages
    int n_pages = 0;     // pages handed out
    int *d_prio = nullptr;
    uint32_t *d_meta = nullptr;
    int *d_pin = nullptr;
    int *d_seq = nullptr;
    int4 *d_cold0 = nullptr;  // answer_rank, work_len, home_server_rank, common_len
    int4 *d_cold1 = nullptr;  // common_server_rank, common_seqno, user work_type, target_rank
    // [2 per slot] the fields a matched Reserve's response carries, in one 32 B
    // record: {answer_rank, work_len, wqseqno, common_len}, {common_server_rank,
    // common_seqno, user work_type, prio} (immutable after the Put)
    int4 *d_rrec = nullptr;
    adlbq::Bucket open;
    std::vector<adlbq::Bucket> rankb;     // per target app rank
    std::vector<int> bucket_ranks;        // ranks that own a bucket, in creation order
    std::unordered_map<int, int> rank_index;  // target rank -> index into rankb
    std::vector<int> rank_index_dense;        // the same for target ranks in [0, A): -1 = no bucket yet
    std::vector<int> tindex_dense;            // type value - tindex_lo -> type index (-1: undeclared), small ranges
    int tindex_lo = 0;
    bool tables_dirty = true;
    // per page id: base prio of the packed offsets, and whether some unit did not fit (wide)
    std::vector<int> page_base, page_wide;
    int *d_pbase = nullptr, *d_pwide = nullptr; int cap_pbase = 0, cap_pwide = 0; bool pinfo_dirty = true;
    int *d_open_pages = nullptr;  int cap_open_pages = 0;
    int *d_rank_pages = nullptr;  int cap_rank_pages = 0;   // CSR over bucket_ranks
    int *d_rank_pstart = nullptr; int cap_rank_pstart = 0;
    int *d_rank_fill = nullptr;   int cap_rank_fill = 0;
    int *d_bucket_ranks = nullptr; int cap_bucket_ranks = 0;
    int *d_rank2b = nullptr; int cap_rank2b = 0;            // [A] app rank -> bucket index or -1
    // per-bucket Reserve lists of a batch (prep_block appends, k_targeted_idx reads and resets)
    int *d_tcnt = nullptr; long long cap_tcnt = 0;
    int *d_tlist = nullptr; long long cap_tlist = 0;
    int tcap = 0;
    int *d_all_pages = nullptr;   int cap_all_pages = 0;    // every page, with fills
    int *d_all_fill = nullptr;    int cap_all_fill = 0;
    // the page tables above are views into d_tab, uploaded by sync_tables in one copy from
    // one of two pinned staging buffers (used in turn behind an event)
    int *d_tab = nullptr; long long cap_dtab = 0;
    int *h_tab[2] = {nullptr, nullptr}; long long cap_htab[2] = {0, 0}; hipEvent_t tab_ev[2] = {nullptr, nullptr};
    int tab_slot = 0;

    // wqseqno -> slot (host mirror for single-event calls, device copy for batches)
    int next_wqseqno = 1;
    std::vector<long long> seq2slot;  // index wqseqno
    long long *d_seq2slot = nullptr; long long cap_seq = 0;
    long long live_units = 0, max_count = 0, live_targeted = 0;
    // per type: an upper bound of the prio of every live unpinned unit, kept on
    // the device (puts and unreserves raise it; a reserve batch lowers it to
    // the live maximum its histogram saw, applied when the batch ends)
    long long *d_anchor = nullptr;
    long long *d_anchor_next = nullptr;   // [T] LLONG_MIN = no update
    // per type: the prio cut guessed for the next scan (the last reserve
    // batch's cut less a margin); pass 1 lists the units at or above it
    long long *d_gcut = nullptr;          // [T] LLONG_MAX = no guess
    long long *d_gcut_next = nullptr;     // [T] LLONG_MIN = no update
    int *d_utypes = nullptr;

    // ---- parked reserves
    int rq_cap = 0;
    int *d_rq_rank = nullptr, *d_rq_types = nullptr, *d_rq_live = nullptr, *d_rq_req = nullptr;
    int *d_rq_seq = nullptr;  // rqseqno per rq slot, ascending
    adlbq::DevCounters *d_ctr = nullptr;
    adlbq::DevCounters ctr{};      // host copy
    bool ctr_stale = false;
    long long rq_n_upper = 0;      // upper bound on rq_n while ctr is stale
    long long rq_next_upper = 0;   // ... and on rq_next
    // rq_n snapshots written by k_finalize into mapped host memory at the end of
    // each reserve batch, so the rq capacity bound tightens without a sync
    static constexpr int NSNAP = 32;  // reserve batches the host may run ahead of the device (rq bound)
    adlbq::DevCounters *h_snap = nullptr;   // [NSNAP] pinned, device-visible
    unsigned long long snap_tag[NSNAP] = {};  // the tag k_finalize stores last into that snapshot (0: unused)
    unsigned long long snap_tags = 0;          // tags handed out
    long long snap_at[NSNAP] = {};         // reserves launched up to and including that batch
    int snap_next = 0;
    adlbq::DevCounters *d_snap = nullptr;   // device address of h_snap (mapped)
    // the newest landed snapshot, looked up once per launch (hint_stamp): index or -1
    long long hint_stamp = 0, landed_stamp = -1;
    int landed_idx = -1;
    long long launched_reserves = 0;

    // ---- qmstat / donor selection
    std::vector<int> qm_hi, qm_qlen;
    std::vector<double> qm_bytes;
    int *d_qm_hi = nullptr, *d_qm_qlen = nullptr; bool qm_dirty = true;
    int *d_rfr_out = nullptr, *d_rfr_to_rank = nullptr;
    std::vector<int> tq;           // 4 ints per entry: app_rank, work_type, server_rank, num_stored
    int *d_tq = nullptr; int cap_tq = 0; bool tq_dirty = true;

    // ---- put staging
    void *d_putrec = nullptr; int *d_putout = nullptr; int cap_put = 0;

    // ---- reserve-batch scratch
    int cap_req = 0;
    unsigned long long *d_mask = nullptr;
    int *d_tmatch = nullptr, *d_umatch = nullptr;
    int2 *d_mslot = nullptr;           // [cap_req] (slot, wqseqno) the last reserve batch gave request j (-1: none)
    int2 *d_rh = nullptr;              // [cap_req] (rank, hang) of the last batch's requests (k_finalize)
    int *d_reqbuf = nullptr, *d_respbuf = nullptr;  // host-API staging
    int *d_dem = nullptr;              // [T]
    int *d_theta = nullptr;            // [T] threshold bin (-1 none)
    int *d_need = nullptr;             // [T]
    int *d_candoff = nullptr, *d_candlen = nullptr, *d_needsort = nullptr;  // [T]
    int *d_binoff = nullptr;           // [T*NB]
    unsigned int *d_coltot = nullptr;  // [T*NB] column totals (k_thresholds)
    int *d_type_cnt = nullptr;         // [T] k_thresholds arrival counters (zero between batches)
    int *d_rank_sync = nullptr;        // [ADLBQ_MAX_TYPES + 6] k_rank's in-launch sort: epochs, ticket, timeouts;
                                       // then k_chain0's rank grid barrier (arrivals, released epoch), then
                                       // k_prep_hist's folded-thresholds counters (arrivals, finished roles)
    unsigned int rank_epoch = 0;       // per reserve batch, never 0 once used
    unsigned short *d_gh = nullptr; long long cap_gh = 0;   // [open pages][T*NB]
    unsigned int *d_spec = nullptr; int *d_specn = nullptr; long long cap_spec = 0;  // [open pages][4][SPEC_CAP], [open pages][4]
    unsigned int *d_csum = nullptr; long long cap_csum = 0; // 2 x [chunks][T*NB] sums -> exclusive prefix in place
    int csum_par = 0;                  // the buffer the next scan uses
    long long csum_used[2] = {0, 0};   // entries of each buffer left to zero
    unsigned long long *d_ckey = nullptr, *d_ckey2 = nullptr; long long cap_cand = 0;
    int *d_cslot = nullptr, *d_cslot2 = nullptr;
    unsigned int *d_crank = nullptr;   // packed global rank << 6 | type, per candidate
    int *d_seg_cnt = nullptr;          // [R/64] chain: untargeted-capable requests per 64 requests
    unsigned long long *d_pmask = nullptr;  // [R/64] k_finalize: ballots of the requests that park
    int *d_lv = nullptr;               // [R][T] k_rank: level rows for the chain's guess (T <= 8)
    unsigned char *d_rtype = nullptr;
    int *d_pm_over = nullptr;          // k_put_match_blk: the staged rq overflowed
    void *h_putrec[2] = {nullptr, nullptr};     // pinned staging of Put batches' records, used in turn
    hipEvent_t put_ev[2] = {nullptr, nullptr};  // the batch that used it has finished on the device
    int put_slot = 0;  // [R] type of the candidate at each global rank (the guess between rows)
    // targeted units' sorted index (k_targeted_idx): keys/vals double buffers,
    // per (bucket, type) ranges, radix-sort scratch; rebuilt after targeted Puts
    unsigned long long *d_tkeys = nullptr, *d_tkeys2 = nullptr;
    int *d_tvals = nullptr, *d_tvals2 = nullptr; long long cap_tidx = 0;
    int *d_tstart = nullptr, *d_tend = nullptr; long long cap_trange = 0;
    long long tidx_groups = 0;  // (bucket, type) groups d_tstart / d_tend hold, as lower bounds; 0: none
    void *d_tsort = nullptr; size_t cap_tsort = 0;
    bool tindex_dirty = true;
    // incremental index: entries [0, tidx_n) of d_tkeys / d_tvals are real (sorted);
    // the keys of targeted units Put since the last build wait in tnew_*
    long long tidx_n = 0; bool tidx_valid = false;
    std::vector<unsigned long long> tnew_keys;
    std::vector<int> tnew_vals;
    unsigned long long *d_tnewk = nullptr; int *d_tnewv = nullptr; long long cap_tnew = 0;
    long long tidx_merges = 0, tidx_rebuilds = 0;
    // delta index (k_targeted_idx reads it beside the main one): the sorted keys of targeted units
    // Put since the main index was last merged or rebuilt; folded into the main index only when it
    // would grow past tdel_max ("tindex_delta", 0: every Put batch merges into the main index)
    unsigned long long *d_dkeys = nullptr, *d_dkeys2 = nullptr;
    int *d_dvals = nullptr, *d_dvals2 = nullptr; long long cap_del = 0, tdel_n = 0, tdel_max = 1 << 18;
    int *d_dstart = nullptr, *d_dend = nullptr; long long cap_drange = 0;
    long long tidx_delta_merges = 0, tidx_folds = 0;
    unsigned long long *h_tnewk[2] = {nullptr, nullptr};  // pinned staging of the sorted new keys / positions,
    int *h_tnewv[2] = {nullptr, nullptr};                 // two buffers used in turn behind their events
    long long cap_htnew[2] = {0, 0};
    hipEvent_t tnew_ev[2] = {nullptr, nullptr};
    int tnew_slot = 0;
    // segmented radix sort of the multi-prio-bin candidate lists (launched
    // when the newest landed batch needed one; k_rank sorts otherwise)
    void *d_ssort = nullptr; size_t cap_ssort = 0;  // launch_segsort
    // launch_segsort_radix: the lists copied aside (keys / slots), the plan (valid, G, lo) on the device
    unsigned long long *d_ckey3 = nullptr; int *d_cslot3 = nullptr; long long cap_c3 = 0; int *d_plan = nullptr;
    // the candidate radix sort (rsort_*): 32-bit keys + indices, ping-pong; per-(digit, tile) counts; per-list OR / AND
    unsigned int *d_rs = nullptr; long long cap_rs = 0; int *d_rs_cnt = nullptr; long long cap_rs_cnt = 0;
    unsigned int *d_rs_acc = nullptr; int rs_parity = 0;
    // zero-copy staging of the synchronous host-buffer Get batch: mapped pinned memory the
    // kernels read and write directly, and a mapped copy of the counters
    int *h_zc = nullptr, *d_zc = nullptr; long long cap_zc = 0;
    adlbq::DevCounters *h_zctr = nullptr, *d_zctr = nullptr;
    long long n_sort_radix = 0;
    long long n_segsort = 0;                          // lists given a device-wide sort (cumulative)
    long long ssort_items = 0;
    // ordered choice (k_chain0 / k_chainr): per segment start used and delta, the
    // delta prefix within its arrival group, group totals / offsets, the
    // per-request choice (next round's seed), the clean flag, arrival counters
    int *d_chS = nullptr, *d_chD = nullptr;                     // [2][nseg][T] (launch parity)
    int *d_chLP = nullptr;                                      // [nseg][T]
    int *d_chGT = nullptr, *d_chGO = nullptr;                   // [8][T]
    int *d_chclean = nullptr;
    unsigned char *d_cht = nullptr;                             // [R]
    unsigned long long *d_chcnt = nullptr;                      // [9]
    int *d_chE = nullptr, *d_chflag = nullptr;                  // round 0's hand-offs: [P][nseg][T], [P][nseg]
    unsigned int chain_epoch = 0;      // per batch, never 0 once used
    int chain_passes = 0;              // round 0's in-launch passes, 0 = auto (adlbq_set_param "chain_passes")
    int chain_rounds = -1;             // round launches after round 0, -1 = auto ("chain_rounds")
    int put_match_block = 1, put_always_match = 0;  // diagnostics ("put_match_block", "put_always_match")
    int split_prep = 0;                // diagnostic ("split_prep"): request preparation and pass 1 as two launches
    int rank_in_select = 1;            // k_select_open ranks the candidates when it can ("rank_in_select")
    int sort_fail_test = 0;            // test hook ("sort_fail_test"): the error path of a failed sort wait
    int chain_stamps = 0;              // diagnostic: phase stamps of the first chain launch ("chain_stamps")
    int kstamps = 0;                   // diagnostic ("kernel_stamps"): per-workgroup phase stamps of passes 1 and 2
    unsigned long long *d_kst = nullptr; int cap_kst = 0, n_kst = 0;
    unsigned long long *d_stamps = nullptr; int cap_stamps = 0, n_stamps = 0;
    int chain_warm = -1;               // round-0 warm-up requests (T <= 8), -1 = auto ("chain_warm")
    long long chain_modes = -1;        // bit k-1: round k uses prefix starts, -1 = auto ("chain_modes")
    unsigned long long *d_kb = nullptr;  // [2 * ADLBQ_MAX_TYPES] per-list key OR / AND (k_keybits)
    int rank_grid = 0;                 // test hook ("rank_grid"): k_rank's grid (0: 4 on a rank hint, else 1280)
    int fuse_rank_chain = 1;           // "fuse_rank_chain": k_rank's blocks in the chain's launch (T <= 8)
    int fin_snap_diag = 0;             // "fin_snap_diag" (timing diagnostic): the finalize snapshot undrained
    int targeted_scan = -1;            // "targeted_scan": 1 = the pre-targeted match scans the rank buckets
                                       //   (k_targeted), 0 = the sorted index (k_targeted_idx), -1 = by size
    long long tscan_batches = 0;       // batches whose targeted phase scanned the buckets (stat "tscan_batches")
    int unres_trust = 1;               // "unres_trust": the unreserve of the last batch's own responses, nothing
                                       //   changed since, from its (slot, wqseqno) records alone
    long long unres_trusted_calls = 0; // such unreserves (stat "unres_trusted")
    unsigned long long rank_arrivals = 0;  // rank blocks launched in k_rank_chain0 so far (their counter's target)
    int *d_jpref = nullptr;            // [cap_req / 64 + 1] exclusive prefix of seg_cnt (k_thresholds' extra workgroup)
    bool jpref_ok = false;             // this batch's k_thresholds wrote d_jpref
    bool open_all_narrow = false;      // every page of the open bucket is narrow (sync_tables)
    // dead open pages (no LIVE unit; full, never the tail): found by k_page_dead in the background
    // (flags in mapped host memory, applied once its event has passed), then reused by Puts
    std::vector<int> free_pages;
    int *h_pdead = nullptr; long long cap_pdead = 0; int pdead_np = 0; bool pdead_pending = false;
    hipEvent_t pdead_ev = nullptr; long long pdead_last = -1000000, pages_recycled = 0;
    int recycle_pages = 1;             // "recycle_pages": 0 = keep every page (the old behaviour)
    int reserve_one = 1;               // "reserve_one": a one-Reserve batch on a large open bucket in one launch
    unsigned long long *d_onepart = nullptr; int cap_onepart = 0; long long one_batches = 0;
    int one_grid = 0;                  // "one_grid": k_reserve_one's workgroups at most (0: 256)
    int select_wave = 1;               // "select_wave": pass 2 with one wave per page (T <= 8); 0 = four
    int rq_compact_calls = 0; long long rq_compactions = 0;  // background rq compaction (maybe_compact_rq)
    long long rq_reclaims_launched = 0;  // k_rq_reclaim launches (DevCounters::rq_reclaims counts the landed ones)
    int small_pages = 4;               // "small_pages": an open bucket of at most this many pages and a batch of
    int small_r = 1024;                //   at most "small_r" Reserves take the one-workgroup choice (0: never)
    int bound_inject = 0;              // "bound_inject" (test only): the next small / one-Reserve choice is told a
                                       //   position past the page list (the fault path of DESIGN.md §9)
    long long small_batches = 0;       // reserve batches served by it (stat "small_batches")
    // the Reserve path of more than ADLBQ_MAX_TYPES types (adlbq_wide.hip): sort buffers and runs
    unsigned long long *d_wk0 = nullptr, *d_wk1 = nullptr, *d_wekey = nullptr;
    int *d_wv0 = nullptr, *d_wv1 = nullptr, *d_wflag = nullptr, *d_wrstart = nullptr, *d_whead = nullptr;
    unsigned long long *d_wrkey = nullptr;  // run keys: (target rank or A) << type bits | type index
    int2 *d_utsorted = nullptr; int n_utsorted = 0;  // > 255 types: (value, first declared index) by value
    int *d_wreq = nullptr, *d_wcnt = nullptr;
    int2 *d_wpages = nullptr;
    void *d_wtmp = nullptr;
    long long cap_wn = 0;
    size_t cap_wtmp = 0;
    int cap_wreq = 0, cap_wpages = 0;
    int group_launch = 1;              // "group_launch": 0 = adlbq_reserve_group_device launches this handle alone
    const int *last_reqs = nullptr;    // the last batch's request array and size (its d_rh rows describe it)
    int last_R = 0;
    // mut_epoch: bumped by every queue change (wq_changed) and reserve launch; mslot_epoch: its value when
    // the last batch that wrote d_mslot was launched (the unreserve of that batch's own responses is then
    // exact from d_mslot alone: adlbq_unreserve_resp_device)
    unsigned long long mut_epoch = 0, mslot_epoch = ~0ull;
    int fin_flat = 512;                // "fin_flat": k_finalize grids up to this size arrive at one counter
    ::GroupRec *grec = nullptr;        // non-null: launch_reserve records its launches (adlbq_reserve_group_device)
    // the group launch's argument tables (kept by the group's first handle): pinned staging x 2, device copy
    char *h_gtab[2] = {nullptr, nullptr};
    hipEvent_t gtab_ev[2] = {nullptr, nullptr};
    char *d_gtab = nullptr;
    size_t cap_gtab = 0;
    int gtab_slot = 0;
    std::vector<hipEvent_t> gjoin;     // one per grouped handle: its stream joins the launch stream
    // keyrank (adlbq_keyrank.hip): 8 < T <= 64, the candidates binned and ranked in one global order
    char *d_kr = nullptr; long long cap_kr = 0;
    int keyrank = 1;                   // "keyrank": 0 = the per-list sort + k_rank
    int kr_bin_max = 1024;             // "keyrank_bin_max": a larger digit bin fails the batch over to k_rank
    long long n_keyrank = 0, kr_fail_seen = 0, kr_skip_until = 0;
    int rq_wait_sync = 1;              // "rq_wait_sync": rq backpressure by stream sync (0: spin on the oldest snapshot, measured slower)
    int targeted_diag = 0;             // diagnostic ("targeted_diag"): parts of k_targeted_idx skipped (1, 2, 4: wrong
                                       //   results); 8: 64 Reserves of a bucket at a time by Jacobi rounds (A/B, exact)
    int kr_par = 0;                    // parity of keyrank's chunk-count rows
    // ---- steal round (adlbq_steal.hip): device export + pinned host mirror
    int *d_export = nullptr; long long cap_export = 0;   // [T*k*8 recs | T nrec]
    long long *d_navail = nullptr;                       // [T]
    int *d_rqx = nullptr; long long cap_rqx = 0;         // [1 count | cap*18 rq entries]
    int *h_steal = nullptr; long long cap_hsteal = 0;    // pinned: recs | nrec | navail (2T) | count | rq
    int steal_k = -1, steal_rqcap = 0;                   // shape of the export in flight (-1: none)
    // a steal group's shard (adlbq_steal_group_create): each reserve batch lists export_extra
    // candidates per type beyond its demand, so that an export right after it is a gather
    // (k_export_after) instead of another scan; batch_export_k = that depth while nothing
    // else has changed the wq since the batch (0: the export scans)
    int export_extra = 0, batch_export_k = 0, batch_export_R = 0;
    hipEvent_t steal_ev = nullptr;
    int *h_apply = nullptr; long long cap_happly = 0;    // pinned staging of grants / deletions
    int *d_apply = nullptr; long long cap_dapply = 0;
    int *d_apply_bad = nullptr;                          // [2] grants not available, deletions not parked
    hipEvent_t apply_ev = nullptr;
    int *d_result = nullptr;           // small result scratch (16 ints)
    int *d_getclaim = nullptr; long long cap_getclaim = 0;  // [wqseqno] lowest claiming Get of a batch (INT_MAX: none)
    int *d_getbuf = nullptr; long long cap_getbuf = 0;      // host-buffer Get batches: pairs, then results
    long long got_seen = 0, got_t_seen = 0;                 // the device Get counters already folded in
    int *d_info = nullptr;                                  // fused info reduction: per-block partials + counter
    int *d_crem = nullptr, *h_crem = nullptr; long long cap_crem = 0;  // check_remote results (device, pinned)
    int *h_result = nullptr;           // pinned host mirror
    long long last_scan_units = 0;

    bool profiling = false;
    int profile_every = 1;                    // stage events on every n-th reserve batch only ("profile_every")
    long long reserve_batches = 0;            // reserve batches launched
    std::string profile_only;                 // empty: every stage
    std::vector<hipEvent_t> event_pool;
    std::unordered_map<std::string, adlbq::StageTimer> timers;
    std::unordered_map<std::string, long long> hacc;  // always-on host section time, ns ("hacc:<name>")
    std::chrono::steady_clock::time_point stage_host_t0;
};

namespace adlbq {

int fail(int code, const char *msg);
int hip_fail(hipError_t e, const char *where);
#define AQ_HIP(call)                                     \
    do {                                                 \
        hipError_t _e = (call);                          \
        if (_e != hipSuccess) return adlbq::hip_fail(_e, #call); \
    } while (0)

int ensure_req_capacity(adlbq_server *h, int n);
int sync_tables(adlbq_server *h);          // page tables, anchors, qmstat, tq -> device
void recycle_apply(adlbq_server *h);       // drop the dead open pages a finished k_page_dead found
int recycle_launch(adlbq_server *h);       // look for dead open pages in the background (when worth it)
void maybe_compact_rq(adlbq_server *h);    // compact a thinned-out rq in the background
int ensure_zc(adlbq_server *h, long long n);  // mapped pinned staging of >= n ints (h_zc / d_zc)
int refresh_counters(adlbq_server *h);     // d_ctr -> ctr (synchronises)
bool wait_last_snapshot(adlbq_server *h);  // spin until the last batch's snapshot lands (no HIP call)
void tighten_rq_bound(adlbq_server *h, bool wait_oldest);
long long rq_live_upper(adlbq_server *h);
bool rank_hint(adlbq_server *h);  // newest landed batch ranked in k_select_open (no sync)
bool plan_hint(adlbq_server *h, int *g, int *lo, int *phi = nullptr);
inline void wq_changed(adlbq_server *h) {
    h->batch_export_k = 0;
    h->mut_epoch++;
}  // the last batch's lists no longer describe the wq  // newest landed batch's candidate sort plan
bool sort_hint(adlbq_server *h);  // parked Reserves alive, upper bound (no sync)  // newest landed batch snapshot -> rq_n_upper
int ensure_rq_capacity(adlbq_server *h, int extra);
void stage_begin(adlbq_server *h, const char *name, hipEvent_t *ev);
void stage_end(adlbq_server *h, const char *name, hipEvent_t ev);
// host time since t0 added to stage `name` (profiling only; no events)
void host_stage_add(adlbq_server *h, const char *name, std::chrono::steady_clock::time_point t0);
int launch_reserve(adlbq_server *h, int n, const int *d_reqs, int *d_resp);
int sync_batch_counters(adlbq_server *h);  // synchronise; h->ctr from the last batch's landed snapshot
int wide_choose(adlbq_server *h, int R, const int *d_reqs);
int launch_keyrank(adlbq_server *h, int R);  // 8 < T <= 64: lists sorted and ranked (k_kr_*)
bool keyrank_hint(adlbq_server *h);         // no failed keyrank landed recently  // T > ADLBQ_MAX_TYPES: the batch's choices
int launch_unreserve_resp(adlbq_server *h, int n, const int *d_reqs18, const int *d_resp12, int trusted);  // k_unreserve_resp
int group_join(adlbq_server *const *hs, const std::vector<int> &m);     // hs[m[0]]'s stream waits for the members'
int group_release(adlbq_server *const *hs, const std::vector<int> &m);  // the members' streams wait for hs[m[0]]'s
int launch_export(adlbq_server *h, int k, int *d_out, long long *d_navail);
bool launch_export_after(adlbq_server *h, int k, int *d_recs, int *d_nrec, long long *d_navail);
// the grouped form (adlbq_steal_group_export): one shard's k_export_after arguments, when its last
// batch's lists serve an export of depth k; EXPORT_GROUP shards per launch, kernel arguments
struct ExportAfterArgs {
    int T, k, R;
    const unsigned char *cht;
    const int *candoff, *candlen, *cslot, *prio, *seqa;
    const int4 *cold0, *cold1;
    int *recs, *nrec;
    long long *navail;
    const unsigned int *coltot;
};
constexpr int EXPORT_GROUP = 16;
struct ExportAfterGroup {
    ExportAfterArgs a[EXPORT_GROUP];
};
bool export_after_args(adlbq_server *h, int k, int *d_recs, int *d_nrec, long long *d_navail, ExportAfterArgs *a);
int launch_export_after_group(const ExportAfterGroup &g, int n, int k, int Tmax, hipStream_t s);

// ---------------------------------------------------------------- device helpers
// SS_UNRESERVE of every unit a reserve batch handed out (k_unreserve_resp, and
// the unreserve workgroups of a fused adlbq_unreserve_reserve_device launch)
__device__ __forceinline__ void unreserve_resp_body(const int *__restrict__ reqs, const int *__restrict__ resp, int n,
                                                    const long long *__restrict__ seq2slot, long long nseq,
                                                    uint32_t *meta, int *pin, const int4 *__restrict__ rrec,
                                                    long long *anchor, const int2 *__restrict__ mslot, int ntypes,
                                                    int bid, const int2 *__restrict__ rh, bool trusted) {
    int i = bid * blockDim.x + threadIdx.x;
    if (trusted) {
        // nothing changed the queue since the batch that wrote mslot (these requests'): its record is the
        // unit's slot and wqseqno, the unit is still live and pinned to the request's rank, and its
        // priority is at most the anchor (that batch's k_thresholds bound every unit its scan saw, the
        // chosen ones included; a small batch leaves the anchor as it was, a one-Reserve batch lowers it
        // to the best priority it saw, at least the chosen unit's) -- no gather of meta / pin / record
        // and no anchor update
        if (i < n) {
            const int rc = resp[(long long)ADLBQ_RESP_INTS * i], seq = resp[(long long)ADLBQ_RESP_INTS * i + 5];
            const int2 ms = mslot[i];
            if (rc == 1 && ms.x >= 0 && ms.y == seq) {
                pin[ms.x] = -1;
                __hip_atomic_fetch_and(meta + ms.x, ~(uint32_t)M_PINNED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return;
    }
    int t = -1, up = INT_MIN;
    // lane u holds anchor[u] (T <= 64), loaded with the responses: only a unit above it needs an
    // atomic max (one per type of the wave; every wave adding to one word would serialise them)
    const long long my_anchor = __lane_id() < ntypes ? __hip_atomic_load(anchor + __lane_id(), __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT) : LLONG_MAX;
    if (i < n) {
        const int rc = resp[(long long)ADLBQ_RESP_INTS * i], seq = resp[(long long)ADLBQ_RESP_INTS * i + 5];
        // the last batch's own requests: (rank, hang) compacted by its prep (8 B instead of a 72 B stride)
        const int rank = rh != nullptr ? rh[i].x : reqs[(long long)ADLBQ_RESERVE_INTS * i];
        const int ms = mslot != nullptr ? mslot[i].x : -1;
        if (rc == 1 && seq > 0 && seq < nseq) {
            long long slot = ms;
            uint32_t m = 0;
            int pn = 0;
            int4 r0 = make_int4(0, 0, 0, 0), r1 = r0;
            if (slot >= 0) {
                m = meta[slot];
                pn = pin[slot];
                r0 = rrec[2 * slot];
                r1 = rrec[2 * slot + 1];
            }
            if (slot < 0 || r0.z != seq) {  // not the last batch's record: the map
                slot = seq2slot[seq];
                if (slot >= 0) {
                    m = meta[slot];
                    pn = pin[slot];
                    r0 = rrec[2 * slot];
                    r1 = rrec[2 * slot + 1];
                }
            }
            if (slot >= 0 && (m & M_LIVE) && pn == rank && r0.z == seq) {
                pin[slot] = -1;
                meta[slot] = m & ~M_PINNED;
                t = m & M_TYPE;
                up = r1.w;
            }
        }
    }
    // available again: keep the anchor above it, one atomic max per distinct type of the wave that rose
    const long long at = __shfl(my_anchor, t >= 0 ? t : 0, 64);
    if (t >= 0 && (long long)up <= at) t = -1;
    for (unsigned long long b = __ballot(t >= 0); b;) {
        const int leader = __ffsll((long long)b) - 1;
        const int lt = __shfl(t, leader, 64);
        int mx = t == lt ? up : INT_MIN;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
        if (__lane_id() == leader) atomicMax(anchor + lt, (long long)mx);
        b &= ~__ballot(t == lt);
    }
}


__device__ __forceinline__ unsigned long long make_key(int prio, unsigned int order) {
    // larger key == better: priority descending, then `order` ascending
    return ((unsigned long long)((unsigned int)prio ^ 0x80000000u) << 32) |
           (unsigned long long)(~order);
}

// Keep anchor[t] >= prio.  Most calls do not raise it, so the anchor is read
// first; the lanes of a wave that do raise it agree on one atomic per type
// (a single device-scope word per type would otherwise serialise them).
// Every lane of the wave must call it (INT_MIN: nothing to raise).
__device__ __forceinline__ void raise_anchor(long long *anchor, int t, int prio) {
    bool up = __hip_atomic_load(anchor + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (long long)prio;
    while (true) {
        const unsigned long long b = __ballot(up);
        if (!b) break;
        const int leader = __ffsll((long long)b) - 1;
        const int lt = __shfl(t, leader, 64);
        int m = (up && t == lt) ? prio : INT_MIN;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
        if (__lane_id() == leader) atomicMax(anchor + lt, (long long)m);
        if (t == lt) up = false;
    }
}

// SS_UNRESERVE of triple i (rank, wqseqno, new pin) (adlb.c:2057-2063): a unit
// still live, pinned for that rank and with that wqseqno goes back to the
// queue.  Every lane of the wave calls it (raise_anchor).
__device__ __forceinline__ void unreserve_triple(int i, const int *__restrict__ trip, int n,
                                                 const long long *__restrict__ seq2slot, long long nseq,
                                                 uint32_t *meta, int *pin, const int4 *__restrict__ rrec,
                                                 long long *anchor) {
    int t = 0, up = INT_MIN;
    if (i < n) {
        int rank = trip[3 * i], seq = trip[3 * i + 1], np = trip[3 * i + 2];
        long long slot = (seq > 0 && seq < nseq) ? seq2slot[seq] : -1;
        if (slot >= 0) {
            // meta, pin and the slot's response record (wqseqno, prio) in one round trip
            const uint32_t m = meta[slot];
            const int pn = pin[slot];
            const int4 r0 = rrec[2 * slot], r1 = rrec[2 * slot + 1];
            if ((m & M_LIVE) && pn == rank && r0.z == seq) {
                pin[slot] = np;
                meta[slot] = m & ~M_PINNED;
                t = m & M_TYPE;
                up = r1.w;
            }
        }
    }
    raise_anchor(anchor, t, up);  // available again: keep the anchor above it
}

// The rq slot holding rqseqno (-1: none).  rq_seq is ascending over the
// slots in use: FIFO order is rqseqno order, and k_rq_reclaim keeps it.
__device__ __forceinline__ int rq_slot_of(const int *rq_seq, int n, int rqseqno) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (rq_seq[mid] < rqseqno) lo = mid + 1;
        else hi = mid;
    }
    return (lo < n && rq_seq[lo] == rqseqno) ? lo : -1;
}

// Histogram bins of a distance d = anchor - prio: [0, NBX) exact (one
// priority each), then NBH half-octave bins up to 2^(5 + NBH/2), then octaves;
// the last bin (NB - 1) is unbounded.  A threshold in a multi-priority bin
// takes the whole bin into the candidate list (sorted later), so the finer
// bins where thresholds usually fall keep that overshoot at most 50%.
constexpr int NBH = 24;
constexpr int OCT_H = 5 + NBH / 2;  // first octave with a single bin
__device__ __forceinline__ int bin_of(long long d) {
    if (d < NBX) return (int)d;
    const int o = 63 - __clzll((unsigned long long)d);  // >= 5
    const int b = o < OCT_H ? NBX + 2 * (o - 5) + (int)((d >> (o - 1)) & 1) : NBX + NBH + (o - OCT_H);
    return b < NB ? b : NB - 1;
}

// bin_of for a distance known to fit 32 bits (an int anchor less an int prio),
// branch-free (selects only: it runs once per unit in pass 1)
__device__ __forceinline__ int bin_of32(unsigned int d) {
    const int o = 31 - __clz((int)(d | 32u));  // >= 5
    const int bh = NBX + 2 * (o - 5) + (int)((d >> (o - 1)) & 1u), bo = NBX + NBH + (o - OCT_H);
    const int b = min(o < OCT_H ? bh : bo, NB - 1);
    return d < (unsigned int)NBX ? (int)d : b;
}

// the smallest distance bin b holds, and the largest (NB - 1: unbounded)
__host__ __device__ __forceinline__ long long bin_lo(int b) {
    if (b < NBX) return b;
    const int k = b - NBX;
    if (k < NBH) return (long long)(2 + (k & 1)) << (5 + k / 2 - 1);
    return 1ll << (OCT_H + (k - NBH));
}
__host__ __device__ __forceinline__ long long bin_hi(int b) {
    return b >= NB - 1 ? (1ll << 40) : bin_lo(b + 1) - 1;
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
    unsigned int lane = __lane_id();
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

}  // namespace adlbq
