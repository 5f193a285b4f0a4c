/*
 * adlbq.h -- C ABI of the MI355X-native ADLB server work-queue engine.
 *
 * One opaque handle = the queue state of one ADLB server rank: its work queue
 * (wq), its parked Reserves (rq), its targeted-remote index (tq), its copy of
 * the qmstat status table and the RFR throttling state.  The matching itself
 * runs as HIP kernels on gfx950 over a structure-of-arrays store in HBM; the
 * caller (the C server loop in the reference's src/adlb.c, ADLBP_Server) keeps
 * the MPI wire protocol and payload buffers and calls these entry points at the
 * sites listed per function.  See INTEGRATION.md for the call-site patch.
 *
 * Conventions
 *   - return value: ADLBQ_OK (0) or a negative ADLBQ_ERR_* code;
 *   - no ownership of caller buffers; host pointers unless a name says _device;
 *   - one caller thread per handle; calls are synchronous on return except
 *     the _device variants, which are ordered on the handle's HIP stream;
 *   - ranks are MPI world ranks exactly as in the reference (apps are
 *     [0, num_app_ranks), servers follow: adlb.c:246-258, no debug server).
 *
 * Results are bit-identical to processing the same events one at a time
 * through the reference handlers (tests/test_gpu_parity.py).
 */
#ifndef ADLBQ_H
#define ADLBQ_H

#ifdef __cplusplus
extern "C" {
#endif

#define ADLBQ_OK                 0
#define ADLBQ_ERR_ARG           -1   /* bad argument / handle */
#define ADLBQ_ERR_HIP           -2   /* HIP runtime failure (message via adlbq_last_error) */
#define ADLBQ_ERR_NOMEM         -3
#define ADLBQ_ERR_TYPE          -4   /* work type not declared at create (ADLBP_Put aborts: adlb.c:2762) */
#define ADLBQ_ERR_UNSUPPORTED   -5   /* e.g. more than ADLBQ_MAX_TYPES_VWIDE types, or a steal export over 64 */
#define ADLBQ_ERR_DEVICE        -6   /* a device-side wait gave up: the batch was answered ADLB_ERROR
                                        (-1 in word 0 of every reply), nothing pinned or parked */

#define ADLBQ_MAX_TYPES          64  /* request type sets are 64-bit masks on the device */
#define ADLBQ_MAX_TYPES_WIDE    255  /* more types than 64: a correct, slower Reserve path (adlbq_wide.hip) */
#define ADLBQ_MAX_TYPES_VWIDE  (1 << 22) /* more than 255: the same path, every page wide (type index bits in meta) */
#define ADLBQ_REQ_TYPES          16  /* REQ_TYPE_VECT_SZ, src/xq.h:37 */
#define ADLBQ_RESP_INTS          12  /* TA_RESERVE_RESP int[12], src/adlb.c:1213-1222 */
#define ADLBQ_PUT_INTS            9
#define ADLBQ_RESERVE_INTS       18
#define ADLBQ_LOWEST_PRIO  (-999999999) /* ADLB_LOWEST_PRIO, include/adlb/adlb.h:22 */

typedef struct adlbq_server adlbq_server;

/* Replaces the per-server queue setup of ADLBP_Init (src/adlb.c:295-320:
 * wq/rq/iq/tq/cq = xq_create(), qmstat_tbl rows = LOWEST, next_wqseqno = 1,
 * next_rqseqno = 1, rfr_to_rank = -1, rfr_out = 0).  max_units is a sizing hint
 * for HBM (the store grows on demand).  device = HIP device ordinal, or -1
 * for my_server_idx modulo the visible devices. */
int adlbq_create(adlbq_server **out, int ntypes, const int *user_types, int num_app_ranks,
                 int num_servers, int my_server_idx, long long max_units, int device);
int adlbq_destroy(adlbq_server *h);

/* FA_PUT_HDR after the payload arrived, for n Puts in arrival order
 * (src/adlb.c:963-1046: wq_node_create(next_wqseqno++) + wq_append, then
 * rq_find_rank_queued_for_type(target_rank, work_type) and pin on a hit).
 * units9[i] = {work_type, work_prio, answer_rank, target_rank, work_len,
 *              home_server_rank, common_len, common_server_rank, common_seqno}
 * (the FA_PUT_HDR info_buf fields, adlb.c:903-970).
 * out3[i]   = {wqseqno, matched_rank or -1, matched_rqseqno or -1}; on a match
 * the caller sends TA_RESERVE_RESP to matched_rank (adlb.c:996-1008). */
int adlbq_put_batch(adlbq_server *h, int n, const int *units9, int *out3);
/* The same with out3 in device memory: nothing waits for the device (a
 * GPU-resident front end reads the matches from d_out3 in stream order). */
int adlbq_put_batch_device(adlbq_server *h, int n, const int *units9, int *d_out3);

/* n FA_RESERVE messages in arrival order (src/adlb.c:1199-1317): for each,
 * wq_find_pre_targeted_hi_prio(rank) then wq_find_hi_prio (xq.c:190-247), pin
 * on a hit; otherwise park on rq (hang) with the RFR donor choice of
 * find_cand_rank_with_worktype (adlb.c:1278-1309, 3487-3534), or NO_CURR_WORK.
 * reqs18[i]  = {from_rank, hang_flag, req_types[16]}  (FA_RESERVE's int[17]
 *              buffer, adlb.c:2903-2923, prefixed with the sender rank).
 * resp12[i]  = TA_RESERVE_RESP {rc, type, prio, len, answer_rank, wqseqno,
 *              server_rank, common_len, common_server, common_seqno} with
 *              rc = 1 (SUCCESS) / -2 (NO_CURR_WORK) / 0 (parked), and
 *              [10] = rqseqno if parked, [11] = server rank an SS_RFR goes to
 *              (-1 if none).
 * ADLBQ_ERR_DEVICE (never a silent wrong match): a device-side wait of the
 * batch gave up; every reply is ADLB_ERROR and the queues are unchanged.  The
 * _device variant writes the same replies (stat "batch_failed" counts them). */
int adlbq_reserve_batch(adlbq_server *h, int n, const int *reqs18, int *resp12);

/* Same, with reqs18/resp12 in device memory, enqueued on the handle's stream
 * (no host synchronisation).  Used when requests are staged in HBM. */
int adlbq_reserve_batch_device(adlbq_server *h, int n, const int *d_reqs18, int *d_resp12);

/* adlbq_reserve_batch_device for the local server shards of one process
 * (handles hs[0..n), distinct, one device; counts[i] Reserves for hs[i]), as
 * ONE launch per pipeline kernel over all of them (grid.y = shard) on hs[0]'s
 * stream, which first waits for every shard's stream; every shard's stream
 * then waits for the last launch.  Results are those of n separate
 * adlbq_reserve_batch_device calls.  A shard whose batch needs an extra launch
 * in between (targeted units, a read-back sort) or with T > 8 runs alone on
 * its stream.  The reference serves each server's Reserves in its own process
 * (src/adlb.c:1181-1320); this entry is the multi-shard-per-GPU form of it. */
int adlbq_reserve_group_device(adlbq_server *const *hs, int n, const int *const *d_reqs18, int *const *d_resp12,
                               const int *counts);

/* FA_GET_RESERVED (src/adlb.c:1347-1381): wq_find_pinned_for_rank(rank, wqseqno)
 * (xq.c:249-264) then wq_delete.  out5 = {rc (1 / -1 not found), work_len,
 * work_type, work_prio, answer_rank}. */
int adlbq_get_reserved(adlbq_server *h, int rank, int wqseqno, int *out5);

/* n FA_GET_RESERVEDs in arrival order (one kernel pair, one synchronisation):
 * pairs2[i] = {rank, wqseqno}; out5[i] as adlbq_get_reserved.  A unit can be
 * got once: of several valid Gets of one wqseqno the first wins, as in the
 * sequential server loop. */
int adlbq_get_reserved_batch(adlbq_server *h, int n, const int *pairs2, int *out5);
/* The same with device-resident pairs2 / out5, enqueued without a host
 * synchronisation (the host's unit counts catch up at the next counter read). */
int adlbq_get_reserved_batch_device(adlbq_server *h, int n, const int *d_pairs2, int *d_out5);

/* SS_UNRESERVE (src/adlb.c:2057-2063): pin_rank = new_pin_rank, pinned = 0. */
int adlbq_unreserve(adlbq_server *h, int rank, int wqseqno, int new_pin_rank, int *found);

/* n SS_UNRESERVEs with device-resident (rank, wqseqno, new_pin) triples. */
int adlbq_unreserve_batch_device(adlbq_server *h, int n, const int *d_triples);

/* SS_UNRESERVE (src/adlb.c:2051-2070) of every unit a reserve batch handed
 * out, taken straight from that batch's device-resident reqs18 / resp12 (rows
 * with rc 1): pin_rank = -1, pinned = 0.  Enqueued on the handle's stream.
 * When d_reqs18 / n are the last reserve batch's own and no call has changed
 * the queue since, each row is checked against that batch's record of what it
 * gave (slot, wqseqno) and the unit is released without a lookup; the request
 * rows must then still hold what the batch read (the caller's buffer is not
 * rewritten in between). */
int adlbq_unreserve_resp_device(adlbq_server *h, int n, const int *d_reqs18, const int *d_resp12);

/* adlbq_unreserve_resp_device for several handles of one process (distinct,
 * one device; counts[i] responses of hs[i]) as one launch on hs[0]'s stream,
 * ordered like adlbq_reserve_group_device. */
int adlbq_unreserve_resp_group_device(adlbq_server *const *hs, int n, const int *const *d_reqs18,
                                      const int *const *d_resp12, const int *counts);

/* update_local_state (src/adlb.c:3581-3593): qlen = wq_get_num_unpinned_untargeted
 * (xq.c:298-311), type_hi_prio[t] = wq_get_avail_hi_prio_of_type(user_types[t])
 * (xq.c:313-329); also stored as this server's qmstat row. */
int adlbq_qmstat_row(adlbq_server *h, int *qlen, int *type_hi_prio);

/* The SS_QMSTAT ring hop's unpack of another server's row (adlb.c:1716-1728). */
int adlbq_set_qmstat_row(adlbq_server *h, int server_idx, int qlen, double nbytes_used,
                         const int *type_hi_prio);

/* SS_PUSH_QUERY_RESP's update of the pushee's nbytes_used alone (adlb.c:2168-2169). */
int adlbq_set_qmstat_nbytes(adlbq_server *h, int server_idx, double nbytes_used);

/* check_remote_work_for_queued_apps (src/adlb.c:3536-3579): for each parked
 * Reserve in FIFO order without an outstanding RFR, the first type with a donor
 * (tq_find_first_rt, else qmstat argmax) gets an SS_RFR.  out3[k] = {rqseqno,
 * for_rank, donor_server_rank}; *count = k (at most cap). */
int adlbq_check_remote(adlbq_server *h, int cap, int *out3, int *count);

/* SS_RFR_RESP bookkeeping (src/adlb.c:1877-1878). */
int adlbq_rfr_done(adlbq_server *h, int from_server_rank, int for_rank);
/* The same for n SS_RFRs at once, pairs[2k] = from_server_rank, pairs[2k+1] =
 * for_rank, applied in order by one launch per 32 pairs (a steal group's server
 * clears the records of every SS_RFR it leaves to the next round together). */
int adlbq_rfr_done_batch(adlbq_server *h, int n, const int *pairs);

/* FA_DID_PUT_AT_REMOTE's tq update (src/adlb.c:1167-1178); the caller then
 * runs adlbq_check_remote like adlb.c:1179. */
int adlbq_tq_add(adlbq_server *h, int app_rank, int work_type, int server_rank);

/* Remove a parked Reserve by rqseqno (rq_find_seqno + rq_delete, adlb.c:1883-1933). */
int adlbq_rq_delete(adlbq_server *h, int rqseqno, int *found);

/* tq_find_rtr + num_stored-- (delete at 0): SS_RFR_RESP for a targeted unit
 * (adlb.c:1935-1947) and SS_MOVING_TARGETED_WORK (2077-2084). */
int adlbq_tq_dec(adlbq_server *h, int app_rank, int work_type, int server_rank);

/* SS_RFR_RESP failure (adlb.c:1971-2005): the donor's qmstat row gets
 * type_hi_prio = LOWEST for every type of the request (a wildcard first entry
 * = every declared type) and each tq record (for_rank, donor, type) loses one
 * unit.  types16 = the request's req_types as the SS_RFR_RESP echoes them. */
int adlbq_rfr_failed(adlbq_server *h, int donor_rank, int for_rank, const int *types16);

/* The retry that follows (adlb.c:2007-2041): if rqseqno is still parked
 * (*found = 1), its first type with a donor gets a new SS_RFR: *donor_rank =
 * that server (rfr_to_rank / rfr_out set) or -1. */
int adlbq_rfr_retry(adlbq_server *h, int rqseqno, int *found, int *donor_rank);

/* target_rank of a live unit (kept through a pin): the prev_target field of the
 * donor's SS_RFR_RESP (adlb.c:1824, 1837).  ADLBQ_ERR_ARG if no such unit. */
int adlbq_unit_target(adlbq_server *h, int wqseqno, int *target_rank);

/* ---- steal round: replaces the SS_RFR / SS_RFR_RESP round
 * trips (adlb.c:1280-1308, 1802-1933, 3536-3579) between co-resident servers
 * by one export + all-gather + deterministic merge (adlb_amd/shards.py). */

/* The donor side of SS_RFR for every possible request at once: per work type
 * (user_types order), the k >= 1 best available units -- unpinned,
 * untargeted, prio > ADLB_LOWEST_PRIO -- in wq_find_hi_prio preference order
 * (prio desc, wqseqno asc; xq.c:190-217).  recs8[t][i] = {work_prio, wqseqno,
 * work_type, work_len, answer_rank, common_len, common_server_rank,
 * common_seqno} (the SS_RFR_RESP fields, adlb.c:1828-1840); nrec[t] = records
 * written (<= k); navail[t] = available units of type t in all. */
int adlbq_steal_export(adlbq_server *h, int k, int *recs8, int *nrec, long long *navail);

/* A steal round answers every SS_RFR this shard's parks sent (resp[11]):
 * _begin clears rfr_to_rank / rfr_out as each SS_RFR_RESP would
 * (adlb.c:1877-1878).
 * The same export split in two so that many handles (shards on one GPU) scan
 * concurrently: _begin enqueues the scan, the rq compaction and the copies to
 * pinned host memory on the handle's stream; _collect waits and hands out the
 * top-k records (any of recs8 / nrec / navail may be NULL) and the live rq
 * entries as adlbq_rq_export does (out18 up to cap, *count = all live). */
int adlbq_steal_begin(adlbq_server *h, int k);
int adlbq_steal_collect(adlbq_server *h, int *recs8, int *nrec, long long *navail, int cap, int *out18,
                        int *count);

/* The live rq in FIFO (rqseqno) order: out18[i] = {rqseqno, world_rank,
 * req_types[16]} (rq_struct_t, xq.h:79-86).  *count = live entries (only
 * min(count, cap) are written). */
int adlbq_rq_export(adlbq_server *h, int cap, int *out18, int *count);

/* The serialised steal round over S shards (pure host function, same result
 * on every caller).  recs8 [S][T][k][8], nrec [S][T], navail [S][T]: every
 * shard's adlbq_steal_export.  reqs19[r] = {shard_idx, rqseqno, world_rank,
 * req_types[16]} in (shard_idx, rqseqno) order.  For each request in that
 * order: donor = find_cand_rank_with_worktype over the current heads
 * (adlb.c:1280-1308, 3487-3534), unit = the donor's wq_find_hi_prio over the
 * request's types (adlb.c:1816-1818).  out3[r] = {donor shard_idx, type
 * index, record index} or {-1, -1, -1}.  *n_decided = requests settled
 * before the first one that needs a unit past some shard's exported k; it
 * and all later requests get -1 (they stay parked). */
int adlbq_steal_merge(int S, int T, const int *user_types, int k, const int *recs8, const int *nrec,
                      const long long *navail, int nreq, const int *reqs19, int *out3, int *n_decided);

/* Donor side of a granted steal (adlb.c:1820-1824): pin_rank = rank,
 * pinned = (rank >= 0).  pairs2[i] = {rank, wqseqno}; found[i] = 0 if that
 * unit is no longer live, unpinned and untargeted. */
int adlbq_grant_batch(adlbq_server *h, int n, const int *pairs2, int *found);

/* Requester side: rq_find_seqno + rq_delete for each rqseqno (adlb.c:1883,
 * 1933); found[i] = 1 if it was parked. */
int adlbq_rq_delete_batch(adlbq_server *h, int n, const int *rqseqnos, int *found);

/* Both sides of a settled steal round for one shard, enqueued without a host
 * synchronisation (inputs are staged; the buffers may be reused on return):
 * the grants it donates and the rqseqnos it settled.  adlbq_steal_check
 * synchronises and returns how many grants found their unit no longer
 * available and how many rqseqnos were no longer parked since the last check
 * (both 0 when every shard applied the same merge). */
int adlbq_steal_apply(adlbq_server *h, int ngrant, const int *pairs2, int ndel, const int *rqseqnos);
int adlbq_steal_check(adlbq_server *h, int *bad_grants, int *bad_deletes);

/* ---- the steal round of the shards one process holds, with
 * no per-shard host round trip.  _create: n handles on one device (same types
 * and server count), k records per type, at most rqcap parked Reserves per
 * shard per round (later ones wait for the next round).  _export enqueues, on
 * each shard's stream, the SS_RFR_RESP reset, the top-k scan and the rq
 * compaction into one device blob of _blob_ints ints (region j = shard j;
 * d_blob = NULL: an internal buffer).  The caller may all-gather the blobs of
 * nproc processes (RCCL) into d_all = [nproc][blob]; _settle then copies
 * d_all (NULL: the local blob, nproc = 1) to pinned memory once, runs the
 * merge of adlbq_steal_merge over every shard in it, and enqueues each local
 * shard's grants and rq deletions (adlbq_steal_apply) without synchronising.
 * _responses: the replies of the local Reserves the round settled, rows
 * {shard, rqseqno, rank, TA_RESERVE_RESP[12]}; _check: adlbq_steal_check
 * summed over the shards (synchronises). */
/* A group's shards list every later Reserve batch's candidates k deeper than
 * its demand: an export right after a shard's batch (nothing else changed its
 * wq since) gathers the k best available units per type from that batch's
 * lists instead of scanning again; results are the same either way. */
typedef struct adlbq_steal_group adlbq_steal_group;
int adlbq_steal_group_create(adlbq_steal_group **g, adlbq_server **shards, int n, int k, int rqcap);
long long adlbq_steal_group_blob_ints(adlbq_steal_group *g);
int adlbq_steal_group_export(adlbq_steal_group *g, int *d_blob);
int adlbq_steal_group_settle(adlbq_steal_group *g, const int *d_all, int nproc, int *n_decided, int *n_settled);
/* The same round over a host transport (an MPI_Allgather among a node's
 * server processes, or gloo): _export_host runs _export into the internal
 * buffer and copies the blob to h_blob (_blob_ints ints; synchronises);
 * _settle_host takes the gathered host blobs h_all = [nproc][blob]. */
int adlbq_steal_group_export_host(adlbq_steal_group *g, int *h_blob);
int adlbq_steal_group_settle_host(adlbq_steal_group *g, const int *h_all, int nproc, int *n_decided, int *n_settled);
int adlbq_steal_group_responses(adlbq_steal_group *g, int cap, int *out15, int *count);
/* the units the local shards pinned in the last settle: rows {local shard j, rank, wqseqno} */
int adlbq_steal_group_grants(adlbq_steal_group *g, int cap, int *out3, int *count);
int adlbq_steal_group_check(adlbq_steal_group *g, int *bad_grants, int *bad_deletes);
/* SS_UNRESERVE (adlb.c:2051-2070) of every unit the last settle granted (a
 * benchmark restores its queues this way): one launch on the first shard's
 * stream, after the work already enqueued on every shard's stream; every
 * other shard's stream waits for it. */
int adlbq_steal_group_unreserve_grants(adlbq_steal_group *g);
/* host phase times of the last settle: "copy_ns", "merge_ns", "apply_ns"; "requests" merged */
long long adlbq_steal_group_stat(adlbq_steal_group *g, const char *name);
int adlbq_steal_group_destroy(adlbq_steal_group *g);

/* Memory-pressure push choice (src/adlb.c:513-528): the first unpinned unit
 * (wq_find_unpinned, xq.c:266-281) and the server with the smallest
 * nbytes_used below threshold (strict <, lowest index wins).  -1 when none. */
int adlbq_push_select(adlbq_server *h, double threshold, int *cand_server_rank, int *wqseqno);

/* ---- the push protocol that follows (SS_PUSH_*, adlb.c:2109-2362).
 * Pushee, SS_PUSH_QUERY with room (adlb.c:2146-2160): a unit with the next
 * wqseqno, held for this server (pinned to it: nothing matches it, it is not
 * available) until adlbq_push_commit or adlbq_push_discard.  units9 as
 * adlbq_put_batch, target_rank = the unit's real target (the reference keeps
 * it aside as temp_target_rank); bytes as a put. */
int adlbq_push_accept(adlbq_server *h, const int *units9, int *wqseqno);
/* Pusher, SS_PUSH_QUERY_RESP (adlb.c:2179-2222): if wqseqno is still live
 * and unpinned, remove it and return its fields: out10 = {1, work_type,
 * work_prio, work_len, answer_rank, target_rank, home_server_rank,
 * common_len, common_server_rank, common_seqno}; else out10[0] = 0 (a Reserve
 * or Get took it meanwhile: the caller sends SS_PUSH_DEL). */
int adlbq_push_take(adlbq_server *h, int wqseqno, int *out10);
/* Pushee, SS_PUSH_HDR (adlb.c:2232-2340): the held unit becomes available
 * (unpinned, its real target), then the put-side parked-Reserve match
 * (rq_find_rank_queued_for_type, xq.c:388-405): out3 = {found, matched_rank
 * or -1, matched_rqseqno or -1}; on a match the caller sends TA_RESERVE_RESP. */
int adlbq_push_commit(adlbq_server *h, int wqseqno, int *out3);
/* Pushee, SS_PUSH_DEL (adlb.c:2353-2360): the held unit is removed. */
int adlbq_push_discard(adlbq_server *h, int wqseqno, int *found);

/* The reference's allocation sizes on LP64 (xq.h:8-79): xq_node_t 24 B + wq_struct_t 72 B per
 * work unit (plus its payload), + rq_struct_t 80 B per parked Reserve, + tq_struct_t 16 B per
 * tq entry.  The handle's byte count adds exactly these (callers that bound it must too). */
#define ADLBQ_BYTES_WQ (24 + 72)
#define ADLBQ_BYTES_RQ (24 + 80)
#define ADLBQ_BYTES_TQ (24 + 16)

/* ---- byte accounting (SURVEY hard part 5; adlb.c:3419-3474).  The handle
 * keeps the reference's curr_bytes_dmalloced / hwm_bytes_dmalloced for the
 * structures it replaces: 24 + 72 B plus the payload per wq unit (pmalloc +
 * wq_node_create, adlb.c:933, 963), 24 + 80 B per parked Reserve
 * (rq_node_create), 24 + 16 B per tq entry; the caller adds its own
 * allocations (init tables, Isend buffers, common prefixes) with
 * adlbq_bytes_adjust, so the count is the server's.  adlbq_qmstat_row stores
 * it as this server's nbytes_used (adlb.c:3586). */
int adlbq_bytes(adlbq_server *h, double *curr, double *hwm);  /* synchronises */
int adlbq_bytes_adjust(adlbq_server *h, double delta);        /* enqueued in order */
/* FA_PUT_HDR's memory check (adlb.c:908-931): rejected = curr + work_len >
 * max_malloc; then hint = the server with the smallest nbytes_used below
 * 0.95 * max_malloc (THRESHOLD_TO_START_PUSH, adlb.c:93), excluding this one,
 * lowest index on ties, or -1 -- ack_buf[1] of the ADLB_PUT_REJECTED reply. */
int adlbq_put_check(adlbq_server *h, int work_len, double max_malloc, int *rejected, int *hint_server_rank);

/* Counters: wq->count, wq->max_count (ADLB_INFO_MAX_WQ_COUNT, adlb.c:3135), rq->count. */
int adlbq_info(adlbq_server *h, int *wq_count, int *wq_max_count, int *rq_count);

/* FA_INFO_NUM_WORK_UNITS (src/adlb.c:2466-2496): the reference's two wq
 * passes as one fused reduction over every page. */
int adlbq_info_type(adlbq_server *h, int work_type, int *max_prio, int *num_max_prio,
                    int *num_type);

/* Stream / timing plumbing. */
int  adlbq_set_stream(adlbq_server *h, void *hip_stream); /* NULL = handle's own stream */
void *adlbq_get_stream(adlbq_server *h);
int  adlbq_sync(adlbq_server *h);
/* Per-kernel GPU time (HIP events on the handle's stream around each launch of
 * a reserve batch) when enabled.  Stage names: "prep" (k_req_prep), "hist"
 * (k_hist_open), "thresholds", "select" (k_select_open), "sort"
 * (k_sort_types), "targeted", "rank", "chain" (k_chain0 + the k_chainr
 * round launches), "finalize" (k_finalize, which also parks). */
int  adlbq_profile_enable(adlbq_server *h, int on);
/* Profile one stage only (NULL: every stage); enables profiling. */
int  adlbq_profile_only(adlbq_server *h, const char *stage);
int  adlbq_profile_read(adlbq_server *h, const char *stage, double *total_ms, long long *launches);
/* Bytes the last reserve batch's open-bucket scan touched algorithmically:
 * 16 B x live units. */
long long adlbq_last_scan_units(adlbq_server *h);
/* Diagnostics of the last reserve batch: "chain_rounds" (Jacobi rounds of the
 * ordered-choice kernels, all wavefronts), "chain_passes" (passes of the
 * first launch plus the round launches that were not no-ops),
 * "chain_recomputed" (segment re-solves after pass 1), "chain_fallback"
 * (segments the last launch's in-order walk re-solved; 0 once a pass or round
 * reached the fixed point), "chain_timeouts" (bounded hand-off waits between
 * passes that gave up, cumulative; they cost time only), "parked" (Reserves parked), "candidates",
 * "sort_timeouts" (waits of the rank pass for an in-launch sort that gave up,
 * cumulative; 0 unless something is broken), "device_sorted_lists" (candidate
 * lists long enough for a device-wide radix sort of their own, cumulative),
 * "master" (the world rank of the first server, adlb.c:256; no device access).
 * -1 if unknown. */
long long adlbq_stat(adlbq_server *h, const char *name);
/* Tuning: "chain_passes" = passes of the ordered choice's first launch (1..8;
 * 0 = auto: 3 for up to 8 types, else 2): pass 1 solves every segment from a
 * guess, each later pass re-solves a segment whose start differs from its
 * predecessor's end of the pass before; "chain_rounds" = further launches
 * (0..30; -1 = auto: 0 for up to 8 types, else 2), the last of which walks in
 * order whatever is still off the fixed point; "chain_modes" = bit k-1 set:
 * round launch k starts each segment from the prefix sum of the earlier
 * segments' deltas, clear: from its predecessor's end (-1 = auto: prefix);
 * "chain_warm" = requests replayed ahead of each segment in pass 1 for up to 8
 * types (-1 = auto (512); or 0, 256, 512); "segsort_wide" = candidate-list
 * length from which a multi-priority list is sorted by a device-wide radix
 * sort of its own rather than a shared segmented sort (default 16384) when the
 * lists are not sorted together; "segsort_merged" = 1 (default) sorts every
 * list in one device-wide radix sort when no list's keys differ in their top
 * 6 bits, 0 always sorts list by list; "segsort_async" = 1 (default) sizes
 * that merged sort from the last landed batch's plan instead of reading the
 * list bounds back (a plan that does not hold leaves the sort to k_rank);
 * "tindex_delta" = capacity of the delta targeted index that Put batches merge
 * into (0: every Put batch merges into the main index); "fuse_finalize" = 1
 * runs the batch's finalize inside the ordered choice's launch (up to 8 types,
 * up to 65,536 Reserves; default 0); "rank_grid" = k_rank's grid (0 = auto);
 * "profile_every" = stage events on every n-th batch only (adlbq_stat
 * "gpu_ns:<stage>"); "hist_variant", "select_chunk", "seg_guess" select
 * measured-and-rejected kernel variants kept for their parity tests.
 * Results never depend on them; tests lower them to force the other paths. */
int adlbq_set_param(adlbq_server *h, const char *name, long long value);
const char *adlbq_last_error(void);
const char *adlbq_version(void);

#ifdef __cplusplus
}
#endif
#endif
