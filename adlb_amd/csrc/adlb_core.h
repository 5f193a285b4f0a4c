/* adlb_core.h -- the ADLB server's message handlers, without MPI.
 *
 * One adlbsrv object = one server rank.  Each function is the handler of one
 * inbound message kind of the reference server loop (ADLBP_Server,
 * src/adlb.c:382-2500) and emits its replies through the callback given at
 * create, in the order the reference sends them.  The queue work runs on the
 * GPU through the adlbq engine (include/adlbq.h); payloads, common prefixes
 * and timestamps stay in host memory here.
 *
 * Two drivers use it: the MPI server loop (adlb_mpi.cpp, libadlb.so) and the
 * replay of recorded reference event streams (tests/test_gpu_server.py).
 */
#ifndef ADLB_CORE_H
#define ADLB_CORE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct adlbsrv adlbsrv;
/* dest = world rank; buf/nbytes are only valid during the call */
typedef void (*adlbsrv_emit_fn)(void *ctx, int dest, int tag, const void *buf, int nbytes);

int adlbsrv_create(adlbsrv **out, int ntypes, const int *user_types, int num_app_ranks, int num_servers,
                   int my_world_rank, double max_malloc, int device, adlbsrv_emit_fn emit, void *ctx);
int adlbsrv_destroy(adlbsrv *s);
const char *adlbsrv_last_error(void);

/* FA_PUT_HDR (adlb.c:891-962): acks (or rejects / answers NO_MORE_WORK);
 * *need_payload = 1 when the sender will now send the payload, which goes to
 * adlbsrv_put_payload (adlb.c:963-1049). */
int adlbsrv_put_hdr(adlbsrv *s, int src, const int *hdr12, int *need_payload);
int adlbsrv_put_payload(adlbsrv *s, int src, const int *hdr12, const void *buf, int len);
/* Batched Puts (the MPI loop drains a run of waiting FA_PUT_HDRs): _stage
 * keeps an accepted Put's payload instead of appending it, _flush appends
 * every staged Put with one adlbq_put_batch (arrival order: the same queue
 * and rq matches as one at a time) and sends, per Put in order, the
 * TA_RESERVE_RESP of a matched parked Reserve and the final ack.  While Puts
 * are staged, adlbsrv_put_hdr's memory check (adlb.c:908) is decided from
 * exact bounds on the staged Puts' bytes (each adds BYTES_WQ + len and an rq
 * match frees BYTES_RQ); an undecidable check flushes first.  Every other
 * handler requires nothing staged (the driver flushes at the end of the run). */
int adlbsrv_put_stage(adlbsrv *s, int src, const int *hdr12, const void *buf, int len);
int adlbsrv_put_flush(adlbsrv *s);
int adlbsrv_put_staged(adlbsrv *s);
/* FA_PUT_COMMON_HDR / _MSG (adlb.c:1054-1134), FA_PUT_BATCH_DONE (1135-1160),
 * FA_GET_COMMON (1321-1332) */
int adlbsrv_put_common_hdr(adlbsrv *s, int src, int common_len, int *need_payload);
int adlbsrv_put_common_payload(adlbsrv *s, int src, const void *buf, int len);
int adlbsrv_batch_done(adlbsrv *s, int src, int cqseqno, int refcnt);
int adlbsrv_get_common(adlbsrv *s, int src, int cqseqno);
/* FA_DID_PUT_AT_REMOTE (adlb.c:1161-1180) */
int adlbsrv_did_put_at_remote(adlbsrv *s, int type, int target, int server_rank);
/* n FA_RESERVEs in arrival order (adlb.c:1181-1320): one adlbq_reserve_batch */
int adlbsrv_reserve_batch(adlbsrv *s, int n, const int *src, const int *bufs17);
/* n FA_GET_RESERVEDs in arrival order (adlb.c:1333-1384): one adlbq_get_reserved_batch */
int adlbsrv_get_batch(adlbsrv *s, int n, const int *src, const int *wqseqno);
/* FA_INFO_NUM_WORK_UNITS (adlb.c:2466-2496) */
int adlbsrv_info_num(adlbsrv *s, int src, int work_type);
/* FA_NO_MORE_WORK / SS_NO_MORE_WORK (adlb.c:1385-1492): set the flag and
 * answer every parked Reserve; returns 1 if the flag was newly set */
int adlbsrv_no_more_work(adlbsrv *s);
/* SS_DONE_BY_EXHAUSTION (adlb.c:1627-1650, 757-772): answer every parked Reserve */
int adlbsrv_exhausted(adlbsrv *s);
/* SS_QMSTAT (adlb.c:1705-1757): install the other servers' rows, then
 * check_remote_work_for_queued_apps (3536-3579).  qlen[S], nbytes[S], hi[S*T]. */
int adlbsrv_qmstat(adlbsrv *s, const int *qlen, const double *nbytes, const int *hi);
/* update_local_state (adlb.c:3581-3593): this server's row */
int adlbsrv_my_row(adlbsrv *s, int *qlen, double *nbytes, int *hi);
/* SS_RFR (adlb.c:1802-1866), SS_RFR_RESP (1867-2050), SS_UNRESERVE (2051-2070) */
int adlbsrv_rfr(adlbsrv *s, int src, const int *buf28);
int adlbsrv_rfr_resp(adlbsrv *s, int src, const int *buf28);
int adlbsrv_unreserve(adlbsrv *s, int src, const int *buf12);

/* Memory-pressure push (adlb.c:509-556, 2109-2362).  push_tick: the loop-top
 * check -- above 0.95 max_malloc with no query out, the first unpinned unit
 * goes as SS_PUSH_QUERY to the server with the smallest nbytes_used below the
 * threshold; returns 1 if a query was sent.  push_query (pushee, double[12]),
 * push_query_resp (pusher, double[12]: SS_PUSH_HDR + SS_PUSH_WORK or
 * SS_PUSH_DEL), push_hdr (pushee, int[12] + the SS_PUSH_WORK payload; len of
 * that payload from push_len), push_del (pushee), moving_targeted (home
 * server, SS_MOVING_TARGETED_WORK int[12], adlb.c:2071-2108). */
int adlbsrv_push_tick(adlbsrv *s);
int adlbsrv_push_query(adlbsrv *s, int src, const double *d12);
int adlbsrv_push_query_resp(adlbsrv *s, int src, const double *d12);
int adlbsrv_push_len(adlbsrv *s, int wqseqno);
int adlbsrv_push_hdr(adlbsrv *s, int src, const int *b12, const void *payload, int len);
int adlbsrv_push_del(adlbsrv *s, int src, const int *b12);
int adlbsrv_moving_targeted(adlbsrv *s, int src, const int *b12);

/* Steal group (the north star's cross-shard merge): the
 * node's server processes settle their parked Reserves by rounds of export ->
 * all-gather of the blobs (the driver's transport: MPI_Allgather among the
 * servers) -> the deterministic merge of adlbq_steal_merge, which replays the
 * SS_RFR round trips (adlb.c:1280-1308, 1802-1948, 3536-3579) on one snapshot.
 * _create: k exported units per type, rqcap parked Reserves per round; from
 * then on parks send no SS_RFR unless the donor may hold targeted work for
 * the rank (a tq entry: adlb.c:3493-3500), which a round never exports.
 * _export writes this server's blob (_blob_ints ints); _settle takes the
 * gathered blobs of all nproc servers ([nproc][blob], any order), answers the
 * Reserves of this server the round settled (TA_RESERVE_RESP), pins the units
 * it donates, and checks that every grant and deletion applied (*settled =
 * this server's answered Reserves).  Between _export and _settle the caller
 * must not hand the server any other message.  _stat: 0 rounds, 1 Reserves
 * settled by rounds, 2 SS_RFRs sent. */
int adlbsrv_group_create(adlbsrv *s, int k, int rqcap);
long long adlbsrv_group_blob_ints(adlbsrv *s);
int adlbsrv_group_export(adlbsrv *s, int *blob);
int adlbsrv_group_settle(adlbsrv *s, const int *all, int nproc, int *settled);
/* the same with the blobs in device memory (d_blob: _blob_ints ints; d_all: [nproc][blob],
 * all-gathered by RCCL between the server processes) */
int adlbsrv_group_export_device(adlbsrv *s, int *d_blob);
int adlbsrv_group_settle_device(adlbsrv *s, const int *d_all, int nproc, int *settled);
long long adlbsrv_group_stat(adlbsrv *s, int which);

/* A native server-loop driver for recorded event streams (adlb_replay.cpp):
 * n shards' traces (oracle/replay.h format) through the engine ABI, one host
 * thread per shard; runs of Puts / Reserves / Gets as one batch call each.
 * outs[j] (caps[j] ints) receives adlb_amd/replay.py's output layout;
 * nouts[j] = ints written, ncalls[j] = ABI calls made (may be NULL).
 * Returns 0, -1 (an engine error: adlbsrv_replay_error), -2 (output full). */
typedef struct adlbq_server adlbq_server;
int adlbsrv_replay_many(adlbq_server **hs, int n, int ntypes, const int *const *traces, const long long *lens,
                        int *const *outs, const long long *caps, long long *nouts, long long *ncalls);
const char *adlbsrv_replay_error(void);
/* Config 5 at its SURVEY shape (oracle/gen_c5.c): S shards' traces with steal
 * rounds (event 23 at the same place in every trace).  Between rounds each
 * shard's Puts / Reserves / Gets go down as device-side batches from its own
 * host thread (inputs staged in HBM first, outputs left there: no
 * synchronisation per call); a round runs adlbq_steal_group_export + _settle
 * over all S shards (export depth k, rqcap parked Reserves per shard) and its
 * responses are appended to steals (rows of 15).  outs[j] receives the replay
 * layout; *seconds the wall time of the replay (staging excluded). */
int adlbsrv_replay_rounds(adlbq_server **hs, int S, int ntypes, const int *const *traces, const long long *lens,
                          int k, int rqcap, int *const *outs, const long long *caps, long long *nouts,
                          int *steals, long long steal_cap, long long *nsteals, double *seconds, long long *ncalls);
/* The same; closed != 0: a shard issues each Get only once the reply it depends on (its Reserve's
 * TA_RESERVE_RESP, the put-side match of its parked Reserve, or the steal round's answer) has landed in
 * mapped host memory, with the wqseqno from that reply (tsp.c:157-162).  cl_stats[3] (may be NULL):
 * Get calls that waited, seconds waited, replies whose wqseqno differs from the recorded Get's. */
int adlbsrv_replay_rounds2(adlbq_server **hs, int S, int ntypes, const int *const *traces, const long long *lens,
                           int k, int rqcap, int *const *outs, const long long *caps, long long *nouts,
                           int *steals, long long steal_cap, long long *nsteals, double *seconds, long long *ncalls,
                           int closed, double *cl_stats);
void adlbsrv_replay_prof(double *out8);

/* state for the driver */
int adlbsrv_num_parked(adlbsrv *s);     /* rq->count */
long long adlbsrv_activity(adlbsrv *s); /* events that changed a queue (exhaustion check) */
long long adlbsrv_row_stamp(adlbsrv *s); /* changes when this server's qmstat row may have (queues, bytes, misses) */
int adlbsrv_rfr_outstanding(adlbsrv *s);
int adlbsrv_nmw(adlbsrv *s);
/* ADLB_Info_get keys (adlb.h ADLB_INFO_*, adlb.c:3072-3141) */
int adlbsrv_info_get(adlbsrv *s, int key, double *val);

#ifdef __cplusplus
}
#endif
#endif
