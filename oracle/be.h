/*
 * oracle/be.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Queue-backend interface used by the event-replay oracle (replay.c).  Two
 * implementations exist:
 *   be_own.c  -- this repo's clean-room CPU restatement of the reference's
 *                xq queue layer (src/xq.c), same doubly-linked list with one
 *                node allocation plus one record allocation per unit, same scan
 *                order and tie rules.  This is the oracle shipped to the GPU box
 *                and the timed CPU baseline ("port").
 *   be_ref.c  -- thin adapter onto the reference's own src/xq.c, compiled only
 *                in this container (oracle/Makefile, target _ref) to generate and
 *                pin golden vectors.  Never travels to the GPU box as source.
 *
 * Handles are opaque (void *); NULL means "not found", exactly as the
 * reference's xq_node_t * returns (xq.c:190-264, 388-419, 539-571).
 */
#ifndef ADLBQ_ORACLE_BE_H
#define ADLBQ_ORACLE_BE_H

#define ORC_REQ_TYPES 16            /* REQ_TYPE_VECT_SZ, xq.h:37 */
#define ORC_LOWEST_PRIO (-999999999) /* ADLB_LOWEST_PRIO, adlb.h:22 */

typedef struct be_unit_view {
    int target_rank, pin_rank, pinned, work_type, work_prio, work_len;
    int answer_rank, wqseqno, home_server_rank;
    int common_len, common_server_rank, common_server_commseqno;
} be_unit_view;

void  be_reset(void);

/* wq (xq.c:113-347) */
void *be_wq_add(int type, int prio, int seqno, int answer, int target, int len,
                int home, int clen, int csrv, int cseq);
void *be_wq_find_pre_targeted_hi_prio(int rank, const int *types16);
void *be_wq_find_hi_prio(const int *types16);
void *be_wq_find_pinned_for_rank(int rank, int seqno);
void *be_wq_find_unpinned(void);
void *be_wq_find_seqno(int seqno);
int   be_wq_num_unpinned_untargeted(void);
int   be_wq_avail_hi_prio_of_type(int type);
void  be_wq_view(void *u, be_unit_view *v);
void  be_wq_set_pin(void *u, int pin_rank, int pinned);
void  be_wq_set_target(void *u, int target_rank);
void  be_wq_delete(void *u);
int   be_wq_count(void);
int   be_wq_max_count(void);
void *be_wq_first(void);
void *be_wq_next(void *u);

/* rq (xq.c:350-444) */
void *be_rq_add(int rank, const int *types16, int rqseqno);
void *be_rq_find_rank_queued_for_type(int rank, int type);
void *be_rq_find_seqno(int rqseqno);
void *be_rq_first(void);
void *be_rq_next(void *r);
void  be_rq_view(void *r, int *rank, int *rqseqno, int *types16);
void  be_rq_delete(void *r);
int   be_rq_count(void);

/* The reference server's byte accounting (dmalloc/pmalloc/dfree,
 * adlb.c:3419-3474) over the queue structures: node + record per wq unit
 * (24 + 72 B) plus its payload, per rq entry (24 + 80 B), per tq entry
 * (24 + 16 B).  *curr = bytes held now, *hwm = the high-water mark (-1 where
 * the backend cannot tell); both include whatever the backend allocated at
 * init (the caller subtracts the value it saw after be_reset). */
void  be_bytes(double *curr, double *hwm);

/* tq (xq.c:505-585) */
int   be_tq_find_first_rt(int rank, int type); /* remote server rank or -1 */
int   be_tq_bump_or_add(int rank, int type, int server); /* FA_DID_PUT_AT_REMOTE */

#endif
