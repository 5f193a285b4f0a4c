/*
 * oracle/be_ref.c -- TEST INFRASTRUCTURE ONLY.  Adapter from the oracle's
 * backend interface (be.h) onto the REFERENCE's own queue layer,
 * /root/reference/src/xq.c, compiled where it lies by oracle/Makefile into
 * oracle/_ref/libxqref.so (gitignored).  Used only in this container to
 * generate and pin the golden vectors under tests/golden/.  Every call below
 * is a call into unmodified reference code; this file only unwraps
 * xq_node_t->data.
 */
#include <stdlib.h>
#include <mpi.h>
#include <adlb/adlb.h> /* /root/reference/include/adlb/adlb.h */
#include "xq.h"        /* /root/reference/src/xq.h */
#include "be.h"

/* adlb.c's allocators (global functions of the reference, adlb.c:3419-3474) */
void *pmalloc(int nbytes, const char *funcname, int linenum);
void dfree(void *ptr, int nbytes, const char *funcname, int linenum);

static void drain(xq_t *q, void (*del)(xq_node_t *))
{
    xq_node_t *n;
    while ((n = xq_first(q)) != NULL)
        del(n);
}

void be_reset(void)
{
    static int inited;
    if (!inited) {
        /* xq.c allocates through adlb.c's dmalloc, whose limit (max_malloc) is
         * only set by ADLBP_Init (adlb.c:218); run it as a singleton MPI job of
         * one server rank, which also creates wq/rq/iq/tq/cq (adlb.c:301-305). */
        int flag = 0, am_server, am_dbg, t0 = 0;
        MPI_Comm app;
        MPI_Initialized(&flag);
        if (!flag)
            MPI_Init(NULL, NULL);
        ADLBP_Init(1, 0, 0, 1, &t0, &am_server, &am_dbg, &app);
        inited = 1;
    }
    drain(wq, wq_delete);
    drain(rq, rq_delete);
    drain(tq, tq_delete);
    wq->count = wq->max_count = 0;
    rq->count = rq->max_count = 0;
    tq->count = tq->max_count = 0;
}

void *be_wq_add(int type, int prio, int seqno, int answer, int target, int len,
                int home, int clen, int csrv, int cseq)
{
    /* adlb.c:933 + 963-973: the payload through the reference's pmalloc (so
     * its accounting holds it, and wq_delete's afree releases it, xq.c:167),
     * then wq_node_create + field fill + wq_append */
    void *buf = len > 0 ? pmalloc(len, __FUNCTION__, __LINE__) : NULL;
    xq_node_t *n = wq_node_create(type, prio, seqno, answer, target, len, buf);
    wq_struct_t *ws = (wq_struct_t *)n->data;
    ws->home_server_rank = home;
    ws->common_len = clen;
    ws->common_server_rank = csrv;
    ws->common_server_commseqno = cseq;
    wq_append(n);
    return n;
}

void *be_wq_find_pre_targeted_hi_prio(int rank, const int *t) { return wq_find_pre_targeted_hi_prio(rank, (int *)t); }
void *be_wq_find_hi_prio(const int *t) { return wq_find_hi_prio((int *)t); }
void *be_wq_find_pinned_for_rank(int rank, int seqno) { return wq_find_pinned_for_rank(rank, seqno); }
void *be_wq_find_unpinned(void) { return wq_find_unpinned(); }
int be_wq_num_unpinned_untargeted(void) { return wq_get_num_unpinned_untargeted(); }
int be_wq_avail_hi_prio_of_type(int type) { return wq_get_avail_hi_prio_of_type(type); }

void be_wq_view(void *h, be_unit_view *v)
{
    const wq_struct_t *ws = (const wq_struct_t *)((xq_node_t *)h)->data;
    v->target_rank = ws->target_rank;
    v->pin_rank = ws->pin_rank;
    v->pinned = ws->pinned;
    v->work_type = ws->work_type;
    v->work_prio = ws->work_prio;
    v->work_len = ws->work_len;
    v->answer_rank = ws->answer_rank;
    v->wqseqno = ws->wqseqno;
    v->home_server_rank = ws->home_server_rank;
    v->common_len = ws->common_len;
    v->common_server_rank = ws->common_server_rank;
    v->common_server_commseqno = ws->common_server_commseqno;
}

void be_wq_set_pin(void *h, int pin_rank, int pinned)
{
    wq_struct_t *ws = (wq_struct_t *)((xq_node_t *)h)->data;
    ws->pin_rank = pin_rank;
    ws->pinned = pinned;
}

void be_wq_set_target(void *h, int target_rank) { ((wq_struct_t *)((xq_node_t *)h)->data)->target_rank = target_rank; }
void *be_wq_find_seqno(int seqno) { return wq_find_seqno(seqno); }
void be_wq_delete(void *h) { wq_delete((xq_node_t *)h); }
int be_wq_count(void) { return wq->count; }
int be_wq_max_count(void) { return wq->max_count; }
void *be_wq_first(void) { return xq_first(wq); }
void *be_wq_next(void *h) { return xq_next(wq, (xq_node_t *)h); }

void *be_rq_add(int rank, const int *t, int rqseqno)
{
    xq_node_t *n = rq_node_create(rank, (int *)t, rqseqno);
    rq_append(n);
    return n;
}

void *be_rq_find_rank_queued_for_type(int rank, int type) { return rq_find_rank_queued_for_type(rank, type); }
void *be_rq_find_seqno(int rqseqno) { return rq_find_seqno(rqseqno); }
void *be_rq_first(void) { return xq_first(rq); }
void *be_rq_next(void *h) { return xq_next(rq, (xq_node_t *)h); }

void be_rq_view(void *h, int *rank, int *rqseqno, int *t)
{
    const rq_struct_t *rs = (const rq_struct_t *)((xq_node_t *)h)->data;
    *rank = rs->world_rank;
    *rqseqno = rs->rqseqno;
    for (int i = 0; i < REQ_TYPE_VECT_SZ; i++)
        t[i] = rs->req_types[i];
}

void be_rq_delete(void *h) { rq_delete((xq_node_t *)h); }
int be_rq_count(void) { return rq->count; }

/* The reference keeps curr_bytes_dmalloced static (adlb.c:121); only its
 * high-water mark is readable (ADLBP_Info_get(ADLB_INFO_MALLOC_HWM),
 * adlb.c:3074-3078).  curr is read by a probe: pmalloc(X) raises the mark to
 * curr + X when X exceeds the mark's lead over curr, and dfree returns it.
 * Each probe uses a larger X (by 1 MiB), so it reads curr exactly while curr
 * never drops by a MiB between probes (fixture traces are far smaller); the
 * mark itself is then unusable (*hwm = -1). */
void be_bytes(double *curr, double *hwm)
{
    static int probes;
    const int x = (1 << 30) + (++probes << 20);
    void *p = pmalloc(x, __FUNCTION__, __LINE__);
    double m = 0;
    ADLBP_Info_get(ADLB_INFO_MALLOC_HWM, &m);
    dfree(p, x, __FUNCTION__, __LINE__);
    *curr = m - (double)x;
    *hwm = -1;
}

int be_tq_find_first_rt(int rank, int type)
{
    xq_node_t *n = tq_find_first_rt(rank, type);
    return n ? ((tq_struct_t *)n->data)->remote_server_rank : -1;
}

int be_tq_bump_or_add(int rank, int type, int server)
{
    /* adlb.c:1167-1178 */
    xq_node_t *n = tq_find_rtr(rank, type, server);
    if (n)
        return ++((tq_struct_t *)n->data)->num_stored;
    n = tq_node_create(rank, type, server, 1);
    tq_append(n);
    return 1;
}
