/*
 * oracle/replay.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of the reference server loop's queue handlers (src/adlb.c) on
 * top of a queue backend (be.h).  Linked with be_own.c it is the oracle; with
 * be_ref.c + /root/reference/src/xq.c it produces the golden vectors.
 * MPI sends are replaced by writing the message contents to the output stream.
 */
#include <stdlib.h>
#include <string.h>
#include "be.h"
#include "replay.h"

static struct {
    int ntypes, *user_types;
    int num_app_ranks, num_servers, my_idx;
    int my_world_rank, master_server_rank, num_world;
    int next_wqseqno, next_rqseqno;
    int *qm_hi;       /* [num_servers][ntypes]  qmstat_tbl[i].type_hi_prio */
    int *qm_qlen;     /* [num_servers]          qmstat_tbl[i].qlen_unpin_untarg */
    double *qm_bytes; /* [num_servers]          qmstat_tbl[i].nbytes_used */
    int *rfr_out;     /* [num_world]  (adlb.c:112, zeroed: SURVEY hard part 4) */
    int *rfr_to_rank; /* [num_app_ranks] */
    double bytes0;    /* the backend's byte count after init (queue bytes are relative to it) */
    int *temp_target; /* [cap_tt] ws->temp_target_rank of units accepted by SS_PUSH_QUERY, by wqseqno */
    int cap_tt;
} S;

int orc_init(int ntypes, const int *user_types, int num_app_ranks, int num_servers,
             int my_server_idx)
{
    free(S.user_types); free(S.qm_hi); free(S.qm_qlen); free(S.qm_bytes);
    free(S.rfr_out); free(S.rfr_to_rank);
    S.ntypes = ntypes;
    S.user_types = (int *)malloc(sizeof(int) * (ntypes > 0 ? ntypes : 1));
    memcpy(S.user_types, user_types, sizeof(int) * ntypes);
    S.num_app_ranks = num_app_ranks;
    S.num_servers = num_servers;
    S.my_idx = my_server_idx;
    /* rank layout without a debug server, adlb.c:246-258 */
    S.master_server_rank = num_app_ranks;
    S.my_world_rank = num_app_ranks + my_server_idx;
    S.num_world = num_app_ranks + num_servers;
    S.next_wqseqno = 1; /* adlb.c:319 */
    S.next_rqseqno = 1; /* adlb.c:320 */
    S.qm_hi = (int *)malloc(sizeof(int) * num_servers * (ntypes > 0 ? ntypes : 1));
    S.qm_qlen = (int *)calloc(num_servers, sizeof(int));
    S.qm_bytes = (double *)calloc(num_servers, sizeof(double));
    for (int i = 0; i < num_servers * ntypes; i++)
        S.qm_hi[i] = ORC_LOWEST_PRIO; /* adlb.c:301-316 */
    free(S.temp_target);
    S.temp_target = NULL;
    S.cap_tt = 0;
    S.rfr_out = (int *)calloc(S.num_world, sizeof(int));
    S.rfr_to_rank = (int *)malloc(sizeof(int) * num_app_ranks);
    for (int i = 0; i < num_app_ranks; i++)
        S.rfr_to_rank[i] = -1;
    be_reset();
    double h;
    be_bytes(&S.bytes0, &h);
    return 0;
}

static int type_idx(int work_type) /* get_type_idx, adlb.c:3476-3485 */
{
    for (int i = 0; i < S.ntypes; i++)
        if (S.user_types[i] == work_type)
            return i;
    return -1;
}

/* find_cand_rank_with_worktype, adlb.c:3487-3534 */
static int find_cand(int for_rank, int work_type)
{
    int t = be_tq_find_first_rt(for_rank, work_type);
    if (t >= 0)
        return t;
    int bsf = -1, hi = ORC_LOWEST_PRIO;
    for (int i = 0; i < S.num_servers; i++) {
        int srv = S.master_server_rank + i;
        if (srv == S.my_world_rank || S.rfr_out[srv])
            continue;
        if (S.qm_qlen[i] <= 0)
            continue;
        const int *row = S.qm_hi + (long)i * S.ntypes;
        if (work_type < 0) {
            for (int j = 0; j < S.ntypes; j++)
                if (row[j] > hi) {
                    hi = row[j];
                    bsf = srv;
                }
        } else {
            int ti = type_idx(work_type);
            if (ti >= 0 && row[ti] > hi) { /* ti < 0 is UB in the reference; traces avoid it */
                hi = row[ti];
                bsf = srv;
            }
        }
    }
    return bsf;
}

/* walk one parked request's types in order (adlb.c:1280-1308, 3549-3577) */
static int rfr_for(int rank, const int *types16)
{
    for (int i = 0; i < ORC_REQ_TYPES; i++) {
        if (types16[i] < -1)
            break;
        int cand = find_cand(rank, types16[i]);
        if (cand >= 0) {
            S.rfr_to_rank[rank] = cand;
            S.rfr_out[cand] = 1;
            return cand;
        }
    }
    return -1;
}

/* check_remote_work_for_queued_apps, adlb.c:3536-3579 */
static long check_remote(int *o, long cap)
{
    long k = 0;
    int types[ORC_REQ_TYPES], rank, rqseqno;
    for (void *r = be_rq_first(); r; r = be_rq_next(r)) {
        be_rq_view(r, &rank, &rqseqno, types);
        if (S.rfr_to_rank[rank] >= 0)
            continue;
        int cand = rfr_for(rank, types);
        if (cand >= 0) {
            if (1 + 3 * (k + 1) > cap)
                return -1;
            o[1 + 3 * k] = rqseqno;
            o[2 + 3 * k] = rank;
            o[3 + 3 * k] = cand;
            k++;
        }
    }
    o[0] = (int)k;
    return 1 + 3 * k;
}

int orc_event_nargs(int op, int ntypes)
{
    switch (op) {
    case ORC_OP_PUT: return 9;
    case ORC_OP_RESERVE: return 2 + ORC_REQ_TYPES;
    case ORC_OP_GET: return 2;
    case ORC_OP_UNRESERVE: return 3;
    case ORC_OP_QMROW: return 0;
    case ORC_OP_SETROW: return 3 + ntypes;
    case ORC_OP_CHECKREM: return 0;
    case ORC_OP_RFRDONE: return 2;
    case ORC_OP_TQADD: return 3;
    case ORC_OP_PUSHSEL: return 1;
    case ORC_OP_INFO: return 0;
    case ORC_OP_RQDEL: return 1;
    case ORC_OP_INFOTYPE: return 1;
    case ORC_OP_RFR: return 2 + ORC_REQ_TYPES;
    case ORC_OP_RQLIST: return 0;
    case ORC_OP_BYTES: return 0;
    case ORC_OP_PUTCHECK: return 2;
    case ORC_OP_HWM: return 0;
    case ORC_OP_PUSHACCEPT: return 9;
    case ORC_OP_PUSHTAKE: return 1;
    case ORC_OP_PUSHCOMMIT: return 1;
    case ORC_OP_PUSHDEL: return 1;
    case ORC_OP_ROUND: return 0;
    default: return -1;
    }
}

long orc_replay(const int *tr, long ntrace, int *out, long outcap)
{
    long ip = 0, op = 0;
    int T = S.ntypes;
    while (ip < ntrace) {
        int code = tr[ip];
        int na = orc_event_nargs(code, T);
        if (na < 0 || ip + 1 + na > ntrace)
            return -2;
        const int *a = tr + ip + 1;
        ip += 1 + na;
        /* every event writes at most max(16, 1+T, 1+3*rq) ints; check loosely */
        if (op + 2 + (ORC_RESP_INTS > T + 1 ? ORC_RESP_INTS : T + 1) > outcap)
            return -1;
        int *o = out + op + 1;
        long n = 0;
        switch (code) {
        case ORC_OP_PUT: {
            /* FA_PUT_HDR after the payload arrives, adlb.c:963-1046 */
            int seq = S.next_wqseqno++;
            void *u = be_wq_add(a[0], a[1], seq, a[2], a[3], a[4], a[5], a[6], a[7], a[8]);
            void *r = be_rq_find_rank_queued_for_type(a[3], a[0]); /* rank may be -1 */
            o[0] = seq;
            o[1] = -1;
            o[2] = -1;
            if (r) {
                int rank, rqs, types[ORC_REQ_TYPES];
                be_rq_view(r, &rank, &rqs, types);
                be_wq_set_pin(u, rank, rank >= 0 ? 1 : 0); /* 993-995 */
                o[1] = rank;
                o[2] = rqs;
                be_rq_delete(r); /* 1040 */
            }
            n = 3;
            break;
        }
        case ORC_OP_RESERVE: {
            /* FA_RESERVE, adlb.c:1199-1317 */
            int rank = a[0], hang = a[1];
            const int *types = a + 2;
            void *u = be_wq_find_pre_targeted_hi_prio(rank, types);
            if (!u)
                u = be_wq_find_hi_prio(types);
            memset(o, 0, sizeof(int) * ORC_RESP_INTS);
            o[10] = -1;
            o[11] = -1;
            if (u) {
                be_unit_view v;
                be_wq_view(u, &v);
                be_wq_set_pin(u, rank, rank >= 0 ? 1 : v.pinned); /* 1210-1212 */
                o[0] = 1;
                o[1] = v.work_type;
                o[2] = v.work_prio;
                o[3] = v.work_len;
                o[4] = v.answer_rank;
                o[5] = v.wqseqno;
                o[6] = S.my_world_rank;
                o[7] = v.common_len;
                o[8] = v.common_server_rank;
                o[9] = v.common_server_commseqno;
            } else if (hang) {
                int rqs = S.next_rqseqno++; /* 1244-1277 */
                be_rq_add(rank, types, rqs);
                o[10] = rqs;
                if (S.rfr_to_rank[rank] < 0) /* 1278-1309 */
                    o[11] = rfr_for(rank, types);
            } else {
                o[0] = -2; /* NO_CURR_WORK, 1311-1316 */
            }
            n = ORC_RESP_INTS;
            break;
        }
        case ORC_OP_GET: {
            /* FA_GET_RESERVED, adlb.c:1347-1381 */
            void *u = be_wq_find_pinned_for_rank(a[0], a[1]);
            if (!u) {
                o[0] = -1; o[1] = o[2] = o[3] = o[4] = 0;
            } else {
                be_unit_view v;
                be_wq_view(u, &v);
                o[0] = 1; o[1] = v.work_len; o[2] = v.work_type; o[3] = v.work_prio;
                o[4] = v.answer_rank;
                be_wq_delete(u);
            }
            n = 5;
            break;
        }
        case ORC_OP_UNRESERVE: {
            /* SS_UNRESERVE, adlb.c:2057-2063 */
            void *u = be_wq_find_pinned_for_rank(a[0], a[1]);
            o[0] = 0;
            if (u) {
                be_wq_set_pin(u, a[2], 0);
                o[0] = 1;
            }
            n = 1;
            break;
        }
        case ORC_OP_QMROW: {
            /* update_local_state, adlb.c:3581-3593 */
            int q = be_wq_num_unpinned_untargeted();
            o[0] = q;
            S.qm_qlen[S.my_idx] = q;
            for (int i = 0; i < T; i++) {
                int h = be_wq_avail_hi_prio_of_type(S.user_types[i]);
                o[1 + i] = h;
                S.qm_hi[(long)S.my_idx * T + i] = h;
            }
            n = 1 + T;
            break;
        }
        case ORC_OP_SETROW: {
            /* the ring hop's unpack keeps the local row (adlb.c:1716-1728) */
            int i = a[0];
            if (i >= 0 && i < S.num_servers && i != S.my_idx) {
                S.qm_qlen[i] = a[1];
                S.qm_bytes[i] = (double)a[2];
                for (int j = 0; j < T; j++)
                    S.qm_hi[(long)i * T + j] = a[3 + j];
            }
            n = 0;
            break;
        }
        case ORC_OP_CHECKREM:
            n = check_remote(o, outcap - op - 1);
            if (n < 0)
                return -1;
            break;
        case ORC_OP_RFRDONE:
            /* SS_RFR_RESP bookkeeping, adlb.c:1877-1878 */
            if (a[1] >= 0 && a[1] < S.num_app_ranks)
                S.rfr_to_rank[a[1]] = -1;
            if (a[0] >= 0 && a[0] < S.num_world)
                S.rfr_out[a[0]] = 0;
            n = 0;
            break;
        case ORC_OP_TQADD:
            /* FA_DID_PUT_AT_REMOTE, adlb.c:1163-1179 */
            be_tq_bump_or_add(a[0], a[1], a[2]);
            n = check_remote(o, outcap - op - 1);
            if (n < 0)
                return -1;
            break;
        case ORC_OP_PUSHSEL: {
            /* memory-pressure push donor choice, adlb.c:513-528 */
            void *u = be_wq_find_unpinned();
            o[0] = -1;
            o[1] = -1;
            if (u) {
                be_unit_view v;
                be_wq_view(u, &v);
                double smallest = 999999999999.9, thr = (double)a[0];
                int cand = -1;
                for (int i = 0; i < S.num_servers; i++) {
                    int srv = S.master_server_rank + i;
                    if (srv != S.my_world_rank && S.qm_bytes[i] < thr && S.qm_bytes[i] < smallest) {
                        smallest = S.qm_bytes[i];
                        cand = srv;
                    }
                }
                o[0] = cand;
                o[1] = v.wqseqno;
            }
            n = 2;
            break;
        }
        case ORC_OP_BYTES: {
            double c, h;
            be_bytes(&c, &h);
            o[0] = (int)(c - S.bytes0);
            n = 1;
            break;
        }
        case ORC_OP_PUSHACCEPT: {
            /* SS_PUSH_QUERY at the pushee, room left (adlb.c:2146-2160): a unit
             * with the next local seqno, targeted at and pinned to this server
             * until SS_PUSH_HDR; the real target is kept aside */
            int seq = S.next_wqseqno++;
            void *u = be_wq_add(a[0], a[1], seq, a[2], S.my_world_rank, a[4], a[5], a[6], a[7], a[8]);
            be_wq_set_pin(u, S.my_world_rank, 1);
            if (seq >= S.cap_tt) {
                int nc = 2 * seq + 16;
                S.temp_target = (int *)realloc(S.temp_target, sizeof(int) * nc);
                S.cap_tt = nc;
            }
            S.temp_target[seq] = a[3];
            o[0] = seq;
            n = 1;
            break;
        }
        case ORC_OP_PUSHTAKE: {
            /* SS_PUSH_QUERY_RESP at the pusher (adlb.c:2179-2222): the unit goes
             * unless a Reserve pinned it or a Get took it meanwhile */
            void *u = be_wq_find_seqno(a[0]);
            be_unit_view v;
            memset(o, 0, sizeof(int) * 10);
            if (u) be_wq_view(u, &v);
            if (u && !v.pinned) {
                o[0] = 1; o[1] = v.work_type; o[2] = v.work_prio; o[3] = v.work_len; o[4] = v.answer_rank;
                o[5] = v.target_rank; o[6] = v.home_server_rank; o[7] = v.common_len;
                o[8] = v.common_server_rank; o[9] = v.common_server_commseqno;
                be_wq_delete(u); /* 2221-2222 (the payload leaves with the Isend) */
            }
            n = 10;
            break;
        }
        case ORC_OP_PUSHCOMMIT: {
            /* SS_PUSH_HDR at the pushee (adlb.c:2232-2340): the real target,
             * unpinned, then the parked-Reserve match of a put */
            void *u = be_wq_find_seqno(a[0]);
            o[0] = 0; o[1] = -1; o[2] = -1;
            if (u) {
                be_unit_view v;
                be_wq_set_target(u, a[0] < S.cap_tt ? S.temp_target[a[0]] : -1); /* 2240 */
                be_wq_set_pin(u, -1, 0);                                         /* 2241-2242 */
                be_wq_view(u, &v);
                o[0] = 1;
                void *r = be_rq_find_rank_queued_for_type(v.target_rank, v.work_type); /* 2287 */
                if (r) {
                    int rank, rqs, types[ORC_REQ_TYPES];
                    be_rq_view(r, &rank, &rqs, types);
                    be_wq_set_pin(u, rank, rank >= 0 ? 1 : 0); /* 2291-2293 */
                    o[1] = rank;
                    o[2] = rqs;
                    be_rq_delete(r); /* 2338 */
                }
            }
            n = 3;
            break;
        }
        case ORC_OP_PUSHDEL: {
            /* SS_PUSH_DEL at the pushee (adlb.c:2353-2360) */
            void *u = be_wq_find_seqno(a[0]);
            o[0] = u != NULL;
            if (u) be_wq_delete(u);
            n = 1;
            break;
        }
        case ORC_OP_HWM: {
            double c, h;
            be_bytes(&c, &h);
            o[0] = h < 0 ? -1 : (int)(h - S.bytes0);
            n = 1;
            break;
        }
        case ORC_OP_PUTCHECK: {
            /* FA_PUT_HDR's memory check and reject hint, adlb.c:908-931 */
            double c, h;
            be_bytes(&c, &h);
            o[0] = (c - S.bytes0) + (double)a[0] > (double)a[1];
            o[1] = -1;
            if (o[0]) {
                const double thr = 0.95 * (double)a[1]; /* THRESHOLD_TO_START_PUSH, adlb.c:93 */
                double smallest = 999999999999.9;
                for (int i = 0; i < S.num_servers; i++) {
                    int srv = S.master_server_rank + i;
                    if (srv != S.my_world_rank && S.qm_bytes[i] < thr && S.qm_bytes[i] < smallest) {
                        smallest = S.qm_bytes[i];
                        o[1] = srv;
                    }
                }
            }
            n = 2;
            break;
        }
        case ORC_OP_INFO:
            o[0] = be_wq_count();
            o[1] = be_wq_max_count();
            o[2] = be_rq_count();
            n = 3;
            break;
        case ORC_OP_RQDEL: {
            void *r = be_rq_find_seqno(a[0]);
            o[0] = 0;
            if (r) {
                be_rq_delete(r);
                o[0] = 1;
            }
            n = 1;
            break;
        }
        case ORC_OP_RFR: {
            /* SS_RFR at the donor, adlb.c:1802-1866: the pre-targeted scan for
             * for_rank, then the untargeted scan; pin and answer SS_RFR_RESP */
            int for_rank = a[1];
            const int *types = a + 2;
            void *u = be_wq_find_pre_targeted_hi_prio(for_rank, types);
            if (!u)
                u = be_wq_find_hi_prio(types);
            if (u) {
                be_unit_view v;
                be_wq_view(u, &v);
                be_wq_set_pin(u, for_rank, for_rank >= 0 ? 1 : v.pinned); /* 1820-1824 */
                o[0] = 1;
                o[1] = a[0];
                o[2] = for_rank;
                o[3] = v.work_type;
                o[4] = v.work_prio;
                o[5] = v.work_len;
                o[6] = v.answer_rank;
                o[7] = v.wqseqno;
                o[8] = v.target_rank; /* prev_target */
                o[9] = v.common_len;
                o[10] = v.common_server_rank;
                o[11] = v.common_server_commseqno;
                n = 12;
            } else {
                /* NO_CURR_WORK; the donor refreshes its own qmstat row (1858) */
                int q = be_wq_num_unpinned_untargeted();
                S.qm_qlen[S.my_idx] = q;
                for (int i = 0; i < T; i++)
                    S.qm_hi[(long)S.my_idx * T + i] = be_wq_avail_hi_prio_of_type(S.user_types[i]);
                o[0] = -2;
                o[1] = a[0];
                o[2] = for_rank;
                n = 3;
            }
            break;
        }
        case ORC_OP_ROUND: {
            for (int i = 0; i < S.num_world; i++)
                S.rfr_out[i] = 0;
            for (int i = 0; i < S.num_app_ranks; i++)
                S.rfr_to_rank[i] = -1;
            n = 0;
            break;
        }
        case ORC_OP_RQLIST: {
            /* the rq in FIFO order (xq_first / xq_next over rq) */
            long k = 0;
            int rank, rqseqno, types[ORC_REQ_TYPES];
            for (void *r = be_rq_first(); r; r = be_rq_next(r)) {
                if (op + 2 + 18 * (k + 1) > outcap)
                    return -1;
                be_rq_view(r, &rank, &rqseqno, types);
                int *e = o + 1 + 18 * k;
                e[0] = rqseqno;
                e[1] = rank;
                memcpy(e + 2, types, sizeof(types));
                k++;
            }
            o[0] = (int)k;
            n = 1 + 18 * k;
            break;
        }
        case ORC_OP_INFOTYPE: {
            /* FA_INFO_NUM_WORK_UNITS, adlb.c:2466-2496 */
            int mx = ORC_LOWEST_PRIO, nmax = 0, ntot = 0;
            be_unit_view v;
            for (void *u = be_wq_first(); u; u = be_wq_next(u)) {
                be_wq_view(u, &v);
                if (v.work_type == a[0]) {
                    if (v.work_prio > mx)
                        mx = v.work_prio;
                    ntot++;
                }
            }
            for (void *u = be_wq_first(); u; u = be_wq_next(u)) {
                be_wq_view(u, &v);
                if (v.work_type == a[0] && v.work_prio == mx)
                    nmax++;
            }
            o[0] = mx; o[1] = nmax; o[2] = ntot;
            n = 3;
            break;
        }
        default:
            return -2;
        }
        out[op] = (int)n;
        op += 1 + n;
    }
    return op;
}
