/*
 * oracle/gen_c5.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The config-5 stream of SURVEY §8(d) at its full shape: a tsp.c-style
 * branch-and-bound workload over S server shards, driven against the repo's
 * clean-room restatement (liboracle.so, one private copy per shard) so that
 * every event's expected output is known:
 *
 *   * work units: type W untargeted, prio = 1 + len (tsp.c:240-241), Put
 *     round robin over the servers from the putter's home (adlb.c:2771-2773);
 *   * bound updates: type B targeted at a rank, prio 999999999 (tsp.c:17,
 *     189-193, 251-252), Put to the target's home server (adlb.c:2767-2768);
 *   * Reserves ask for {B, W} (tsp.c:157-161), some for {W} or the wildcard,
 *     a tenth without hang; a matched unit is fetched with a Get (tsp.c:162)
 *     on the server that holds it, and the worker Puts its children;
 *   * every `round_every` events (all shards together): a qmstat snapshot
 *     (each shard's update_local_state row, adlb.c:3581-3593, sent to every
 *     other shard) and a steal round: the parked Reserves of shard 0, 1, ...
 *     in rqseqno order, each against the donors' current rows, the donor's
 *     SS_RFR (adlb.c:1802-1866) and the requester's rq_delete (1868-1933),
 *     one exchange at a time.  A round first clears every shard's outstanding
 *     RFR record (the answers the round replaces, adlb.c:1877-1878).
 *
 * The round is the one adlbq_steal_group_settle performs: it stops at the
 * first Reserve whose decision would need a unit below some shard's exported
 * top k of a type (adlbq_steal.hip, merge_views), and so does this
 * generator, so the two are comparable event for event.
 *
 * Output per shard: the event trace (oracle/replay.h format; a round is the
 * 0-argument event ORC_OP_ROUND at the same place in every shard's trace)
 * and the oracle's outputs; per round, the steals as rows of 15 ints
 * {shard, rqseqno, rank, TA_RESERVE_RESP[12]}, in serial order.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "be.h"
#include "replay.h"

#define T_W 1
#define T_B 2
#define NT 2
#define BOUND_PRIO 999999999

typedef struct {
    int *p;
    long n, cap;
} Vec;

static void vpush(Vec *v, const int *x, long k) {
    if (v->n + k > v->cap) {
        long c = v->cap ? v->cap : 1024;
        while (c < v->n + k) c *= 2;
        v->p = (int *)realloc(v->p, sizeof(int) * c);
        v->cap = c;
    }
    memcpy(v->p + v->n, x, sizeof(int) * k);
    v->n += k;
}

typedef struct {
    void *dl;
    int (*init)(int, const int *, int, int, int);
    long (*replay)(const int *, long, int *, long);
    void *(*wq_first)(void);
    void *(*wq_next)(void *);
    void (*wq_view)(void *, be_unit_view *);
    Vec tr, out;  /* the shard's trace and the oracle's outputs */
    Vec xtr;      /* the trace plus this shard's part of every steal round (its SS_RFR answers as donor, its
                     rq deletions as requester): what one server process replays alone (bench cpu baseline) */
    Vec pend;     /* Puts addressed to this shard, not yet issued */
    long live;    /* units held (model bookkeeping for the queue level) */
} Shard;

enum { IDLE = 0, HOLD = 1, PARKED = 2 };
typedef struct {
    int state, shard, seq;  /* HOLD: (shard, wqseqno); PARKED: (home shard, rqseqno) */
    int next_put;           /* the server its next untargeted Put goes to (adlb.c:377, 2771-2773) */
} Rank;

typedef struct C5 {
    int S, A, k, q0;
    Shard *sh;
    Rank *rk;
    Vec steals;       /* rows of 15 */
    Vec round_nsteal; /* steals per round */
    long events, rounds, stopped;
    double seconds;
    uint64_t rng;
    char err[256];
} C5;

static uint64_t nxt(C5 *g) { /* splitmix64 */
    uint64_t z = (g->rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double unif(C5 *g) { return (double)(nxt(g) >> 11) * (1.0 / 9007199254740992.0); }
static int below(C5 *g, int n) { return (int)(unif(g) * n); }

static const int UT[NT] = {T_W, T_B};

/* one event (or a run of same-op events) on shard s: appended to its trace,
 * replayed, outputs appended; returns the first output int of this call */
static int *issue(C5 *g, int s, const int *ev, long nint, long *nout) {
    Shard *h = &g->sh[s];
    long cap = 64 + 4 * nint + 4096;
    static int *ob = NULL;
    static long obcap = 0;
    if (cap > obcap) {
        obcap = cap * 2;
        ob = (int *)realloc(ob, sizeof(int) * obcap);
    }
    long n = h->replay(ev, nint, ob, obcap);
    if (n < 0) {
        snprintf(g->err, sizeof g->err, "oracle rejected an event on shard %d (rc %ld)", s, n);
        return NULL;
    }
    vpush(&h->tr, ev, nint);
    vpush(&h->xtr, ev, nint);
    long o0 = h->out.n;
    vpush(&h->out, ob, n);
    *nout = n;
    return h->out.p + o0;
}

/* a query on shard s that is not part of its trace (the round's fresh rows) */
static long query(C5 *g, int s, const int *ev, long nint, int *o, long cap) { return g->sh[s].replay(ev, nint, o, cap); }

static int put_ev(int *e, int type, int prio, int answer, int target, int len, int home) {
    e[0] = ORC_OP_PUT;
    e[1] = type; e[2] = prio; e[3] = answer; e[4] = target; e[5] = len; e[6] = home;
    e[7] = 0; e[8] = -1; e[9] = -1;
    return 10;
}

/* issue shard s's pending Puts as one run; a Put that matched a parked
 * Reserve (put-side FIFO match) hands the unit to that rank */
static int flush_puts(C5 *g, int s) {
    Shard *h = &g->sh[s];
    if (!h->pend.n) return 0;
    long nout = 0;
    int *o = issue(g, s, h->pend.p, h->pend.n, &nout);
    if (!o) return -1;
    long ne = h->pend.n / 10;
    g->events += ne;
    h->live += ne;
    for (long i = 0; i < ne; i++) {
        const int *r = o + 4 * i;  /* [3, wqseqno, rank, rqseqno] */
        if (r[2] >= 0) {
            Rank *x = &g->rk[r[2]];
            x->state = HOLD;
            x->shard = s;
            x->seq = r[1];
        }
    }
    h->pend.n = 0;
    return 0;
}

/* a finished worker's Puts: children of the work unit it took, and now and then bound updates */
static void worker_puts(C5 *g, int r) {
    Rank *x = &g->rk[r];
    const int home = r % g->S;
    int e[10];
    Shard *hs = &g->sh[x->next_put];
    /* keep each shard's queue near q0: fewer children when it is fuller */
    double m = 1.0 + 0.6 * ((double)g->q0 - (double)hs->live) / (double)g->q0;
    if (m < 0.4) m = 0.4;
    if (m > 1.6) m = 1.6;
    int nc = (unif(g) < m - (int)m) + (int)m + (unif(g) < 0.5 ? 0 : (unif(g) < 0.5 ? -1 : 1));
    if (nc < 0) nc = 0;
    for (int c = 0; c < nc; c++) {
        const int len = 4 + below(g, 56);
        const int to = x->next_put;
        put_ev(e, T_W, 1 + len, r, -1, len, home);
        vpush(&g->sh[to].pend, e, 10);
        x->next_put = (x->next_put + 1) % g->S;
    }
    if (unif(g) < 0.15) {
        const int nb = 1 + below(g, 2);
        for (int b = 0; b < nb; b++) {
            const int tgt = below(g, g->A);
            put_ev(e, T_B, BOUND_PRIO, r, tgt, 8, tgt % g->S);
            vpush(&g->sh[tgt % g->S].pend, e, 10);
        }
    }
}

/* the qmstat snapshot and the steal round (see the header) */
static int steal_round(C5 *g) {
    const int S = g->S;
    int *rows = (int *)malloc(sizeof(int) * S * (1 + NT));
    int ev[64];
    const long ocap = 64 + 18l * g->A;  /* the longest rq list: every rank parked */
    int *o = (int *)malloc(sizeof(int) * ocap);
    long nout;
    /* 1. every shard's row (in its trace), then every other shard's row set (in its trace) */
    for (int s = 0; s < S; s++) {
        ev[0] = ORC_OP_QMROW;
        int *r = issue(g, s, ev, 1, &nout);
        if (!r) return -1;
        memcpy(rows + s * (1 + NT), r + 1, sizeof(int) * (1 + NT));
        g->events++;
    }
    for (int s = 0; s < S; s++)
        for (int j = 0; j < S; j++) {
            if (j == s) continue;
            ev[0] = ORC_OP_SETROW;
            ev[1] = j;
            ev[2] = rows[j * (1 + NT)];
            ev[3] = 0;
            memcpy(ev + 4, rows + j * (1 + NT) + 1, sizeof(int) * NT);
            if (!issue(g, s, ev, 4 + NT, &nout)) return -1;
            g->events++;
        }
    /* 2. the round marker: every shard's outstanding RFR records cleared */
    for (int s = 0; s < S; s++) {
        ev[0] = ORC_OP_ROUND;
        if (!issue(g, s, ev, 1, &nout)) return -1;
    }
    /* 3. the exported top k per (shard, type): available = untargeted, unpinned, prio above LOWEST */
    long *avail = (long *)calloc((size_t)S * NT, sizeof(long));
    int *granted = (int *)calloc((size_t)S * NT, sizeof(int));
    for (int s = 0; s < S; s++) {
        Shard *h = &g->sh[s];
        be_unit_view v;
        for (void *u = h->wq_first(); u; u = h->wq_next(u)) {
            h->wq_view(u, &v);
            if (v.target_rank < 0 && !v.pinned && v.work_prio > ORC_LOWEST_PRIO)
                avail[s * NT + (v.work_type == T_W ? 0 : 1)]++;
        }
    }
#define UNK(s, t) (granted[(s) * NT + (t)] >= g->k && avail[(s) * NT + (t)] > g->k)
    long nst = 0;
    int stop = 0;
    for (int i = 0; i < S && !stop; i++) {
        ev[0] = ORC_OP_RQLIST;
        long n = query(g, i, ev, 1, o, ocap);
        if (n < 0) {
            snprintf(g->err, sizeof g->err, "rq list of shard %d too long", i);
            return -1;
        }
        const int k = o[1];
        int *lst = (int *)malloc(sizeof(int) * 18 * (k > 0 ? k : 1));
        memcpy(lst, o + 2, sizeof(int) * 18 * k);
        for (int e = 0; e < k && !stop; e++) {
            const int rqs = lst[18 * e], rank = lst[18 * e + 1];
            const int *types = lst + 18 * e + 2;
            /* fresh rows of every shard (the merge sees every earlier steal) */
            for (int s = 0; s < S; s++) {
                ev[0] = ORC_OP_QMROW;
                int q[16];
                if (query(g, s, ev, 1, q, 16) < 0) return -1;
                memcpy(rows + s * (1 + NT), q + 1, sizeof(int) * (1 + NT));
            }
            /* find_cand over the type vector in order (adlb.c:1280-1308, 3487-3534) */
            int donor = -1;
            for (int x = 0; x < ORC_REQ_TYPES && donor < 0 && !stop; x++) {
                const int v = types[x];
                if (v < -1) break;
                int tl[NT], nt = 0;
                if (v == -1) {
                    tl[nt++] = 0;
                    tl[nt++] = 1;
                } else if (v == T_W || v == T_B) {
                    tl[nt++] = v == T_W ? 0 : 1;
                } else {
                    continue;
                }
                for (int a = 0; a < nt; a++)
                    for (int s = 0; s < S; s++)
                        if (s != i && UNK(s, tl[a])) stop = 1;
                if (stop) break;
                int best = -1, hi = ORC_LOWEST_PRIO;
                for (int s = 0; s < S; s++) {
                    if (s == i || rows[s * (1 + NT)] <= 0) continue;
                    for (int a = 0; a < nt; a++) {
                        const int h = rows[s * (1 + NT) + 1 + tl[a]];
                        if (h > hi) hi = h, best = s;
                    }
                }
                donor = best;
            }
            if (stop) break;
            if (donor < 0) continue;
            /* the donor's unit over the request's whole set: stop if a list of the set is past its export */
            int set = 0;
            for (int x = 0; x < ORC_REQ_TYPES; x++) {
                const int v = types[x];
                if (v < -1) break;
                if (v == -1) set = 3;
                else if (v == T_W) set |= 1;
                else if (v == T_B) set |= 2;
            }
            for (int t = 0; t < NT; t++)
                if (((set >> t) & 1) && UNK(donor, t)) stop = 1;
            if (stop) break;
            ev[0] = ORC_OP_RFR;
            ev[1] = rqs;
            ev[2] = rank;
            memcpy(ev + 3, types, sizeof(int) * ORC_REQ_TYPES);
            int rr[32];
            if (query(g, donor, ev, 3 + ORC_REQ_TYPES, rr, 32) < 0 || rr[0] != 12 || rr[1] != 1) {
                snprintf(g->err, sizeof g->err, "a donor chosen on a fresh table had no unit (shard %d)", donor);
                return -1;
            }
            vpush(&g->sh[donor].xtr, ev, 3 + ORC_REQ_TYPES);
            ev[0] = ORC_OP_RQDEL;
            ev[1] = rqs;
            vpush(&g->sh[i].xtr, ev, 2);
            int dd[16];
            if (query(g, i, ev, 2, dd, 16) < 0 || dd[1] != 1) {
                snprintf(g->err, sizeof g->err, "steal of an rq entry that is gone (shard %d)", i);
                return -1;
            }
            const int *x = rr + 1;  /* SS_RFR_RESP {1, rqseqno, rank, type, prio, len, answer, wqseqno, prev_target, clen, csrv, cseq} */
            granted[donor * NT + (x[3] == T_W ? 0 : 1)]++;
            int row[15] = {i, rqs, rank, 1, x[3], x[4], x[5], x[6], x[7], g->A + donor, x[9], x[10], x[11], -1, -1};
            vpush(&g->steals, row, 15);
            nst++;
            Rank *rk = &g->rk[rank];
            rk->state = HOLD;
            rk->shard = donor;
            rk->seq = x[7];
        }
        free(lst);
    }
#undef UNK
    if (stop) g->stopped++;
    int ns = (int)nst;
    vpush(&g->round_nsteal, &ns, 1);
    g->rounds++;
    free(avail);
    free(granted);
    free(rows);
    free(o);
    return 0;
}

/* one model step on shard s: its pending Puts, the Gets of the ranks holding
 * its units (each then Puts children), the Reserves of some of its idle ranks */
static int shard_step(C5 *g, int s) {
    if (flush_puts(g, s)) return -1;
    /* Gets */
    Vec ev = {0}, who = {0};
    for (int r = 0; r < g->A; r++) {
        Rank *x = &g->rk[r];
        if (x->state != HOLD || x->shard != s) continue;
        int e[3] = {ORC_OP_GET, r, x->seq};
        vpush(&ev, e, 3);
        vpush(&who, &r, 1);
    }
    if (ev.n) {
        long nout;
        int *o = issue(g, s, ev.p, ev.n, &nout);
        if (!o) return -1;
        g->events += who.n;
        g->sh[s].live -= who.n;
        for (long i = 0; i < who.n; i++) {
            const int r = who.p[i];
            const int *q = o + 6 * i;  /* [5, rc, len, type, prio, answer] */
            g->rk[r].state = IDLE;
            if (q[1] == 1 && q[3] == T_W) worker_puts(g, r);
        }
    }
    ev.n = who.n = 0;
    /* Reserves: about half of the idle ranks of this home shard */
    for (int r = s; r < g->A; r += g->S) {
        Rank *x = &g->rk[r];
        if (x->state != IDLE || unif(g) < 0.5) continue;
        int e[2 + 1 + ORC_REQ_TYPES];
        e[0] = ORC_OP_RESERVE;
        e[1] = r;
        e[2] = unif(g) < 0.9;
        for (int k = 0; k < ORC_REQ_TYPES; k++) e[3 + k] = -2;
        const double u = unif(g);
        if (u < 0.75) e[3] = T_B, e[4] = T_W;
        else if (u < 0.9) e[3] = T_W;
        else e[3] = -1;
        vpush(&ev, e, 3 + ORC_REQ_TYPES);
        vpush(&who, &r, 1);
    }
    if (ev.n) {
        long nout;
        int *o = issue(g, s, ev.p, ev.n, &nout);
        if (!o) return -1;
        g->events += who.n;
        for (long i = 0; i < who.n; i++) {
            const int r = who.p[i];
            const int *q = o + (1 + ORC_RESP_INTS) * i + 1;
            Rank *x = &g->rk[r];
            if (q[0] == 1) {
                x->state = HOLD;
                x->shard = s;
                x->seq = q[5];
            } else if (q[0] == 0) {
                x->state = PARKED;
                x->shard = s;
                x->seq = q[10];
            }
        }
    }
    free(ev.p);
    free(who.p);
    return 0;
}

C5 *c5_new(const char *liboracle, int S, int A, int k, int q0, unsigned long long seed) {
    C5 *g = (C5 *)calloc(1, sizeof(C5));
    g->S = S, g->A = A, g->k = k, g->q0 = q0;
    g->rng = seed * 0x9E3779B97F4A7C15ull + 12345;
    g->sh = (Shard *)calloc(S, sizeof(Shard));
    g->rk = (Rank *)calloc(A, sizeof(Rank));
    for (int s = 0; s < S; s++) {
        /* a private copy per shard: the oracle keeps one server's queues in globals */
        char tmpl[] = "/tmp/orc_c5_XXXXXX";
        int fd = mkstemp(tmpl);
        FILE *in = fopen(liboracle, "rb");
        if (fd < 0 || !in) {
            snprintf(g->err, sizeof g->err, "cannot copy %s", liboracle);
            return g;
        }
        char buf[65536];
        size_t m;
        while ((m = fread(buf, 1, sizeof buf, in)) > 0)
            if (write(fd, buf, m) != (ssize_t)m) break;
        fclose(in);
        close(fd);
        Shard *h = &g->sh[s];
        h->dl = dlopen(tmpl, RTLD_NOW | RTLD_LOCAL);
        unlink(tmpl);
        if (!h->dl) {
            snprintf(g->err, sizeof g->err, "dlopen: %s", dlerror());
            return g;
        }
        h->init = (int (*)(int, const int *, int, int, int))dlsym(h->dl, "orc_init");
        h->replay = (long (*)(const int *, long, int *, long))dlsym(h->dl, "orc_replay");
        h->wq_first = (void *(*)(void))dlsym(h->dl, "be_wq_first");
        h->wq_next = (void *(*)(void *))dlsym(h->dl, "be_wq_next");
        h->wq_view = (void (*)(void *, be_unit_view *))dlsym(h->dl, "be_wq_view");
        if (!h->init || !h->replay || !h->wq_first || !h->wq_next || !h->wq_view || h->init(NT, UT, A, S, s)) {
            snprintf(g->err, sizeof g->err, "oracle copy %d: missing symbols or init failed", s);
            return g;
        }
    }
    for (int r = 0; r < A; r++) g->rk[r].next_put = r % S;
    return g;
}

const char *c5_error(C5 *g) { return g->err; }

/* the stream: seed units, then model steps over the shards in turn, a round
 * every round_every events, until n_events have been issued */
int c5_run(C5 *g, long n_events, long round_every, int seed_units) {
    if (g->err[0]) return -1;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int e[10];
    /* the root tasks on one server (tsp.c: rank 0 puts the first work), so the
     * other servers' ranks start parked and the first rounds steal */
    for (int i = 0; i < seed_units; i++) {
        const int len = 4 + below(g, 36);
        put_ev(e, T_W, 1 + len, 0, -1, len, 0);
        vpush(&g->sh[0].pend, e, 10);
    }
    long next_round = round_every;
    int s = 0;
    while (g->events < n_events) {
        if (shard_step(g, s)) return -1;
        s = (s + 1) % g->S;
        if (g->events >= next_round) {
            for (int q = 0; q < g->S; q++)
                if (flush_puts(g, q)) return -1;
            if (steal_round(g)) return -1;
            next_round = g->events + round_every;
        }
    }
    for (int q = 0; q < g->S; q++)
        if (flush_puts(g, q)) return -1;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    g->seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return 0;
}

long c5_events(C5 *g) { return g->events; }
long c5_rounds(C5 *g) { return g->rounds; }
long c5_stopped(C5 *g) { return g->stopped; }
double c5_seconds(C5 *g) { return g->seconds; }
long c5_trace(C5 *g, int s, const int **p) { *p = g->sh[s].tr.p; return g->sh[s].tr.n; }
long c5_out(C5 *g, int s, const int **p) { *p = g->sh[s].out.p; return g->sh[s].out.n; }
long c5_xtrace(C5 *g, int s, const int **p) { *p = g->sh[s].xtr.p; return g->sh[s].xtr.n; }
long c5_steals(C5 *g, const int **p) { *p = g->steals.p; return g->steals.n / 15; }
long c5_round_nsteal(C5 *g, const int **p) { *p = g->round_nsteal.p; return g->round_nsteal.n; }

void c5_free(C5 *g) {
    if (!g) return;
    for (int s = 0; s < g->S; s++) {
        free(g->sh[s].tr.p);
        free(g->sh[s].out.p);
        free(g->sh[s].xtr.p);
        free(g->sh[s].pend.p);
        if (g->sh[s].dl) dlclose(g->sh[s].dl);
    }
    free(g->sh);
    free(g->rk);
    free(g->steals.p);
    free(g->round_nsteal.p);
    free(g);
}
