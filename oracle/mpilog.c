/* oracle/mpilog.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A PMPI message recorder linked into the reference build of an example
 * (oracle/Makefile target `nqref`): every point-to-point message a rank sends
 * or receives is appended to $ADLB_MSGLOG_DIR/rank<world rank>.bin in the
 * order the rank's code saw it.  tests/golden/gen_nq.py turns the server
 * ranks' logs into the config-1 fixtures (the reference server's inbound
 * event stream plus what it answered), which tests/test_gpu_server.py
 * replays through the repo's own server core.
 *
 * Record: int32 {dir (0 recv, 1 send), peer world rank, tag, comm (0 world-
 * sized, 1 other), nbytes} followed by the payload padded to 4 bytes.
 *
 * Hooked: MPI_Send/Ssend/Rsend/Isend/Issend (logged when posted: the buffer
 * is final then), MPI_Recv, MPI_Irecv completed by MPI_Wait, and PMPI_Test,
 * which the reference server calls directly on its qmstat receive
 * (adlb.c:864); that one is interposed and forwarded with dlsym(RTLD_NEXT).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static FILE *logf_;
static int inited_;

static void log_open(void) {
    if (inited_) return;
    inited_ = 1;
    const char *dir = getenv("ADLB_MSGLOG_DIR");
    if (!dir) return;
    int r;
    PMPI_Comm_rank(MPI_COMM_WORLD, &r);
    char path[4096];
    snprintf(path, sizeof path, "%s/rank%d.bin", dir, r);
    logf_ = fopen(path, "wb");
}

static int world_rank_of(MPI_Comm comm, int r) {
    if (r < 0) return r;
    MPI_Group g, w;
    int out = r;
    PMPI_Comm_group(comm, &g);
    PMPI_Comm_group(MPI_COMM_WORLD, &w);
    PMPI_Group_translate_ranks(g, 1, &r, w, &out);
    PMPI_Group_free(&g);
    PMPI_Group_free(&w);
    return out;
}

static void rec(int dir, int peer, int tag, MPI_Comm comm, const void *buf, int nbytes) {
    log_open();
    if (!logf_) return;
    int ws, cs;
    PMPI_Comm_size(MPI_COMM_WORLD, &ws);
    PMPI_Comm_size(comm, &cs);
    int h[5] = {dir, world_rank_of(comm, peer), tag, cs == ws ? 0 : 1, nbytes};
    fwrite(h, sizeof h, 1, logf_);
    if (nbytes > 0) fwrite(buf, 1, (size_t)nbytes, logf_);
    static const char pad[4];
    if (nbytes & 3) fwrite(pad, 1, (size_t)(4 - (nbytes & 3)), logf_);
    fflush(logf_);
}

static int type_bytes(MPI_Datatype dt, int count) {
    int sz = 1;
    PMPI_Type_size(dt, &sz);
    return sz * count;
}

static void rec_status(MPI_Comm comm, const void *buf, const MPI_Status *st) {
    int n = 0;
    PMPI_Get_count(st, MPI_BYTE, &n);
    rec(0, st->MPI_SOURCE, st->MPI_TAG, comm, buf, n);
}

/* outstanding receives: request -> (buffer, comm) */
#define NPEND 256
static struct { MPI_Request req; const void *buf; MPI_Comm comm; } pend_[NPEND];

static void pend_add(MPI_Request r, const void *buf, MPI_Comm comm) {
    for (int i = 0; i < NPEND; i++)
        if (pend_[i].req == MPI_REQUEST_NULL || pend_[i].buf == NULL) {
            pend_[i].req = r, pend_[i].buf = buf, pend_[i].comm = comm;
            return;
        }
}

static int pend_take(MPI_Request r, const void **buf, MPI_Comm *comm) {
    for (int i = 0; i < NPEND; i++)
        if (pend_[i].buf && pend_[i].req == r) {
            *buf = pend_[i].buf, *comm = pend_[i].comm;
            pend_[i].buf = NULL;
            return 1;
        }
    return 0;
}

int MPI_Send(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm) {
    rec(1, dest, tag, comm, buf, type_bytes(dt, count));
    return PMPI_Send(buf, count, dt, dest, tag, comm);
}

int MPI_Ssend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm) {
    rec(1, dest, tag, comm, buf, type_bytes(dt, count));
    return PMPI_Ssend(buf, count, dt, dest, tag, comm);
}

int MPI_Rsend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm) {
    rec(1, dest, tag, comm, buf, type_bytes(dt, count));
    return PMPI_Rsend(buf, count, dt, dest, tag, comm);
}

int MPI_Isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *r) {
    rec(1, dest, tag, comm, buf, type_bytes(dt, count));
    return PMPI_Isend(buf, count, dt, dest, tag, comm, r);
}

int MPI_Issend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *r) {
    rec(1, dest, tag, comm, buf, type_bytes(dt, count));
    return PMPI_Issend(buf, count, dt, dest, tag, comm, r);
}

int MPI_Recv(void *buf, int count, MPI_Datatype dt, int src, int tag, MPI_Comm comm, MPI_Status *st) {
    MPI_Status s;
    const int rc = PMPI_Recv(buf, count, dt, src, tag, comm, &s);
    rec_status(comm, buf, &s);
    if (st != MPI_STATUS_IGNORE) *st = s;
    return rc;
}

int MPI_Irecv(void *buf, int count, MPI_Datatype dt, int src, int tag, MPI_Comm comm, MPI_Request *r) {
    const int rc = PMPI_Irecv(buf, count, dt, src, tag, comm, r);
    pend_add(*r, buf, comm);
    return rc;
}

int MPI_Wait(MPI_Request *r, MPI_Status *st) {
    const MPI_Request r0 = *r;
    MPI_Status s;
    const int rc = PMPI_Wait(r, &s);
    const void *buf;
    MPI_Comm comm;
    if (pend_take(r0, &buf, &comm)) rec_status(comm, buf, &s);
    if (st != MPI_STATUS_IGNORE) *st = s;
    return rc;
}

int PMPI_Test(MPI_Request *r, int *flag, MPI_Status *st) {
    static int (*real)(MPI_Request *, int *, MPI_Status *);
    if (!real) real = (int (*)(MPI_Request *, int *, MPI_Status *))dlsym(RTLD_NEXT, "PMPI_Test");
    const MPI_Request r0 = *r;
    MPI_Status s;
    const int rc = real(r, flag, &s);
    const void *buf;
    MPI_Comm comm;
    if (*flag && pend_take(r0, &buf, &comm)) rec_status(comm, buf, &s);
    if (st != MPI_STATUS_IGNORE) *st = s;
    return rc;
}
