/* adlb_deep.c -- a matching-dominated ADLB application: a deep queue.
 *
 * Written against the public API only (include/adlb/adlb.h), so the same
 * source builds against the reference library (oracle/Makefile: _ref/deep_plain)
 * and against adlb_amd/libadlb.so (tests/apps/Makefile).
 *
 * Every app puts n / napps units of its own type (one of four, by app rank)
 * with priorities spread over [0, 1000); after a barrier every unit is queued
 * on the (one) server, and every app takes back n / napps units of the type
 * of the next app by Reserve + Get_reserved.  Each Reserve is served from a
 * queue of up to n units: the reference scans its xq list for the best unit
 * of the type (xq.c:190-217), the engine matches the Reserves that wait at
 * the server together on the GPU.  Every app knows how many units it takes,
 * so the job ends without exhaustion detection; the timed part is the
 * Reserve/Get phase (MPI_Wtime on rank 0 between two barriers).
 *
 * Output (rank 0): "adlb_deep: units U sum S expect U' S' reserve_s T".
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <adlb/adlb.h>

static const int TYPES[4] = {11, 22, 33, 44};

int main(int argc, char **argv) {
    int n = 40000, len = 16;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-n")) n = atoi(argv[++i]);
    }
    int types[4] = {TYPES[0], TYPES[1], TYPES[2], TYPES[3]}, am_server, am_debug;
    MPI_Comm app_comm;
    MPI_Init(&argc, &argv);
    int rank;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (ADLB_Init(1, 0, 0, 4, types, &am_server, &am_debug, &app_comm) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 1);
    if (am_server) {
        ADLB_Server(1e9, 0.0);
        ADLB_Finalize();
        MPI_Finalize();
        return 0;
    }
    int napps, me;
    MPI_Comm_size(app_comm, &napps);
    MPI_Comm_rank(app_comm, &me);
    const int per = n / napps, mytype = TYPES[me % 4], want = TYPES[(me + 1) % 4];
    int w[4];
    long long sum = 0, expect = 0;
    unsigned int seed = 12345u + 7919u * (unsigned int)me;
    for (int i = 0; i < per; i++) {
        seed = seed * 1103515245u + 12345u;
        const int prio = (int)((seed >> 8) % 1000u);
        w[0] = me * per + i;
        w[1] = mytype;
        w[2] = prio;
        w[3] = 0;
        if (ADLB_Put(w, len, -1, me, mytype, prio) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 2);
        expect += w[0];
    }
    MPI_Barrier(app_comm);
    const double t0 = MPI_Wtime();
    /* the apps of type (me + 1) % 4 put per units each; the apps that want them share them */
    int nput = 0, nwant = 0;
    for (int a = 0; a < napps; a++) {
        nput += TYPES[a % 4] == want;
        nwant += TYPES[(a + 1) % 4] == want;
    }
    int rank_in = 0;
    for (int a = 0; a < me; a++) rank_in += TYPES[(a + 1) % 4] == want;
    const int total = nput * per, take = total / nwant + (rank_in < total % nwant ? 1 : 0);
    int req[2] = {want, -1};
    int got = 0;
    for (int k = 0; k < take; k++) {
        int type, prio, handle[ADLB_HANDLE_SIZE], wlen, answer;
        const int rc = ADLB_Reserve(req, &type, &prio, handle, &wlen, &answer);
        if (rc != ADLB_SUCCESS) {
            fprintf(stderr, "app %d: reserve rc %d after %d\n", me, rc, k);
            MPI_Abort(MPI_COMM_WORLD, 3);
        }
        if (ADLB_Get_reserved(w, handle) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 4);
        if (w[1] != type || type != want || w[2] != prio) MPI_Abort(MPI_COMM_WORLD, 5);
        sum += w[0];
        got++;
    }
    MPI_Barrier(app_comm);
    const double t1 = MPI_Wtime();
    long long loc[3] = {got, sum, expect}, all[3];
    MPI_Reduce(loc, all, 3, MPI_LONG_LONG, MPI_SUM, 0, app_comm);
    if (me == 0)
        printf("adlb_deep: units %lld sum %lld expect %d %lld reserve_s %.4f\n", all[0], all[1], per * napps, all[2],
               t1 - t0);
    ADLB_Finalize();
    MPI_Finalize();
    return 0;
}
