/* adlb_push.c -- an ADLB application that makes a server push work.
 *
 * Public API only (include/adlb/adlb.h).  With 2 servers, targeted Puts go to
 * the target rank's server (rank % 2), so rank 0 putting n units targeted at
 * rank 2 fills the first server alone.  Past 0.95 x the ADLB_Server memory
 * limit (-hi) that server pushes its first unpinned unit to the other server
 * (SS_PUSH_QUERY / _RESP / _HDR / _WORK; adlb.c:509-556, 2109-2362), which
 * reports the targeted unit back to its home (SS_MOVING_TARGETED_WORK), so
 * rank 2's Reserves at home are steered there by the tq (SS_RFR).  Rank 2
 * takes all n units; ranks 1 and 3 wait on a type nobody puts; rank 2 ends
 * the job with ADLB_Set_no_more_work.
 *
 * Output: each server "server R: pushed FROM TO", then rank 0
 * "adlb_push: units U sum S expect U' S'" (U == U', S == S').
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <adlb/adlb.h>

enum { TW = 5, TNONE = 6 };

int main(int argc, char **argv) {
    int n = 300, len = 1000;
    double hi = 80000;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-n")) n = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-len")) len = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-hi")) hi = atof(argv[++i]);
    }
    int types[2] = {TW, TNONE}, am_server = 0, am_debug = 0;
    MPI_Comm app_comm;
    MPI_Init(&argc, &argv);
    int rank;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (ADLB_Init(2, 0, 0, 2, types, &am_server, &am_debug, &app_comm) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 1);
    if (am_server) {
        ADLB_Server(hi, 0.0);
        double pfrom = 0, pto = 0;
        ADLB_Info_get(ADLB_INFO_NPUSHED_FROM_HERE, &pfrom);
        ADLB_Info_get(ADLB_INFO_NPUSHED_TO_HERE, &pto);
        printf("server %d: pushed %.0f %.0f\n", rank, pfrom, pto);
        ADLB_Finalize();
        MPI_Finalize();
        return 0;
    }
    const int nw = len / (int)sizeof(int);
    int *w = malloc((size_t)len + 64);
    long long sum = 0, expect = 0;
    int units = 0;
    if (rank == 0) {
        for (int i = 0; i < n; i++) {
            w[0] = i;
            for (int k = 1; k < nw; k++) w[k] = i * 7 + k;
            if (ADLB_Put(w, len, 2, 0, TW, i % 13) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 2);
        }
    }
    for (int i = 0; i < n; i++) expect += i;
    if (rank == 2) {
        int req[2] = {TW, -1};
        while (units < n) {
            int type, prio, handle[ADLB_HANDLE_SIZE], wlen, answer;
            const int rc = ADLB_Reserve(req, &type, &prio, handle, &wlen, &answer);
            if (rc != ADLB_SUCCESS) {
                fprintf(stderr, "rank 2: reserve rc %d after %d units\n", rc, units);
                MPI_Abort(MPI_COMM_WORLD, 3);
            }
            if (ADLB_Get_reserved(w, handle) != ADLB_SUCCESS || wlen != len) MPI_Abort(MPI_COMM_WORLD, 4);
            for (int k = 1; k < nw; k++)
                if (w[k] != w[0] * 7 + k) {
                    fprintf(stderr, "rank 2: corrupt unit %d\n", w[0]);
                    MPI_Abort(MPI_COMM_WORLD, 5);
                }
            units++;
            sum += w[0];
        }
        ADLB_Set_no_more_work();
    } else if (rank != 0) {
        int req[2] = {TNONE, -1};
        int type, prio, handle[ADLB_HANDLE_SIZE], wlen, answer;
        const int rc = ADLB_Reserve(req, &type, &prio, handle, &wlen, &answer);
        if (rc != ADLB_NO_MORE_WORK && rc != ADLB_DONE_BY_EXHAUSTION) MPI_Abort(MPI_COMM_WORLD, 6);
    }
    long long tot[2] = {units, sum}, all[2];
    MPI_Reduce(tot, all, 2, MPI_LONG_LONG, MPI_SUM, 0, app_comm);
    if (rank == 0) printf("adlb_push: units %lld sum %lld expect %d %lld\n", all[0], all[1], n, expect);
    free(w);
    ADLB_Finalize();
    MPI_Finalize();
    return 0;
}
