/* adlb_mix.c -- an ADLB application that drives every server path.
 *
 * Written against the public API only (include/adlb/adlb.h), so the same
 * source builds against the reference library (oracle/Makefile: with the
 * message recorder, for fixtures) and against adlb_amd/libadlb.so (GPU run).
 *
 * Rank 0 puts n pairs of units, type A then type B: untargeted puts walk the
 * servers round robin, so with 2 servers every A lands on the first server
 * and every B on the second.  Apps served by the first server ask for B (and
 * the others for A), so their Reserves park and are settled by steals
 * (SS_RFR / SS_RFR_RESP).  Every 10th pair also carries a unit of type C
 * targeted at a worker, and one batch of type-D units shares a common prefix
 * (Begin/End_batch_put, FA_GET_COMMON).  Workers use Reserve, Ireserve,
 * Get_reserved_timed and Info_num_work_units; the job ends by exhaustion.
 * With -hi small, servers reject puts (PUT_REJECTED walk, puts of targeted
 * work away from the target's server: FA_DID_PUT_AT_REMOTE and the tq).
 *
 * With -ntypes K (K > 4) the servers declare K work types: the four above and
 * K - 4 more that no unit carries (K > 64: the engine's sorted-runs Reserve
 * path, and SS_RFR steals instead of the steal group's merge).
 *
 * Output (rank 0): "adlb_mix: units U sum S expect U' S'"; U == U' and
 * S == S' whatever the schedule.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <adlb/adlb.h>

enum { TA = 11, TB = 22, TC = 33, TD = 44 };

static void fill(int *w, int nw, int id, int type) {
    w[0] = id;
    w[1] = type;
    for (int k = 2; k < nw; k++) w[k] = id * 31 + k;
}

static int check(const int *w, int nw, int type) {
    if (w[1] != type) return 0;
    for (int k = 2; k < nw; k++)
        if (w[k] != w[0] * 31 + k) return 0;
    return 1;
}

int main(int argc, char **argv) {
    int nservers = 2, n = 200, len = 64, ndbatch = 8, ntypes = 4;
    double hi = 1e8;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "-nservers")) nservers = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-n")) n = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-len")) len = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-hi")) hi = atof(argv[++i]);
        else if (!strcmp(argv[i], "-ntypes")) ntypes = atoi(argv[++i]);
    }
    if (ntypes < 4) ntypes = 4;
    len = (len / 4 < 4 ? 4 : len / 4) * 4;
    const int nw = len / 4;
    /* the four carried types first, then declared-only ones (values below 10010: adlb.c:343-356) */
    int *types = malloc(sizeof(int) * (size_t)ntypes), am_server, am_debug;
    types[0] = TA, types[1] = TB, types[2] = TC, types[3] = TD;
    for (int k = 4; k < ntypes; k++) types[k] = 1000 + k;
    MPI_Comm app_comm;
    MPI_Init(&argc, &argv);
    int world, rank;
    MPI_Comm_size(MPI_COMM_WORLD, &world);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (ADLB_Init(nservers, 0, 0, ntypes, types, &am_server, &am_debug, &app_comm) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 1);
    if (am_server) {
        ADLB_Server(hi, 0.0);
        double hwm = 0, nrej = 0, pfrom = 0, pto = 0;
        ADLB_Info_get(ADLB_INFO_MALLOC_HWM, &hwm);
        ADLB_Info_get(ADLB_INFO_NPUSHED_FROM_HERE, &pfrom);
        ADLB_Info_get(ADLB_INFO_NPUSHED_TO_HERE, &pto);
        ADLB_Info_get(ADLB_INFO_NREJECTED_PUTS, &nrej);
        printf("server %d: malloc hwm %.0f pushed %.0f %.0f rejected puts %.0f\n", rank, hwm, pfrom, pto, nrej);
        ADLB_Finalize();
        MPI_Finalize();
        return 0;
    }
    int napps;
    MPI_Comm_size(app_comm, &napps);
    int *w = malloc((size_t)len + 64);
    long long sum = 0, expect_sum = 0;
    int units = 0, expect_units = 0;
    if (rank == 0) {
        for (int i = 0; i < n; i++) {
            fill(w, nw, 2 * i, TA);
            if (ADLB_Put(w, len, -1, 0, TA, i % 7) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 2);
            fill(w, nw, 2 * i + 1, TB);
            if (ADLB_Put(w, len, -1, 0, TB, (i * 3) % 5) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 2);
            expect_sum += (2 * i) * 10LL + TA + (2 * i + 1) * 10LL + TB;
            expect_units += 2;
            if (i % 10 == 0 && napps > 1) {  // targeted at a worker
                const int id = 100000 + i, target = 1 + (i / 10) % (napps - 1);
                fill(w, nw, id, TC);
                if (ADLB_Put(w, len, target, 0, TC, 5) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 2);
                expect_sum += id * 10LL + TC;
                expect_units++;
            }
        }
        // one batch sharing a common prefix: the unit is common (16 B) + unique part
        char common[16];
        memset(common, 'c', sizeof common);
        if (ADLB_Begin_batch_put(common, (int)sizeof common) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 3);
        for (int j = 0; j < ndbatch; j++) {
            fill(w, nw, 200000 + j, TD);
            if (ADLB_Put(w, len, -1, 0, TD, 2) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 3);
            expect_sum += (200000 + j) * 10LL + TD;
            expect_units++;
        }
        if (ADLB_End_batch_put() != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 3);
    }
    // apps served by the first server want B, the others A; everyone takes C and D
    const int first = (rank % nservers) == 0;
    int req[5] = {rank == 0 ? TA : (first ? TB : TA), TC, TD, rank == 0 ? TB : -1, -1};
    char *buf = malloc((size_t)len + 64);
    int steps = 0;
    while (1) {
        int type, prio, handle[ADLB_HANDLE_SIZE], wlen, answer, rc;
        if (++steps % 16 == 0) {
            int mp, nmp, nt;
            ADLB_Info_num_work_units(TA, &mp, &nmp, &nt);
            rc = ADLB_Ireserve(req, &type, &prio, handle, &wlen, &answer);
            if (rc == ADLB_NO_CURRENT_WORK) continue;
        } else {
            rc = ADLB_Reserve(req, &type, &prio, handle, &wlen, &answer);
        }
        if (rc == ADLB_DONE_BY_EXHAUSTION || rc == ADLB_NO_MORE_WORK) break;
        if (rc != ADLB_SUCCESS) {
            fprintf(stderr, "rank %d: reserve rc %d\n", rank, rc);
            MPI_Abort(MPI_COMM_WORLD, 4);
        }
        double qt = 0;
        if (ADLB_Get_reserved_timed(buf, handle, &qt) != ADLB_SUCCESS) MPI_Abort(MPI_COMM_WORLD, 5);
        const int *u = (const int *)(type == TD ? buf + 16 : buf);
        if (type == TD && (wlen != len + 16 || buf[0] != 'c' || buf[15] != 'c')) MPI_Abort(MPI_COMM_WORLD, 6);
        if (!check(u, nw, type)) {
            fprintf(stderr, "rank %d: corrupt unit type %d id %d\n", rank, type, u[0]);
            MPI_Abort(MPI_COMM_WORLD, 7);
        }
        units++;
        sum += u[0] * 10LL + type;
    }
    long long tot[2] = {units, sum}, all[2];
    MPI_Reduce(tot, all, 2, MPI_LONG_LONG, MPI_SUM, 0, app_comm);
    if (rank == 0) printf("adlb_mix: units %lld sum %lld expect %d %lld\n", all[0], all[1], expect_units, expect_sum);
    free(w);
    free(buf);
    free(types);
    ADLB_Finalize();
    MPI_Finalize();
    return 0;
}
