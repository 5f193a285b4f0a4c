/* adlb_fcall.c -- an ADLB application driven through the Fortran entry points.
 *
 * No Fortran compiler ships in this image, so this C program calls the
 * symbols exactly as compiled Fortran would: lower-case name + '_', every
 * argument by reference, status in the trailing ierr, the communicator as an
 * MPI_Fint (reference src/adlbf.c:6-103).  The prototypes are declared here,
 * not taken from adlb.h, as a Fortran caller has no header either.
 *
 * Rank 0 puts n units of type A (one batch with a 8-byte common prefix) and n
 * of type B; every app rank takes A or B until the servers detect exhaustion.
 * Output: rank 0 "adlb_fcall: units U sum S expect U' S'".
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void adlb_init_(int *, int *, int *, int *, int *, int *, int *, MPI_Fint *, int *);
void adlb_server_(double *, double *, int *);
void adlb_put_(void *, int *, int *, int *, int *, int *, int *);
void adlb_reserve_(int *, int *, int *, int *, int *, int *, int *);
void adlb_ireserve_(int *, int *, int *, int *, int *, int *, int *);
void adlb_get_reserved_(void *, int *, int *);
void adlb_get_reserved_timed_(void *, int *, double *, int *);
void adlb_begin_batch_put_(void *, int *, int *);
void adlb_end_batch_put_(int *);
void adlb_info_get_(int *, double *, int *);
void adlb_info_num_work_units_(int *, int *, int *, int *, int *);
void adlb_finalize_(int *);

/* status codes and the info key as a Fortran include file would spell them */
enum { OK = 1, NO_MORE_WORK = -999999999, DONE_BY_EXHAUSTION = -999999998, NO_CURRENT_WORK = -999999997 };
enum { TA = 3, TB = 8, KEY_HWM = 1, HANDLE_INTS = 5 };

int main(int argc, char **argv) {
    int n = 200;
    if (argc > 2 && !strcmp(argv[1], "-n")) n = atoi(argv[2]);
    MPI_Init(&argc, &argv);
    int rank;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    int nserv = 2, dbg = 0, apf = 0, ntypes = 2, types[2] = {TA, TB}, am_server = 0, am_debug = 0, ierr = 0;
    MPI_Fint fcomm;
    adlb_init_(&nserv, &dbg, &apf, &ntypes, types, &am_server, &am_debug, &fcomm, &ierr);
    if (ierr != OK) MPI_Abort(MPI_COMM_WORLD, 1);
    if (am_server) {
        double hi = 1e8, logt = 0.0, hwm = 0;
        int key = KEY_HWM;
        adlb_server_(&hi, &logt, &ierr);
        adlb_info_get_(&key, &hwm, &ierr);
        printf("server %d: rc %d hwm %.0f\n", rank, ierr, hwm);
        adlb_finalize_(&ierr);
        MPI_Finalize();
        return 0;
    }
    MPI_Comm app_comm = MPI_Comm_f2c(fcomm);
    long long sum = 0, expect = 0;
    int units = 0, w[4];
    if (rank == 0) {
        int len = (int)sizeof w, any = -1, me = 0, ta = TA, tb = TB, clen = 8;
        char common[8];
        memset(common, 'f', sizeof common);
        adlb_begin_batch_put_(common, &clen, &ierr);
        if (ierr != OK) MPI_Abort(MPI_COMM_WORLD, 2);
        for (int i = 0; i < n; i++) {
            int prio = i % 5;
            w[0] = i; w[1] = ~i; w[2] = TA; w[3] = 7 * i;
            adlb_put_(w, &len, &any, &me, &ta, &prio, &ierr);
            if (ierr != OK) MPI_Abort(MPI_COMM_WORLD, 2);
            expect += i * 10LL + TA;
        }
        adlb_end_batch_put_(&ierr);
        for (int i = 0; i < n; i++) {
            int prio = -(i % 3);
            w[0] = n + i; w[1] = ~(n + i); w[2] = TB; w[3] = 7 * (n + i);
            adlb_put_(w, &len, &any, &me, &tb, &prio, &ierr);
            if (ierr != OK) MPI_Abort(MPI_COMM_WORLD, 2);
            expect += (n + i) * 10LL + TB;
        }
    }
    int req[3] = {TA, TB, -1}, steps = 0;
    char buf[64];
    while (1) {
        int type, prio, handle[HANDLE_INTS], wlen, answer;
        if (++steps % 8 == 0) {
            int ta = TA, mp, nmp, nt;
            adlb_info_num_work_units_(&ta, &mp, &nmp, &nt, &ierr);
            adlb_ireserve_(req, &type, &prio, handle, &wlen, &answer, &ierr);
            if (ierr == NO_CURRENT_WORK) continue;
        } else {
            adlb_reserve_(req, &type, &prio, handle, &wlen, &answer, &ierr);
        }
        if (ierr == DONE_BY_EXHAUSTION || ierr == NO_MORE_WORK) break;
        if (ierr != OK) MPI_Abort(MPI_COMM_WORLD, 3);
        double qt = 0;
        if (steps % 2) adlb_get_reserved_(buf, handle, &ierr);
        else adlb_get_reserved_timed_(buf, handle, &qt, &ierr);
        if (ierr != OK) MPI_Abort(MPI_COMM_WORLD, 4);
        const int off = type == TA ? 8 : 0;
        if (wlen != (int)sizeof w + off || (off && buf[0] != 'f')) MPI_Abort(MPI_COMM_WORLD, 5);
        memcpy(w, buf + off, sizeof w);
        if (w[1] != ~w[0] || w[2] != type || w[3] != 7 * w[0]) MPI_Abort(MPI_COMM_WORLD, 6);
        units++;
        sum += w[0] * 10LL + type;
    }
    long long tot[2] = {units, sum}, all[2];
    MPI_Reduce(tot, all, 2, MPI_LONG_LONG, MPI_SUM, 0, app_comm);
    if (rank == 0) printf("adlb_fcall: units %lld sum %lld expect %d %lld\n", all[0], all[1], 2 * n, expect);
    adlb_finalize_(&ierr);
    MPI_Finalize();
    return 0;
}
