// adlb_fortran.cpp -- Fortran-callable entry points of libadlb.so.
//
// Fortran passes every argument by reference and returns the status through a
// trailing INTEGER ierr; names are the lower-case C names plus one trailing
// underscore (the gfortran / flang / ifort default on Linux, which is what the
// reference's FortranCInterface-generated ADLB_FC_GLOBAL macro resolves to
// there -- src/adlbf.c:1-103, src/CMakeLists.txt).  The communicator comes
// back as an MPI_Fint handle (MPI_Comm_c2f), as in src/adlbf.c:9-13.
//
// Each shim forwards to the C API in include/adlb/adlb.h; nothing here keeps
// state of its own.
#include <mpi.h>

#include <adlb/adlb.h>

extern "C" {

void adlb_init_(int *num_servers, int *use_debug_server, int *aprintf_flag, int *ntypes,
                int *type_vect, int *am_server, int *am_debug_server, MPI_Fint *app_comm,
                int *ierr) {
    MPI_Comm c = MPI_COMM_NULL;
    *ierr = ADLB_Init(*num_servers, *use_debug_server, *aprintf_flag, *ntypes, type_vect,
                      am_server, am_debug_server, &c);
    *app_comm = MPI_Comm_c2f(c);
}

void adlb_server_(double *hi_malloc, double *periodic_log_interval, int *ierr) {
    *ierr = ADLB_Server(*hi_malloc, *periodic_log_interval);
}

void adlb_debug_server_(double *timeout, int *ierr) { *ierr = ADLB_Debug_server(*timeout); }

void adlb_put_(void *work_buf, int *work_len, int *reserve_rank, int *answer_rank,
               int *work_type, int *work_prio, int *ierr) {
    *ierr = ADLB_Put(work_buf, *work_len, *reserve_rank, *answer_rank, *work_type, *work_prio);
}

void adlb_reserve_(int *req_types, int *work_type, int *work_prio, int *work_handle,
                   int *work_len, int *answer_rank, int *ierr) {
    *ierr = ADLB_Reserve(req_types, work_type, work_prio, work_handle, work_len, answer_rank);
}

void adlb_ireserve_(int *req_types, int *work_type, int *work_prio, int *work_handle,
                    int *work_len, int *answer_rank, int *ierr) {
    *ierr = ADLB_Ireserve(req_types, work_type, work_prio, work_handle, work_len, answer_rank);
}

void adlb_get_reserved_(void *work_buf, int *work_handle, int *ierr) {
    *ierr = ADLB_Get_reserved(work_buf, work_handle);
}

void adlb_get_reserved_timed_(void *work_buf, int *work_handle, double *qtime, int *ierr) {
    *ierr = ADLB_Get_reserved_timed(work_buf, work_handle, qtime);
}

void adlb_begin_batch_put_(void *common_buf, int *len_common, int *ierr) {
    *ierr = ADLB_Begin_batch_put(common_buf, *len_common);
}

void adlb_end_batch_put_(int *ierr) { *ierr = ADLB_End_batch_put(); }

void adlb_begin_batch_put_2_(void *common_buf, int *len_common, int *ierr) {
    *ierr = ADLB_Begin_batch_put_2(common_buf, *len_common);
}

void adlb_end_batch_put_2_(int *ierr) { *ierr = ADLB_End_batch_put_2(); }

void adlb_set_problem_done_(int *ierr) { *ierr = ADLB_Set_problem_done(); }

void adlb_set_no_more_work_(int *ierr) { *ierr = ADLB_Set_no_more_work(); }

void adlb_info_get_(int *key, double *val, int *ierr) { *ierr = ADLB_Info_get(*key, val); }

void adlb_info_num_work_units_(int *work_type, int *max_prio, int *num_max_prio_type,
                               int *num_type, int *ierr) {
    *ierr = ADLB_Info_num_work_units(*work_type, max_prio, num_max_prio_type, num_type);
}

void adlb_finalize_(int *ierr) { *ierr = ADLB_Finalize(); }

void adlb_abort_(int *code, int *ierr) { *ierr = ADLB_Abort(*code); }

}  // extern "C"
