/*
 * adlb/adlb.h -- the ADLB application API served by libadlb.so.
 *
 * Source-compatible with the reference's public header
 * (include/adlb/adlb.h:42-88 of kc9jud/adlb): the same entry points, return
 * codes and constants, so an ADLB application builds unchanged against this
 * header and links against adlb_amd/libadlb.so instead of the reference's
 * libadlb.a.  The server side of every call runs the GPU work-queue engine
 * (include/adlbq.h) on the server ranks' MI355X devices.
 *
 * Rank layout (as ADLB_Init's callers expect): application ranks
 * [0, A), server ranks [A, A+nservers), then the debug server if requested;
 * app rank r is served by server A + r % nservers.
 */
#ifndef ADLB_ADLB_H_INCLUDED
#define ADLB_ADLB_H_INCLUDED

#include <mpi.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ADLB_VERSION_NUMBER      463

/* return codes */
#define ADLB_SUCCESS                     (1)
#define ADLB_ERROR                      (-1)
#define ADLB_NO_MORE_WORK       (-999999999)
#define ADLB_DONE_BY_EXHAUSTION (-999999998)
#define ADLB_NO_CURRENT_WORK    (-999999997)
#define ADLB_PUT_REJECTED       (-999999996)
#define ADLB_LOWEST_PRIO        (-999999999)

/* ADLB_Info_get keys */
#define ADLB_INFO_MALLOC_HWM               1
#define ADLB_INFO_AVG_TIME_ON_RQ           2
#define ADLB_INFO_NPUSHED_FROM_HERE        3
#define ADLB_INFO_NPUSHED_TO_HERE          4
#define ADLB_INFO_NREJECTED_PUTS           5
#define ADLB_INFO_LOOP_TOP_TIME            6
#define ADLB_INFO_MAX_QMSTAT_TRIP_TIME     7
#define ADLB_INFO_AVG_QMSTAT_TRIP_TIME     8
#define ADLB_INFO_NUM_QMS_EXCEED_INT       9
#define ADLB_INFO_NUM_RESERVES            10
#define ADLB_INFO_NUM_RESERVES_PUT_ON_RQ  11
#define ADLB_INFO_MAX_WQ_COUNT            12

/* Reserve request vectors: up to 16 types, -1 first = any type, -1 later = end */
#define ADLB_RESERVE_REQUEST_ANY    -1
#define ADLB_RESERVE_EOL            -1
#define ADLB_HANDLE_SIZE             5

/* setup / roles */
int ADLB_Init(int num_servers, int use_debug_server, int aprintf_flag, int num_types, int *types,
              int *am_server, int *am_debug_server, MPI_Comm *app_comm);
int ADLB_Server(double hi_malloc, double periodic_logging_time);
int ADLB_Debug_server(double timeout);
int ADLB_Finalize(void);
int ADLB_Abort(int code);

/* work */
int ADLB_Put(void *work_buf, int work_len, int target_rank, int answer_rank, int work_type, int work_prio);
int ADLB_Reserve(int *req_types, int *work_type, int *work_prio, int *work_handle, int *work_len,
                 int *answer_rank);
int ADLB_Ireserve(int *req_types, int *work_type, int *work_prio, int *work_handle, int *work_len,
                  int *answer_rank);
int ADLB_Get_reserved(void *work_buf, int *work_handle);
int ADLB_Get_reserved_timed(void *work_buf, int *work_handle, double *queued_time);
int ADLB_Begin_batch_put(void *common_buf, int len_common);
int ADLB_End_batch_put(void);
int ADLB_Begin_batch_put_2(void *common_buf, int len_common);
int ADLB_End_batch_put_2(void);
int ADLB_Set_problem_done(void);
int ADLB_Set_no_more_work(void); /* deprecated name of ADLB_Set_problem_done */

/* queries */
int ADLB_Info_get(int key, double *val);
int ADLB_Info_num_work_units(int work_type, int *max_prio, int *num_max_prio_type, int *num_type);

/* the un-profiled layer (every ADLB_X calls ADLBP_X) */
int ADLBP_Init(int, int, int, int, int *, int *, int *, MPI_Comm *);
int ADLBP_Server(double hi_malloc, double periodic_logging_time);
int ADLBP_Debug_server(double timeout);
int ADLBP_Put(void *, int, int, int, int, int);
int ADLBP_Reserve(int *, int *, int *, int *, int *, int *);
int ADLBP_Ireserve(int *, int *, int *, int *, int *, int *);
int ADLBP_Get_reserved(void *, int *);
int ADLBP_Get_reserved_timed(void *, int *, double *);
int ADLBP_Begin_batch_put(void *, int);
int ADLBP_End_batch_put(void);
int ADLBP_Set_problem_done(void);
int ADLBP_Set_no_more_work(void);
int ADLBP_Info_get(int, double *);
int ADLBP_Info_num_work_units(int, int *, int *, int *);
int ADLBP_Finalize(void);
int ADLBP_Abort(int);

/* helpers the reference's examples call directly */
void adlbp_dbgprintf(int flag, int linenum, char *fmt, ...);

#ifdef __cplusplus
}
#endif

#endif
