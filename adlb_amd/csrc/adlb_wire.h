/* adlb_wire.h -- the message protocol between ADLB apps and servers.
 *
 * Tag values and buffer layouts are the reference's wire (src/adlb.c:44-91),
 * so an event log recorded from the reference server (oracle/mpilog.c) maps
 * one to one onto this server's handlers (tests/test_gpu_server.py).  The
 * server-to-server control messages that the reference passes around a ring
 * (qmstat, no-more-work, end, exhaustion) are replaced by direct messages
 * (SRV_* tags below): one process per server, every server one hop away.
 */
#ifndef ADLB_WIRE_H
#define ADLB_WIRE_H

enum {
    /* app <-> server (adlb.c:44-83) */
    TAG_PUT_HDR = 1001,           /* int[12] {type, prio, answer, target, len, home, batch, common x3} */
    TAG_PUT_MSG = 1002,           /* payload bytes */
    TAG_PUT_COMMON_HDR = 1003,    /* int[12] {common_len} */
    TAG_PUT_COMMON_MSG = 1004,    /* common bytes */
    TAG_PUT_BATCH_DONE = 1005,    /* int[12] {cqseqno, refcnt} */
    TAG_DID_PUT_AT_REMOTE = 1006, /* int[12] {type, target, server} */
    TAG_RESERVE = 1007,           /* int[17] {hang, req_types[16]} */
    TAG_RESERVE_RESP = 1008,      /* int[12] {rc, type, prio, len, answer, wqseqno, server, common x3} */
    TAG_GET_RESERVED = 1009,      /* int[12] {wqseqno} */
    TAG_GET_RESERVED_RESP = 1010, /* payload bytes */
    TAG_NO_MORE_WORK = 1011,      /* empty */
    TAG_LOCAL_APP_DONE = 1012,    /* empty */
    TAG_SS_NO_MORE_WORK = 1014,
    TAG_SS_QMSTAT = 1015,
    TAG_SS_RFR = 1018,            /* int[28] {rqseqno, for_rank, req_types[16]} */
    TAG_SS_RFR_RESP = 1019,       /* int[28] {rc, rqseqno, for_rank, type, prio, len, answer, wqseqno,
                                     prev_target, common x3} or {-2, rqseqno, for_rank, req_types[16]} */
    TAG_ACK_AND_RC = 1020,        /* int[12] or double[12] */
    TAG_SS_PUSH_QUERY = 1021,     /* double[12] {type, prio, len, answer, time, target, home, wqseqno, common x3} */
    TAG_SS_PUSH_QUERY_RESP = 1022, /* double[12] {to_rank or -1, nbytes_used, wqseqno on pusher, on pushee} */
    TAG_SS_PUSH_HDR = 1023,       /* int[12] {wqseqno on pushee} */
    TAG_SS_PUSH_WORK = 1024,      /* payload bytes */
    TAG_SS_PUSH_DEL = 1025,       /* int[12] {wqseqno on pushee} */
    TAG_SS_UNRESERVE = 1028,      /* int[12] {for_rank, wqseqno, new_pin} */
    TAG_SS_MOVING_TARGETED_WORK = 1029, /* int[12] {target, type, from server, to server} */
    TAG_FA_ABORT = 1027,
    TAG_DS_END = 1032,
    TAG_INFO_NUM_WORK_UNITS = 1037, /* int[12] {type} -> int[12] {max_prio, n_at_max, n, nmw} */
    TAG_GET_COMMON = 1038,        /* int[12] {cqseqno} */
    TAG_GET_COMMON_RESP = 1039,   /* common bytes */

    /* server <-> server control of this implementation */
    TAG_SRV_QMSTAT = 1101,        /* int {server_idx, qlen, hi[T]} + double nbytes (packed as bytes) */
    TAG_SRV_EXH_QUERY = 1102,     /* int[2] {epoch} master -> all */
    TAG_SRV_EXH_REPLY = 1103,     /* long long[3] {epoch, idle, activity} */
    TAG_SRV_EXHAUSTED = 1104,     /* empty: master -> all */
    TAG_SRV_DONE = 1105,          /* empty: every local app finalized -> master */
    TAG_SRV_END = 1106,           /* empty: master -> all */
    TAG_SRV_ABORT = 1107,         /* int[12] {code} */
    TAG_SRV_STEAL = 1108,         /* empty: master -> all, open a steal-group round */
    TAG_SRV_STEAL_WANT = 1109     /* empty: any -> master, a parked Reserve has a donor by the qmstat table */
};

#define WIRE_IBUF 12   /* IBUF_NUMINTS / IBUF_NUMDBLS, adlb.c:89-90 */
#define WIRE_REQ 16    /* REQ_TYPE_VECT_SZ, xq.h:37 */
#define WIRE_RFR 28    /* RFRBUF_NUMINTS, adlb.c:91 */

#define WIRE_SUCCESS 1
#define WIRE_ERROR (-1)
#define WIRE_NO_CURR_WORK (-2) /* adlb.c:87; the client maps it to ADLB_NO_CURRENT_WORK */
/* the public return codes carried on the wire (include/adlb/adlb.h) */
#define WIRE_NO_MORE_WORK (-999999999)
#define WIRE_DONE_BY_EXHAUSTION (-999999998)
#define WIRE_PUT_REJECTED (-999999996)

#endif
