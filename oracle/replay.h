/*
 * oracle/replay.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Event-trace replay of one ADLB server's queue handlers.  A trace is a flat
 * int32 stream of events; each event starts with an opcode followed by a fixed
 * number of arguments.  Replaying writes, per event, [n, v1 .. vn] to the output
 * stream.  The same trace/output format is produced by the product's C ABI
 * replayer (adlb_amd/replay.py), so parity is a byte comparison.
 *
 * Event semantics restate the reference server loop (src/adlb.c) handler by
 * handler; see replay.c for the line citations.
 */
#ifndef ADLBQ_ORACLE_REPLAY_H
#define ADLBQ_ORACLE_REPLAY_H

enum {
    ORC_OP_PUT = 1,       /* type prio answer target len home clen csrv cseq   -> [wqseqno, matched_rank, matched_rqseqno] */
    ORC_OP_RESERVE = 2,   /* rank hang t0..t15                                  -> resp[12] */
    ORC_OP_GET = 3,       /* rank wqseqno                                       -> [rc, len, type, prio, answer] */
    ORC_OP_UNRESERVE = 4, /* rank wqseqno new_pin_rank                          -> [found] */
    ORC_OP_QMROW = 5,     /*                                                    -> [qlen_unpin_untarg, hi_prio[T]] */
    ORC_OP_SETROW = 6,    /* server_idx qlen nbytes hi_prio[T]                  -> [] */
    ORC_OP_CHECKREM = 7,  /*                                                    -> [k, (rqseqno, rank, cand) * k] */
    ORC_OP_RFRDONE = 8,   /* from_server_rank for_rank                          -> [] */
    ORC_OP_TQADD = 9,     /* app_rank type server_rank                          -> like CHECKREM */
    ORC_OP_PUSHSEL = 10,  /* threshold                                          -> [cand_server_rank, wqseqno] */
    ORC_OP_INFO = 11,     /*                                                    -> [wq_count, wq_max_count, rq_count] */
    ORC_OP_RQDEL = 12,    /* rqseqno                                            -> [found] */
    ORC_OP_INFOTYPE = 13, /* type                                               -> [max_prio, num_max_prio, num_type] */
    ORC_OP_RFR = 14,      /* rqseqno for_rank t0..t15 (SS_RFR rfr_buf)          -> SS_RFR_RESP [12] or [-2, rqseqno, for_rank] */
    ORC_OP_RQLIST = 15,   /*                                                    -> [k, (rqseqno, rank, t0..t15) * k] */
    ORC_OP_BYTES = 16,    /*                                                    -> [curr] bytes the queues hold beyond init (adlb.c:3419-3474) */
    ORC_OP_PUTCHECK = 17, /* work_len max_malloc                               -> [rejected, hint_server_rank] (adlb.c:908-931) */
    ORC_OP_HWM = 18,      /*                                                    -> [hwm] their high-water mark beyond init (-1: backend cannot tell) */
    /* memory-pressure push (adlb.c:2109-2362) */
    ORC_OP_PUSHACCEPT = 19, /* type prio answer target len home clen csrv cseq  -> [wqseqno] SS_PUSH_QUERY at the pushee (2146-2160) */
    ORC_OP_PUSHTAKE = 20,   /* wqseqno                                          -> [ok, type, prio, len, answer, target, home, clen, csrv, cseq] SS_PUSH_QUERY_RESP at the pusher (2179-2222) */
    ORC_OP_PUSHCOMMIT = 21, /* wqseqno                                          -> [found, matched_rank, matched_rqseqno] SS_PUSH_HDR at the pushee (2232-2340) */
    ORC_OP_PUSHDEL = 22,    /* wqseqno                                          -> [found] SS_PUSH_DEL at the pushee (2353-2360) */
    /* a steal round of the server group starts here (oracle/gen_c5.c): every outstanding RFR record
     * is cleared, as the SS_RFR_RESPs the round replaces would (adlb.c:1877-1878) -> [] */
    ORC_OP_ROUND = 23,
};

/* TA_RESERVE_RESP layout (adlb.c:1213-1222), plus two slots this build uses
 * for the parked case: [10] = rqseqno of the parked request, [11] = server
 * rank an SS_RFR was sent to (-1 if none). resp[0]: 1 = SUCCESS,
 * -2 = NO_CURR_WORK, 0 = parked on rq (no reply sent yet). */
#define ORC_RESP_INTS 12

int  orc_init(int ntypes, const int *user_types, int num_app_ranks, int num_servers,
              int my_server_idx);
long orc_replay(const int *trace, long ntrace, int *out, long outcap);
int  orc_event_nargs(int op, int ntypes);

#endif
