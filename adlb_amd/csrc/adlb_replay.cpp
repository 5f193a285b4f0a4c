// adlb_replay.cpp -- a native server-loop driver for recorded event streams.
//
// An event trace (the oracle's format, oracle/replay.h; adlb_amd/replay.py is
// the Python twin) is what one ADLB server's queue sees: Puts, Reserves, Gets,
// unreserves, qmstat rows, check_remote, tq, RFR completions, push steps,
// info queries.  This driver issues it through the engine ABI the way the
// server loop does (adlb_core.cpp): a run of consecutive Puts, Reserves or
// Gets as one batch call (the ABI guarantees the sequential result), every
// other event one call.  The output stream has replay.py's layout, so it is
// compared with the oracle's byte for byte.
//
// adlbsrv_replay_many runs several shards' traces at once, one host thread
// per shard (each handle on its own HIP stream): the config-5 leg of bench.py,
// where 8 server shards of one GPU each replay their own stream.
#include "adlb_core.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "adlbq.h"

namespace {

enum {
    OP_PUT = 1, OP_RESERVE = 2, OP_GET = 3, OP_UNRESERVE = 4, OP_QMROW = 5, OP_SETROW = 6, OP_CHECKREM = 7,
    OP_RFRDONE = 8, OP_TQADD = 9, OP_PUSHSEL = 10, OP_INFO = 11, OP_RQDEL = 12, OP_INFOTYPE = 13,
    OP_BYTES = 16, OP_PUTCHECK = 17, OP_HWM = 18, OP_PUSHACCEPT = 19, OP_PUSHTAKE = 20, OP_PUSHCOMMIT = 21,
    OP_PUSHDEL = 22
};

int nargs(int op, int T) {
    switch (op) {
    case OP_PUT: case OP_PUSHACCEPT: return ADLBQ_PUT_INTS;
    case OP_RESERVE: return ADLBQ_RESERVE_INTS;
    case OP_GET: case OP_RFRDONE: case OP_PUTCHECK: return 2;
    case OP_UNRESERVE: case OP_TQADD: return 3;
    case OP_QMROW: case OP_CHECKREM: case OP_INFO: case OP_BYTES: case OP_HWM: return 0;
    case OP_SETROW: return 3 + T;
    case OP_PUSHSEL: case OP_RQDEL: case OP_INFOTYPE: case OP_PUSHTAKE: case OP_PUSHCOMMIT: case OP_PUSHDEL: return 1;
    default: return -1;
    }
}

struct Out {
    int *p;
    long long cap, n = 0;
    bool over = false;
    void put(int v) {
        if (n < cap) p[n] = v;
        else over = true;
        n++;
    }
    void row(std::initializer_list<int> v) {
        put((int)v.size());
        for (int x : v) put(x);
    }
};

struct Replayer {
    adlbq_server *h;
    int T = 0;
    std::string err;
    std::vector<int> buf, res, crem;
    long long calls = 0;

    int fail(const char *what) {
        err = std::string(what) + ": " + adlbq_last_error();
        return -1;
    }
    int checkrem(Out &o) {
        const int cap = 1 << 16;
        crem.resize(3 * (size_t)cap);
        int k = 0;
        if (adlbq_check_remote(h, cap, crem.data(), &k)) return fail("adlbq_check_remote");
        o.put(1 + 3 * k);
        o.put(k);
        for (int i = 0; i < 3 * k; i++) o.put(crem[(size_t)i]);
        return 0;
    }

    int run(const int *tr, long long n, Out &o) {
        long long i = 0;
        while (i < n) {
            const int op = tr[i];
            const int w = 1 + nargs(op, T);
            if (w <= 0) {
                err = "unknown opcode " + std::to_string(op);
                return -1;
            }
            if (i + w > n) {
                err = "trace ends inside an event";
                return -1;
            }
            calls++;
            if (op == OP_PUT || op == OP_RESERVE || op == OP_GET) {
                long long j = i;
                while (j + w <= n && tr[j] == op) j += w;
                const int m = (int)((j - i) / w), a = w - 1;
                buf.resize((size_t)m * a);
                for (int r = 0; r < m; r++) std::memcpy(&buf[(size_t)r * a], tr + i + (long long)r * w + 1, sizeof(int) * a);
                const int ro = op == OP_PUT ? 3 : op == OP_RESERVE ? ADLBQ_RESP_INTS : 5;
                res.resize((size_t)m * ro);
                int rc = op == OP_PUT ? adlbq_put_batch(h, m, buf.data(), res.data())
                         : op == OP_RESERVE ? adlbq_reserve_batch(h, m, buf.data(), res.data())
                                            : adlbq_get_reserved_batch(h, m, buf.data(), res.data());
                if (rc) return fail("batch call");
                for (int r = 0; r < m; r++) {
                    o.put(ro);
                    for (int c = 0; c < ro; c++) o.put(res[(size_t)r * ro + c]);
                }
                i = j;
                continue;
            }
            const int *x = tr + i + 1;
            i += w;
            switch (op) {
            case OP_UNRESERVE: {
                int f = 0;
                if (adlbq_unreserve(h, x[0], x[1], x[2], &f)) return fail("adlbq_unreserve");
                o.row({f});
                break;
            }
            case OP_QMROW: {
                int q = 0;
                std::vector<int> hi((size_t)std::max(T, 1));
                if (adlbq_qmstat_row(h, &q, hi.data())) return fail("adlbq_qmstat_row");
                o.put(1 + T);
                o.put(q);
                for (int t = 0; t < T; t++) o.put(hi[(size_t)t]);
                break;
            }
            case OP_SETROW:
                if (adlbq_set_qmstat_row(h, x[0], x[1], (double)x[2], x + 3)) return fail("adlbq_set_qmstat_row");
                o.put(0);
                break;
            case OP_CHECKREM:
                if (checkrem(o)) return -1;
                break;
            case OP_RFRDONE:
                if (adlbq_rfr_done(h, x[0], x[1])) return fail("adlbq_rfr_done");
                o.put(0);
                break;
            case OP_TQADD:  // FA_DID_PUT_AT_REMOTE: tq_add, then check_remote (adlb.c:1167-1179)
                if (adlbq_tq_add(h, x[0], x[1], x[2])) return fail("adlbq_tq_add");
                if (checkrem(o)) return -1;
                break;
            case OP_PUSHSEL: {
                int c = -1, s = -1;
                if (adlbq_push_select(h, (double)x[0], &c, &s)) return fail("adlbq_push_select");
                o.row({c, s});
                break;
            }
            case OP_INFO: {
                int a = 0, b = 0, c = 0;
                if (adlbq_info(h, &a, &b, &c)) return fail("adlbq_info");
                o.row({a, b, c});
                break;
            }
            case OP_RQDEL: {
                int f = 0;
                if (adlbq_rq_delete(h, x[0], &f)) return fail("adlbq_rq_delete");
                o.row({f});
                break;
            }
            case OP_INFOTYPE: {
                int a = 0, b = 0, c = 0;
                if (adlbq_info_type(h, x[0], &a, &b, &c)) return fail("adlbq_info_type");
                o.row({a, b, c});
                break;
            }
            case OP_BYTES: case OP_HWM: {
                double c = 0, hw = 0;
                if (adlbq_bytes(h, &c, &hw)) return fail("adlbq_bytes");
                o.row({(int)(long long)(op == OP_BYTES ? c : hw)});
                break;
            }
            case OP_PUTCHECK: {
                int rej = 0, hint = -1;
                if (adlbq_put_check(h, x[0], (double)x[1], &rej, &hint)) return fail("adlbq_put_check");
                o.row({rej, hint});
                break;
            }
            case OP_PUSHACCEPT: {
                int s = -1;
                if (adlbq_push_accept(h, x, &s)) return fail("adlbq_push_accept");
                o.row({s});
                break;
            }
            case OP_PUSHTAKE: {
                int r[10] = {0};
                if (adlbq_push_take(h, x[0], r)) return fail("adlbq_push_take");
                o.put(10);
                for (int v : r) o.put(v);
                break;
            }
            case OP_PUSHCOMMIT: {
                int r[3] = {0};
                if (adlbq_push_commit(h, x[0], r)) return fail("adlbq_push_commit");
                o.row({r[0], r[1], r[2]});
                break;
            }
            case OP_PUSHDEL: {
                int f = 0;
                if (adlbq_push_discard(h, x[0], &f)) return fail("adlbq_push_discard");
                o.row({f});
                break;
            }
            }
        }
        return 0;
    }
};

thread_local std::string g_rerr;

}  // namespace

extern "C" {

const char *adlbsrv_replay_error(void) { return g_rerr.c_str(); }

int adlbsrv_replay_many(adlbq_server **hs, int n, int ntypes, const int *const *traces, const long long *lens,
                        int *const *outs, const long long *caps, long long *nouts, long long *ncalls) {
    if (!hs || n < 1 || !traces || !lens || !outs || !caps || !nouts) {
        g_rerr = "adlbsrv_replay_many: bad argument";
        return -1;
    }
    std::vector<Replayer> rp((size_t)n);
    std::vector<Out> os;
    os.reserve((size_t)n);
    std::vector<int> rcs((size_t)n, 0);
    for (int j = 0; j < n; j++) {
        rp[(size_t)j].h = hs[j];
        rp[(size_t)j].T = ntypes;
        os.push_back(Out{outs[j], caps[j]});
    }
    auto work = [&](int j) { rcs[(size_t)j] = rp[(size_t)j].run(traces[j], lens[j], os[(size_t)j]); };
    if (n == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int j = 0; j < n; j++) th.emplace_back(work, j);
        for (auto &t : th) t.join();
    }
    for (int j = 0; j < n; j++) {
        nouts[j] = os[(size_t)j].n;
        if (ncalls) ncalls[j] = rp[(size_t)j].calls;
        if (rcs[(size_t)j]) {
            g_rerr = "shard " + std::to_string(j) + ": " + rp[(size_t)j].err;
            return -1;
        }
        if (os[(size_t)j].over) {
            g_rerr = "shard " + std::to_string(j) + ": output buffer too small";
            return -2;
        }
    }
    return 0;
}

}  // extern "C"
