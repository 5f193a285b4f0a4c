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

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "adlbq.h"

namespace {

enum {
    OP_PUT = 1, OP_RESERVE = 2, OP_GET = 3, OP_UNRESERVE = 4, OP_QMROW = 5, OP_SETROW = 6, OP_CHECKREM = 7,
    OP_RFRDONE = 8, OP_TQADD = 9, OP_PUSHSEL = 10, OP_INFO = 11, OP_RQDEL = 12, OP_INFOTYPE = 13,
    OP_BYTES = 16, OP_PUTCHECK = 17, OP_HWM = 18, OP_PUSHACCEPT = 19, OP_PUSHTAKE = 20, OP_PUSHCOMMIT = 21,
    OP_PUSHDEL = 22, OP_ROUND = 23
};

int nargs(int op, int T) {
    switch (op) {
    case OP_PUT: case OP_PUSHACCEPT: return ADLBQ_PUT_INTS;
    case OP_RESERVE: return ADLBQ_RESERVE_INTS;
    case OP_GET: case OP_RFRDONE: case OP_PUTCHECK: return 2;
    case OP_UNRESERVE: case OP_TQADD: return 3;
    case OP_QMROW: case OP_CHECKREM: case OP_INFO: case OP_BYTES: case OP_HWM: case OP_ROUND: return 0;
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


// ---------------------------------------------------------------- config 5 at its SURVEY shape
// S shards' traces with steal rounds (OP_ROUND at the same place in every
// trace; oracle/gen_c5.c).  Between rounds every shard's Puts, Reserves and
// Gets go down as device-side batches on its own stream from its own host
// thread, their inputs staged in HBM beforehand and their outputs left in HBM:
// nothing waits for a batch to finish (no synchronisation per call; the
// engine's counter snapshots land in mapped memory).  A qmstat row is read
// back where the trace asks for it.  At a round every thread stops; one thread
// runs the steal group's export and settle over all shards (the merge on the
// host, the grants and rq deletions enqueued on the shards' streams) and
// collects the responses; then every thread goes on.
struct RCall {
    int op, n;
    long long in, dout, hout;  // input offset (ints), device output offset, host output offset (QMROW)
    const int *x;              // the event's arguments (single events)
};

struct RShard {
    adlbq_server *h = nullptr;
    std::vector<RCall> calls;
    std::vector<int> hin;        // reserve records (18) and get pairs (2), in call order
    std::vector<int> put;        // put records (9), in call order (host: adlbq_put_batch_device stages them)
    std::vector<int> hqm;        // QMROW outputs
    int *din = nullptr, *dout = nullptr;
    long long nout_dev = 0;
    // closed loop: every output lands in mapped host memory (hout, dout its device address) and the
    // Gets' pairs are written there at run time (hgin, dgin), from the replies that have landed
    int *hout = nullptr, *hgin = nullptr, *dgin = nullptr;
    size_t cursor = 0;           // the next call whose replies are not delivered yet
    long long waits = 0;         // Get calls that had to wait for a reply to land
    double wait_s = 0.0;
    long long mismatch = 0;      // replies whose wqseqno differs from the recorded Get's
    std::string err;
    long long ncalls = 0;
    RShard() = default;
    RShard(const RShard &) = delete;
    RShard &operator=(const RShard &) = delete;
    ~RShard() {  // every return path of adlbsrv_replay_rounds, early errors included
        if (din) (void)hipFree(din);
        if (hout) (void)hipHostFree(hout);
        else if (dout) (void)hipFree(dout);
        if (hgin) (void)hipHostFree(hgin);
    }
};

// a word of mapped host memory the device writes once (INT_MIN until then)
inline int landed(const int *p) {
    int v;
    while ((v = __atomic_load_n(p, __ATOMIC_ACQUIRE)) == INT_MIN) {
    }
    return v;
}

namespace {
int out_ints(int op, int T) {
    switch (op) {
    case OP_PUT: return 3;
    case OP_RESERVE: return ADLBQ_RESP_INTS;
    case OP_GET: return 5;
    case OP_QMROW: return 1 + T;
    default: return 0;
    }
}
}  // namespace

thread_local std::string g_rerr;
// host seconds of the last rounds replay, summed over the shards' threads:
// put, reserve, get, qmstat rows, set rows, waiting at the round barrier, the round itself
double g_rprof[8];
std::mutex g_rprof_mu;

}  // namespace

extern "C" {

const char *adlbsrv_replay_error(void) { return g_rerr.c_str(); }

// host seconds of the last adlbsrv_replay_rounds, summed over its threads: put,
// reserve, get, qmstat row, set row, round barrier (waiting + the round), the
// rounds alone (the last arriver's work), wall
void adlbsrv_replay_prof(double *out8) {
    for (int q = 0; q < 8; q++) out8[q] = g_rprof[q];
}

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


// closed: a shard issues a Get only once the reply it depends on has landed (its Reserve's
// TA_RESERVE_RESP, the Put that matched its parked Reserve, or the steal round's answer), with the
// wqseqno taken from that reply, as a live server's app does (tsp.c:157-162); the replies land in
// mapped host memory and are polled there (no stream synchronisation).  cl_stats (may be null):
// {Get calls that waited, seconds waited, replies whose wqseqno differs from the recorded Get's}.
int adlbsrv_replay_rounds2(adlbq_server **hs, int S, int ntypes, const int *const *traces, const long long *lens,
                           int k, int rqcap, int *const *outs, const long long *caps, long long *nouts,
                           int *steals, long long steal_cap, long long *nsteals, double *seconds, long long *ncalls,
                           int closed, double *cl_stats);

int adlbsrv_replay_rounds(adlbq_server **hs, int S, int ntypes, const int *const *traces, const long long *lens,
                          int k, int rqcap, int *const *outs, const long long *caps, long long *nouts,
                          int *steals, long long steal_cap, long long *nsteals, double *seconds, long long *ncalls) {
    return adlbsrv_replay_rounds2(hs, S, ntypes, traces, lens, k, rqcap, outs, caps, nouts, steals, steal_cap, nsteals,
                                  seconds, ncalls, 0, nullptr);
}

int adlbsrv_replay_rounds2(adlbq_server **hs, int S, int ntypes, const int *const *traces, const long long *lens,
                           int k, int rqcap, int *const *outs, const long long *caps, long long *nouts,
                           int *steals, long long steal_cap, long long *nsteals, double *seconds, long long *ncalls,
                           int closed, double *cl_stats) {
    if (!hs || S < 1 || !traces || !lens || !outs || !caps || !nouts || !steals || !nsteals) {
        g_rerr = "adlbsrv_replay_rounds: bad argument";
        return -1;
    }
    int A = 0;  // app ranks (closed loop: a reply slot per rank)
    const int T = ntypes;
    std::vector<RShard> sh((size_t)S);
    long long nround = -1;
    // ---- untimed: the calls, their staged inputs (HBM) and output space
    for (int j = 0; j < S; j++) {
        RShard &r = sh[(size_t)j];
        r.h = hs[j];
        const int *tr = traces[j];
        const long long n = lens[j];
        long long i = 0, rounds = 0, hq = 0;
        while (i < n) {
            const int op = tr[i], w = 1 + nargs(op, T);
            if (w <= 0 || i + w > n) {
                g_rerr = "shard " + std::to_string(j) + ": bad event at " + std::to_string(i);
                return -1;
            }
            RCall c{op, 1, 0, 0, 0, tr + i + 1};
            if (op == OP_PUT || op == OP_RESERVE || op == OP_GET) {
                long long e = i;
                while (e + w <= n && tr[e] == op) e += w;
                c.n = (int)((e - i) / w);
                std::vector<int> &dst = op == OP_PUT ? r.put : r.hin;
                c.in = (long long)dst.size();
                for (long long q = i; q < e; q += w) dst.insert(dst.end(), tr + q + 1, tr + q + w);
                c.dout = r.nout_dev;
                r.nout_dev += (long long)c.n * out_ints(op, T);
                i = e;
            } else {
                if (op != OP_QMROW && op != OP_SETROW && op != OP_ROUND) {
                    g_rerr = "shard " + std::to_string(j) + ": event " + std::to_string(op) + " is not part of the rounds replay";
                    return -1;
                }
                if (op == OP_QMROW) {
                    c.hout = hq;
                    hq += 1 + T;
                }
                rounds += op == OP_ROUND;
                i += w;
            }
            r.calls.push_back(c);
        }
        r.hqm.assign((size_t)std::max(hq, 1ll), 0);
        if (nround < 0) nround = rounds;
        if (rounds != nround) {
            g_rerr = "the traces do not hold the same number of rounds";
            return -1;
        }
        if (hipMalloc((void **)&r.din, sizeof(int) * std::max<size_t>(r.hin.size(), 1)) != hipSuccess ||
            hipMemcpy(r.din, r.hin.data(), sizeof(int) * r.hin.size(), hipMemcpyHostToDevice) != hipSuccess) {
            g_rerr = "adlbsrv_replay_rounds: device staging";
            return -1;
        }
        if (!closed) {
            if (hipMalloc((void **)&r.dout, sizeof(int) * std::max<long long>(r.nout_dev, 1)) != hipSuccess) {
                g_rerr = "adlbsrv_replay_rounds: device staging";
                return -1;
            }
        } else {
            const size_t no = (size_t)std::max<long long>(r.nout_dev, 1), ni = std::max<size_t>(r.hin.size(), 1);
            if (hipHostMalloc((void **)&r.hout, sizeof(int) * no, hipHostMallocMapped) != hipSuccess ||
                hipHostGetDevicePointer((void **)&r.dout, r.hout, 0) != hipSuccess ||
                hipHostMalloc((void **)&r.hgin, sizeof(int) * ni, hipHostMallocMapped) != hipSuccess ||
                hipHostGetDevicePointer((void **)&r.dgin, r.hgin, 0) != hipSuccess) {
                g_rerr = "adlbsrv_replay_rounds: mapped staging";
                return -1;
            }
            for (size_t q = 0; q < no; q++) r.hout[q] = INT_MIN;  // every reply word is polled until written
            for (long long q = 0; q < n;) {  // the largest rank any event names
                const int op = tr[q], w2 = 1 + nargs(op, T);
                if (op == OP_RESERVE || op == OP_GET) A = std::max(A, tr[q + 1] + 1);
                q += w2;
            }
        }
    }
    // closed loop: the reply each rank holds (its wqseqno; 0: none) per shard holding the unit, written by
    // that shard's thread (its Reserve replies and put-side matches) or by the round under its barrier
    // (a steal: the donor shard), read by the same shard's thread at the Get.  One slot per rank for all
    // shards let a shard's thread that ran ahead deliver the rank's next reply over the one another
    // shard's thread had delivered and not yet consumed (the threads meet only at rounds): that Get then
    // found no reply ("a Get whose reply never arrived")
    const int AH = std::max(A, 1);
    std::vector<std::atomic<int>> held((size_t)S * AH);
    for (auto &x : held) x.store(0, std::memory_order_relaxed);
    const int master = S > 0 ? (int)adlbq_stat(hs[0], "master") : 0;  // world rank of shard 0
    adlbq_steal_group *g = nullptr;
    if (adlbq_steal_group_create(&g, hs, S, k, rqcap)) {
        g_rerr = std::string("adlbq_steal_group_create: ") + adlbq_last_error();
        return -1;
    }
    // ---- timed: the shards' threads, meeting at every round
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    long long gen = 0;
    bool failed = false;
    long long ns = 0;
    std::string gerr;
    std::vector<int> resp;
    double round_s = 0.0;
    auto round_barrier = [&](bool ok) {  // every thread; the last one in runs the round
        std::unique_lock<std::mutex> lk(mu);
        if (!ok) failed = true;
        const long long my = gen;
        if (++arrived == S) {
            const auto r0 = std::chrono::steady_clock::now();
            if (!failed) {
                int dec = 0, set = 0, cnt = 0;
                if (adlbq_steal_group_export(g, nullptr) || adlbq_steal_group_settle(g, nullptr, 1, &dec, &set)) {
                    gerr = std::string("steal round: ") + adlbq_last_error();
                    failed = true;
                } else {
                    resp.resize((size_t)15 * (set + 16));
                    if (adlbq_steal_group_responses(g, set + 16, resp.data(), &cnt)) {
                        gerr = std::string("steal round responses: ") + adlbq_last_error();
                        failed = true;
                    } else {
                        for (int q = 0; q < cnt && ns < steal_cap; q++, ns++) {
                            std::memcpy(steals + 15 * ns, resp.data() + 15 * q, sizeof(int) * 15);
                            const int *row = resp.data() + 15 * q;  // {shard, rqseqno, rank, resp[12]}
                            const int donor = row[3 + 6] - master;  // the shard that holds the granted unit
                            if (closed && row[3] == 1 && row[2] >= 0 && row[2] < A && donor >= 0 && donor < S)
                                held[(size_t)donor * AH + row[2]].store(row[3 + 5], std::memory_order_relaxed);
                        }
                        if (cnt && ns >= steal_cap) {
                            gerr = "steal output full";
                            failed = true;
                        }
                    }
                }
            }
            round_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - r0).count();
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != my; });
        }
        return !failed;
    };
    for (double &v : g_rprof) v = 0.0;
    auto work = [&](int j) {
        RShard &r = sh[(size_t)j];
        adlbq_server *h = r.h;
        std::atomic<int> *const held_j = held.data() + (size_t)j * AH;  // the replies for units this shard holds
        bool ok = true;
        double prof[8] = {0};
        using clk = std::chrono::steady_clock;
        for (const RCall &c : r.calls) {
            if (!ok) {
                if (c.op == OP_ROUND) round_barrier(false);
                continue;
            }
            r.ncalls++;
            int rc = 0;
            const auto c0 = clk::now();
            const int slot = c.op == OP_PUT ? 0 : c.op == OP_RESERVE ? 1 : c.op == OP_GET ? 2 : c.op == OP_QMROW ? 3
                             : c.op == OP_SETROW ? 4 : 5;
            const int *gin = r.din + c.in;
            if (closed && c.op == OP_GET) {
                // every Get's reply: deliver the replies of earlier calls in order until it is held
                const size_t ci = (size_t)(&c - r.calls.data());
                bool waited = false;
                const auto w0 = clk::now();
                for (int e = 0; e < c.n && ok; e++) {
                    const int rank = c.x[3 * e], want = c.x[3 * e + 1];  // the recorded {op, rank, wqseqno}
                    while (held_j[rank].load(std::memory_order_relaxed) == 0 && r.cursor < ci) {
                        const RCall &d = r.calls[r.cursor++];
                        if (d.op == OP_RESERVE) {
                            for (int q = 0; q < d.n; q++) {
                                const int *o = r.hout + d.dout + (long long)q * ADLBQ_RESP_INTS;
                                if (__atomic_load_n(o, __ATOMIC_ACQUIRE) == INT_MIN) waited = true;
                                if (landed(o) == 1)  // TA_RESERVE_RESP success: the rank holds [5]
                                    held_j[r.hin[(size_t)(d.in + (long long)q * ADLBQ_RESERVE_INTS)]].store(
                                        landed(o + 5), std::memory_order_relaxed);
                            }
                        } else if (d.op == OP_PUT) {
                            for (int q = 0; q < d.n; q++) {
                                const int *o = r.hout + d.dout + 3ll * q;
                                if (__atomic_load_n(o + 1, __ATOMIC_ACQUIRE) == INT_MIN) waited = true;
                                const int mr = landed(o + 1);  // a parked Reserve matched: its rank holds [0]
                                if (mr >= 0 && mr < A) held_j[mr].store(landed(o), std::memory_order_relaxed);
                            }
                        }
                    }
                    const int got = held_j[rank].exchange(0, std::memory_order_relaxed);
                    if (got == 0) {
                        r.err = "closed loop: a Get whose reply never arrived (rank " + std::to_string(rank) + ")";
                        ok = false;
                        break;
                    }
                    r.mismatch += got != want;
                    r.hgin[(size_t)(c.in + 2ll * e)] = rank;
                    r.hgin[(size_t)(c.in + 2ll * e + 1)] = got;
                }
                if (!ok) continue;
                if (waited) {
                    r.waits++;
                    r.wait_s += std::chrono::duration<double>(clk::now() - w0).count();
                }
                gin = r.dgin + c.in;
            }
            switch (c.op) {
            case OP_PUT: rc = adlbq_put_batch_device(h, c.n, r.put.data() + c.in, r.dout + c.dout); break;
            case OP_RESERVE: rc = adlbq_reserve_batch_device(h, c.n, r.din + c.in, r.dout + c.dout); break;
            case OP_GET: rc = adlbq_get_reserved_batch_device(h, c.n, gin, r.dout + c.dout); break;
            case OP_QMROW: rc = adlbq_qmstat_row(h, &r.hqm[(size_t)c.hout], &r.hqm[(size_t)c.hout + 1]); break;
            case OP_SETROW: rc = adlbq_set_qmstat_row(h, c.x[0], c.x[1], (double)c.x[2], c.x + 3); break;
            case OP_ROUND: ok = round_barrier(true); break;
            }
            prof[slot] += std::chrono::duration<double>(clk::now() - c0).count();
            if (c.op == OP_ROUND) continue;
            if (rc) {
                r.err = std::string("call ") + std::to_string(c.op) + ": " + adlbq_last_error();
                ok = false;
            }
        }
        std::lock_guard<std::mutex> lk(g_rprof_mu);
        for (int q = 0; q < 6; q++) g_rprof[q] += prof[q];
    };
    const auto t0 = std::chrono::steady_clock::now();
    {
        std::vector<std::thread> th;
        for (int j = 0; j < S; j++) th.emplace_back(work, j);
        for (auto &t : th) t.join();
    }
    // every shard's device work has finished (the engine's batches run on its streams)
    for (int j = 0; j < S; j++) {
        double c0, c1;
        if (adlbq_bytes(hs[j], &c0, &c1)) failed = true;  // synchronises the shard's stream
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
    g_rprof[6] = round_s;
    g_rprof[7] = std::chrono::duration<double>(t1 - t0).count();
    *nsteals = ns;
    adlbq_steal_group_destroy(g);
    // ---- untimed: outputs back, in the replay layout
    int rc = 0;
    for (int j = 0; j < S && !rc; j++) {
        RShard &r = sh[(size_t)j];
        if (ncalls) ncalls[j] = r.ncalls;
        if (!r.err.empty()) {
            g_rerr = "shard " + std::to_string(j) + ": " + r.err;
            rc = -1;
            break;
        }
        std::vector<int> dv((size_t)std::max<long long>(r.nout_dev, 1));
        if (r.hout) {
            std::memcpy(dv.data(), r.hout, sizeof(int) * r.nout_dev);
        } else if (hipMemcpy(dv.data(), r.dout, sizeof(int) * r.nout_dev, hipMemcpyDeviceToHost) != hipSuccess) {
            g_rerr = "output copy";
            rc = -1;
            break;
        }
        Out o{outs[j], caps[j]};
        for (const RCall &c : r.calls) {
            const int oi = out_ints(c.op, T);
            if (c.op == OP_PUT || c.op == OP_RESERVE || c.op == OP_GET) {
                for (int e = 0; e < c.n; e++) {
                    o.put(oi);
                    for (int q = 0; q < oi; q++) o.put(dv[(size_t)(c.dout + (long long)e * oi + q)]);
                }
            } else if (c.op == OP_QMROW) {
                o.put(oi);
                for (int q = 0; q < oi; q++) o.put(r.hqm[(size_t)c.hout + q]);
            } else {
                o.put(0);
            }
        }
        nouts[j] = o.n;
        if (o.over) {
            g_rerr = "shard " + std::to_string(j) + ": output buffer too small";
            rc = -2;
        }
    }
    if (cl_stats) {
        cl_stats[0] = cl_stats[1] = cl_stats[2] = 0.0;
        for (const auto &r : sh) {
            cl_stats[0] += (double)r.waits;
            cl_stats[1] += r.wait_s;
            cl_stats[2] += (double)r.mismatch;
        }
    }
    if (!rc && (failed || !gerr.empty())) {
        g_rerr = gerr.empty() ? "a shard failed" : gerr;
        rc = -1;
    }
    return rc;
}

}  // extern "C"
